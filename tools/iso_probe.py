"""Tail probe of the headline workload (1024 x N=100 nx=12 nu=4, k_max 50): the kk histogram of one batch, the
isolated-batch time through each entry point (ipm_batch, its profiled form, a queue of one batch at several drain
thresholds), and the K-step queue time at each drain threshold.
    python3 tools/iso_probe.py [K ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    Ks = [int(x) for x in sys.argv[1:]] or [20]
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    Q = s.queue(1024, 1024)
    Q.run()
    torch.cuda.synchronize()
    kk = Q.kk.cpu().numpy()
    ret = Q.ret.cpu().numpy()
    h = np.bincount(kk, minlength=51)
    print("kk histogram (kk:count):", {int(i): int(c) for i, c in enumerate(h) if c}, "ret!=0:", int((ret != 0).sum()),
          "sum kk", int(kk.sum()), flush=True)
    s.ipm()
    print(f"ipm_batch (one launch): {min(timed(s.ipm) for _ in range(3)):.2f} ms", flush=True)
    print(f"ipm_batch_profiled: {min(float(s.ipm_profiled().sum()) for _ in range(3)):.2f} ms (sum of pass events)",
          flush=True)
    for dr in (0, 256, 512, 768, 1024):
        os.environ["HPMPC_MI355X_QUEUE_DRAIN"] = str(dr)
        t = min(timed(lambda: s.queue(1024, 1024).run()) for _ in range(3))
        print(f"queue(1024, 1024) drain<={dr}: {t:.2f} ms = {kk.sum() / t * 1e3:.0f} IP-iter/s", flush=True)
    for K in Ks:
        for dr in (0, 768, 2048, 4096):
            os.environ["HPMPC_MI355X_QUEUE_DRAIN"] = str(dr)
            ts = []
            for _ in range(2):
                Qk = s.queue(K * 1024, 8192)
                ts.append(timed(Qk.run))
            it = float(Qk.kk.sum().item())
            d = Qk.drained()
            print(f"K={K} slots 8192 drain<={dr}: {min(ts):.2f} ms, {it / min(ts) * 1e3:.0f} IP-iter/s, drained {d}",
                  flush=True)


if __name__ == "__main__":
    main()
