"""Does the headline rate depend on how long the GPU has been busy?  The K=20 queue timed again and again in one
process, with the elapsed time since the first launch: IP-iter/s per repetition.
    python3 tools/warm_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    T0 = time.perf_counter()
    for r in range(reps):
        Q = s.queue(20 * 1024, 8192)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Q.run()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {r} at {t0 - T0:6.1f} s: {float(Q.kk.sum().item()) / dt:.0f} IP-iter/s ({dt * 1e3:.1f} ms)",
              flush=True)


if __name__ == "__main__":
    main()
