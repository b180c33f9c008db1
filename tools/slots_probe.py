"""Resident-slot sweep of the problem queue on the headline workload (1024 x N=100 nx=12 nu=4 per batch, K batches):
IP-iter/s per slot count, best of two runs each.
    SLOTS_SWEEP=2048,4096,6144 python3 tools/slots_probe.py [K ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def run(solver, K, slots):
    Q = solver.queue(K * 1024, slots)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Q.run()
    torch.cuda.synchronize()
    return float(Q.kk.sum().item()) / (time.perf_counter() - t0)


def main():
    Ks = [int(x) for x in sys.argv[1:]] or [20, 40]
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    for K in Ks:
        for sl in [int(x) for x in os.environ.get("SLOTS_SWEEP", "2048,4096,6144").split(",")]:
            run(s, 2, sl)
            v = max(run(s, K, sl) for _ in range(2))
            print(f"K={K} slots={sl}: {v:.0f} IP-iter/s", flush=True)


if __name__ == "__main__":
    main()
