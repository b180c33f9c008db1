"""Workload of the two-wave Riccati PMC passes (tools/pmc_ric2.sh): 1024 x N=100 nx=12 nu=4 sv batches, 10 launches
on the one-wave kernel (hk_ric_sv) and 10 on the two-wave kernel (hk_ric_sv2), one process."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hpmpc_amd.batch import BatchSolver
from hpmpc_amd.shard import make_shard

s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024, boxes=False), k_max=1)
for w in ("1", "2"):
    os.environ["HPMPC_MI355X_RIC_WAVES"] = w
    for _ in range(10):
        s.ric_sv(compute_pi=1)
    torch.cuda.synchronize()
print("done")
