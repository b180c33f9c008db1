#!/usr/bin/env python3
"""Diagnostic: one batched solve (hpmpc_mi355x_ipm_batch: no queue, no active lists, no refills) of the benchmark
batch, for a rocprofv3 kernel trace of the pass kernels (compare hk_ipm_update with the queue run's)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hpmpc_amd.batch import BatchSolver
from hpmpc_amd.shard import make_shard

slots = int(sys.argv[1]) if len(sys.argv) > 1 else 0
qp = make_shard(100, 12, 4, 0, 1, 1024)
s = BatchSolver(qp, k_max=50)
if slots:
    s.queue(8 * 1024, slots).run()
else:
    s.ipm()
torch.cuda.synchronize()
print("done", int(s.kk.sum().item()))
