"""Diagnostic: cycles per phase of one phase-2 IP iteration (problem 0, iteration 5), HK_STAMPS build."""
import os, sys, ctypes as C
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hpmpc_amd.batch as hb
hb.LIBPATH = hb.LIBPATH.replace("libhpmpc_mi355x.so", "libhpmpc_mi355x_stamps.so")
from hpmpc_amd.batch import BatchSolver, lib
from hpmpc_amd.shard import make_shard
qp = make_shard(100, 12, 4, 0, 1, 1024)
s = BatchSolver(qp, k_max=50)
dbg = torch.zeros(64, dtype=torch.int64, device='cuda')
lib().hpmpc_mi355x_debug_buffer.argtypes = [C.c_void_p]
lib().hpmpc_mi355x_debug_buffer(dbg.data_ptr())
for _ in range(2):
    s.ipm(); torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
names = ["sv backward (+hessian)", "sv forward (+alpha)", "mu_aff pass", "trs (+centering, alpha)",
         "update + residuals"]
tot = t[37] - t[32]
print(f"phase-2 iteration (problem 0, first phase-2 iteration): {tot} cycles = {tot / 101:.0f} per stage")
for i, n in enumerate(names):
    d = t[33 + i] - t[32 + i]
    print(f"  {n:16s} {d:8d}  {d / 101:7.0f}/stage  {100 * d / tot:5.1f}%")
