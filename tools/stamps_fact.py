#!/usr/bin/env python3
"""Diagnostic: cycles per phase of one backward stage (problem 0, stage 50) of the IPM factorisation pass, from
the HK_STAMPS build (hpmpc_amd/build.py build_stamps).  Last writer wins: the stamps are those of the final
hk_ipm_fact pass that problem 0 ran.  Usage: stamps_fact.py [slots] (0: one problem alone)."""
import os, sys, ctypes as C
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hpmpc_amd.batch as hb
hb.LIBPATH = hb.LIBPATH.replace("libhpmpc_mi355x.so", "libhpmpc_mi355x_stamps.so")
from hpmpc_amd.batch import BatchSolver, lib
from hpmpc_amd.shard import make_shard

slots = int(sys.argv[1]) if len(sys.argv) > 1 else 0
qp = make_shard(100, 12, 4, 0, 1, 1 if slots == 0 else 1024)
s = BatchSolver(qp, k_max=50)
dbg = torch.zeros(64, dtype=torch.int64, device="cuda")
lib().hpmpc_mi355x_debug_buffer.argtypes = [C.c_void_p]
lib().hpmpc_mi355x_debug_buffer(dbg.data_ptr())
if slots == 0:
    s.ipm()
else:
    s.queue(2 * 1024, slots).run()
torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
ph = [(0, 5, "stage table (LDS) + readfirstlane"), (5, 6, "prefetch issue (bwd_fetch)"), (6, 1, "store record"),
      (1, 2, "box terms + MFMA + row update"), (2, 16, "u-block Cholesky"), (16, 3, "(empty blocks, kg)"),
      (3, 4, "residuals of stage k-1")]
print(f"slots {slots}: stage 50, total {t[4] - t[0]} cycles")
for a, b, n in ph:
    print(f"  {n:36s} {t[b] - t[a]:7d}")
