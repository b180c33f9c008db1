"""Diagnostic: per-phase cycle breakdown of one stage (problem 0, stage 50) from the HK_STAMPS build."""
import os, sys, ctypes as C
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hpmpc_amd.batch as hb
hb.LIBPATH = hb.LIBPATH.replace("libhpmpc_mi355x.so", "libhpmpc_mi355x_stamps.so")
from hpmpc_amd.batch import BatchSolver, lib
from hpmpc_amd.ocp import mass_spring_qp
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
qp = mass_spring_qp(100, 12, 4, boxes=False, batch=B, time_variant=True, seed=1)
s = BatchSolver(qp, k_max=1)
dbg = torch.zeros(64, dtype=torch.int64, device='cuda')
lib().hpmpc_mi355x_debug_buffer.argtypes = [C.c_void_p]
lib().hpmpc_mi355x_debug_buffer(dbg.data_ptr())
for _ in range(3):
    s.ric_sv(); torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
names = {0: 'bwd top', 1: 'fetch issued', 2: 'mfma+aug done', 3: 'chol done', 4: 'stored',
         8: 'fwd top', 9: 'pre-solve', 10: 'solve done', 11: 'gemv done', 12: 'pi done'}
print(f"batch {B}: backward stage 50 (cycles from loop top):")
for i in [1, 2, 3, 4]:
    print(f"  {names[i]:16s} {t[i]-t[0]:6d}  (+{t[i]-t[i-1]})")
print("  chol blocks done at: " + " ".join(f"b{b}: {t[16+2*b]-t[2]:5d}" for b in range(4)))
print("  block 1 detail: " + " ".join(f"{n}:{t[24+i]-t[24]}" for i, n in enumerate(
    ["top", "bcast", "piv0", "piv1", "piv2", "piv3", "sel", ]) ) + f" after-mfma:{t[18]-t[24]}")
print("forward stage 50:")
for i in [9, 10, 11, 12]:
    print(f"  {names[i]:16s} {t[i]-t[8]:6d}  (+{t[i]-t[i-1]})")
