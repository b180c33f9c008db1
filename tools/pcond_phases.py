"""Per-phase cycle totals of hk_pcond workgroup (block 0, problem 0) at configs[4] (512 x N=200 nx=24 nu=6 -> 20
blocks, no boxes), from the -DHK_STAMPS build (build.py build_stamps; HPMPC_MI355X_LIB=.../libhpmpc_mi355x_stamps.so)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpmpc_amd.pcond as hp  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
qp = make_shard(200, 24, 6, 0, 1, B, boxes=False)  # bench.py's configs[4] leg
s = hp.PcondSolver(qp, 20)
dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
L = hp.lib()
L.hpmpc_mi355x_pcond_debug.argtypes = [C.c_void_p]
s.condense()
torch.cuda.synchronize()
assert L.hpmpc_mi355x_pcond_debug(dbg.data_ptr()) == 0
s.condense()
torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
names = {1: "BAbt phase: Gamma_0 / loop top", 2: "BAbt_j staging", 11: "BAbt_{j+1} prefetch issue",
         12: "Gamma_j gemm + Gamma store", 3: "B rows, barrier", 4: "B2 store, barrier",
         5: "RSQ: D store, Gamma_{s-1} load", 6: "chol_aug (wave 0) | M (waves 1-3)", 7: "wait for M",
         13: "RSQ / Gamma DMA issue", 14: "W gemm", 8: "wait RSQ, barrier", 9: "W and pL gemms", 10: "DCtd, tail"}
tot = t[1:15].sum()
print(f"batch {B}: hk_pcond block (0, 0): {tot} cycles")
for i in (1, 2, 11, 12, 3, 4, 5, 6, 7, 13, 14, 8, 9, 10):
    print(f"  {names[i]:34s} {t[i]:10d}  {100.0 * t[i] / max(tot, 1):5.1f} %")
