"""Per-phase cycle totals of one wide-IPM solve (workgroup 0) at configs[4] with boxes, from the -DHK_STAMPS build
(build.py build_stamps; loaded through HPMPC_MI355X_LIB=.../libhpmpc_mi355x_stamps.so)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpmpc_amd.pcond as hp  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
qp = make_shard(200, 24, 6, 0, 1, B, boxes=True, x0_scale=0.2)  # bench.py's configs[4] IPM leg
s = hp.PcondSolver(qp, 20)
s.condense()
dbg = torch.zeros(32, dtype=torch.int64, device="cuda")
L = hp.lib()
L.hpmpc_mi355x_wide_ipm_debug.argtypes = [C.c_void_p]
s.ipm()
torch.cuda.synchronize()
assert L.hpmpc_mi355x_wide_ipm_debug(dbg.data_ptr()) == 0
s.ipm()
torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
names = ["hess_grad_res", "ric_sv", "dt_dlam (pred)", "mu_aff + centering", "grad_res", "ric_trs", "dt_dlam (corr)",
         "update_var", "residuals", "loop test"]
tot = t[:10].sum()
print(f"batch {B}: problem 0, {t[31]} stamps, {tot} cycles in the phase-2 loop")
for i, n in enumerate(names):
    print(f"  {n:20s} {t[i]:12d}  {100.0 * t[i] / max(tot, 1):5.1f} %")
sub = ["stage top -> W load", "W load (lib4 -> LDS)", "W = BAbt Lxx (MFMA)", "Pb, row", "syrk W W' (MFMA)",
       "-> general terms", "DCt diag DCt' (MFMA)", "panel factor (wave 0)", "trailing update (MFMA)",
       "factor store, Lxx copy", "forward substitution"]
st = t[12:23]
print(f"  inside every ric_sv of the solve (phase 1 included), {st.sum()} cycles:")
for i, n in enumerate(sub):
    print(f"    {n:26s} {st[i]:12d}  {100.0 * st[i] / max(st.sum(), 1):5.1f} %")
tsub = ["backward: L, BAbt, q loads", "backward: box + DCt qx_g", "backward: + BAbt w, n-form solve",
        "backward: Pb, w", "forward: BAbt load, L' x product", "forward: t-form solve (wave 0)",
        "forward: x_{k+1}, next L load", "forward: pi"]
tt = t[23:31]
print(f"  inside every ric_trs of the solve, {tt.sum()} cycles:")
for i, n in enumerate(tsub):
    print(f"    {n:34s} {tt[i]:12d}  {100.0 * tt[i] / max(tt.sum(), 1):5.1f} %")
