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
L.hk_wide_ipm_debug.argtypes = [C.c_void_p]
s.ipm()
torch.cuda.synchronize()
assert L.hk_wide_ipm_debug(dbg.data_ptr()) == 0
s.ipm()
torch.cuda.synchronize()
t = dbg.cpu().numpy().astype(np.int64)
names = ["hess_grad_res", "ric_sv", "dt_dlam (pred)", "mu_aff + centering", "grad_res", "ric_trs", "dt_dlam (corr)",
         "update_var", "residuals", "loop test"]
tot = t[:10].sum()
print(f"batch {B}: problem 0, {t[31]} stamps, {tot} cycles in the phase-2 loop")
for i, n in enumerate(names):
    print(f"  {n:20s} {t[i]:12d}  {100.0 * t[i] / max(tot, 1):5.1f} %")
