"""configs[4] with boxes (512 x N=200 nx=24 nu=6 -> 20 blocks): per-problem distance of the GPU pipeline (condense ->
wide IPM -> expand) from the oracle's pipeline, for converged problems, beside the distance between the oracle and
its own -mfma -ffp-contract=fast build (oracle/liboracle_fma.so) on the same problems: how far the GPU point sits
from the CPU point compared with the CPU builds' own spread."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from hpmpc_amd.cabi import HpmpcAPI, load  # noqa: E402
from hpmpc_amd.pcond import PcondSolver  # noqa: E402
from hpmpc_amd.shard import global_block  # noqa: E402

o1 = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")
o2 = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle_fma.so")), "orc_")
bq = global_block(200, 24, 6, 0, 512)
s = PcondSolver(bq, 20)
s.solve_ipm(k_max=60)
torch.cuda.synchronize()
ret = s.ret2.cpu().numpy()
conv = np.nonzero(ret == 0)[0]


def rel(a, b):
    m = 0.0
    for x, y in zip(a, b):
        n = min(len(x), len(y))
        x, y = np.asarray(x[:n]), np.asarray(y[:n])
        m = max(m, float(np.max(np.abs(x - y) / np.maximum(1.0, np.abs(y)), initial=0.0)))
    return m


for p in [int(conv[i]) for i in np.linspace(0, conv.size - 1, 6).astype(int)]:
    qp = bq.problem(p)
    es = []
    for o in (o1, o2):
        c, _ = o.part_cond(qp.copy(), 20)
        r = o.ipm(c.copy(), k_max=60)
        es.append(o.part_expand(qp, c, r["ux"], r["pi"], r["lam"], r["t"]))
    U, Pi = s.solution(p)
    Lm, T = s.multipliers(p)
    e1, e2 = es
    print(f"problem {p}: gpu-oracle ux {rel(U, e1['ux']):.1e} pi {rel(Pi, e1['pi']):.1e} lam {rel(Lm, e1['lam']):.1e} "
          f"t {rel(T, e1['t']):.1e} | oracle_fma-oracle ux {rel(e2['ux'], e1['ux']):.1e} pi {rel(e2['pi'], e1['pi']):.1e} "
          f"lam {rel(e2['lam'], e1['lam']):.1e} t {rel(e2['t'], e1['t']):.1e}", flush=True)
