"""Debug probe: the wide KKT re-solve on size patterns between the passing and the failing case."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hpmpc_amd.cabi import HpmpcAPI, load  # noqa: E402
from helpers import random_qp  # noqa: E402

P = HpmpcAPI(load(os.path.join(ROOT, "hpmpc_amd", "lib", "libhpmpc_mi355x.so")))
O = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)), initial=0.0))


def kerr(qp, a, b):
    out = {}
    for key in ("ux", "pi", "lam", "t"):
        e = 0.0
        for k in range(len(b[key])):
            n = qp.nux(k) if key == "ux" else (int(qp.nx[k + 1]) if key == "pi" else qp.nconstr(k))
            e = max(e, rel(a[key][k][:n], b[key][k][:n]))
        out[key] = f"{e:.1e}"
    return out


CASES = [
    ("uniform", 4, [0] + [20] * 4, [4] * 4 + [0], [4] + [6] * 4),
    ("nu_vary", 4, [0] + [20] * 4, [4, 6, 3, 5, 0], [4] + [6] * 4),
    ("nx_vary", 4, [0, 20, 24, 18, 22], [4] * 4 + [0], [4] + [6] * 4),
    ("nx_vary_nobox", 4, [0, 20, 24, 18, 22], [4] * 4 + [0], None),
    ("both", 4, [0, 20, 24, 18, 22], [4, 6, 3, 5, 0], [4] + [6] * 4),
]
for tag, N, nx, nu, nb in CASES:
    qp = random_qp(N, nx, nu, nb, seed=3)
    a = P.ipm(qp.copy(), k_max=60)
    b = O.ipm(qp.copy(), k_max=60)
    rng = np.random.default_rng(1)
    bb = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    qq = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ka = P.kkt_new_rhs(qp.copy(), a["work"], bb, qq)
    kb = O.kkt_new_rhs(qp.copy(), b["work"], bb, qq)
    print(tag, "ipm", a["kk"], b["kk"], kerr(qp, a, b), "kkt", kerr(qp, ka, kb))
