"""Debug probe for the wide IPM: per-iteration stat and outputs against the oracle on one problem."""
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


def report(tag, qp, a, b):
    eu = max(rel(a["ux"][k][: qp.nux(k)], b["ux"][k][: qp.nux(k)]) for k in range(qp.N + 1))
    ep = max(rel(a["pi"][k][: int(qp.nx[k + 1])], b["pi"][k][: int(qp.nx[k + 1])]) for k in range(qp.N))
    print(f"{tag}: kk {a['kk']}/{b['kk']} ret {a['ret']}/{b['ret']} ux {eu:.2e} pi {ep:.2e}")
    if "stat" in a:
        n = min(len(a["stat"]), len(b["stat"]))
        print("  stat gpu", np.array2string(np.asarray(a["stat"][:n]).reshape(-1, 5)[:4], precision=6))
        print("  stat orc", np.array2string(np.asarray(b["stat"][:n]).reshape(-1, 5)[:4], precision=6))


import test_gpu_wide_ipm as T  # noqa: E402


def keyerr(qp, a, b):
    out = {}
    for key in ("ux", "pi", "lam", "t"):
        e = 0.0
        for k in range(len(b[key])):
            n = qp.nux(k) if key == "ux" else (int(qp.nx[k + 1]) if key == "pi" else qp.nconstr(k))
            e = max(e, rel(a[key][k][:n], b[key][k][:n]))
        out[key] = e
    return out


sel = [int(x) for x in sys.argv[1:]] or range(len(T.CASES))
for ci in sel:
    N, nx, nu, nb, ng = T.CASES[ci]
    qp = random_qp(N, nx, nu, nb, seed=97 * N + len(nx), ng=ng)
    b = O.ipm(qp.copy(), k_max=60)
    for km in range(1, b["kk"] + 1):
        a = P.ipm(qp.copy(), k_max=km)
        bb = O.ipm(qp.copy(), k_max=km)
        st = np.max(np.abs(np.asarray(a["stat"]) - np.asarray(bb["stat"])) / np.maximum(1e-300, np.abs(bb["stat"])))
        print(ci, km, a["kk"], bb["kk"], {k: f"{v:.1e}" for k, v in keyerr(qp, a, bb).items()}, f"stat {st:.1e}")

    a = P.ipm(qp.copy(), k_max=60)
    rng = np.random.default_rng(N + 3)
    bb_ = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    qq_ = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ka = P.kkt_new_rhs(qp.copy(), a["work"], bb_, qq_)
    kb = O.kkt_new_rhs(qp.copy(), b["work"], bb_, qq_)
    print("kkt", ci, {k: f"{v:.1e}" for k, v in keyerr(qp, ka, kb).items()})
    for k in range(N + 1):
        n = qp.nux(k)
        print("   stage", k, "ux", f"{rel(ka['ux'][k][:n], kb['ux'][k][:n]):.1e}",
              "lam", f"{rel(ka['lam'][k][:qp.nconstr(k)], kb['lam'][k][:qp.nconstr(k)]):.1e}",
              "pi", f"{rel(ka['pi'][k][:int(qp.nx[k + 1])], kb['pi'][k][:int(qp.nx[k + 1])]):.1e}" if k < N else "")
