"""Per-problem distance to the CPU oracle (helpers.compare_ipm's measure) of the batched passes, the single-wave solo
kernel and the multi-wave solo kernel on configs[3]-style shard problems (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from helpers import compare_ipm  # noqa: E402
from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.cabi import HpmpcAPI, load  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402

oracle = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
qp = make_shard(100, 12, 4, 0, 1, B)
s = BatchSolver(qp, k_max=50)
N = qp.N


def grab():
    torch.cuda.synchronize()
    return {n: getattr(s, n).cpu().numpy().copy() for n in ("ux", "pi", "lam", "t", "kk", "ret")}


def run(how):
    for n in ("ux", "pi", "lam", "t"):
        getattr(s, n).zero_()
    if how == "batch":
        s.ipm()
    else:
        os.environ["HPMPC_MI355X_SOLO"] = "1" if how == "single" else "0"
        s.ipm_solo()
    return grab()


res = {h: run(h) for h in ("batch", "single", "mw")}
for p in range(B):
    r = oracle.ipm(qp.problem(p), k_max=50)
    line = [f"p{p} kk {r['kk']} ret {r['ret']}"]
    for h, g in res.items():
        got = dict(kk=int(g["kk"][p]), ret=int(g["ret"][p]), ux=[g["ux"][p, k] for k in range(N + 1)],
                   pi=[g["pi"][p, k] for k in range(N)], lam=[g["lam"][p, k] for k in range(N + 1)],
                   t=[g["t"][p, k] for k in range(N + 1)])
        try:
            e = compare_ipm(qp.problem(p), got, r, tol=1.0, allow_divergent=True)
            line.append(f"{h} {e:.1e}")
        except AssertionError as ex:
            line.append(f"{h} FAIL {ex}")
    print(" | ".join(line), flush=True)
