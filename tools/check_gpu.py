"""Quick GPU-vs-oracle diagnostic (prints max abs errors per entry point)."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpmpc_amd.ocp import mass_spring_qp
from hpmpc_amd.cabi import load, HpmpcAPI, bq_from_qp
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
gpu = HpmpcAPI(load(os.path.join(root, 'hpmpc_amd/lib/libhpmpc_mi355x.so')))
orc = HpmpcAPI(load(os.path.join(root, 'oracle/liboracle.so')), 'orc_')
def md(A, B, n=None):
    return max(float(np.max(np.abs(a[:len(b)] - b))) if len(b) else 0.0 for a, b in zip(A, B))
for (N, nx, nu) in [(10, 8, 3), (30, 8, 3), (100, 12, 4)]:
    qp = mass_spring_qp(N, nx, nu, boxes=False)
    t0 = time.time()
    g = gpu.ric_sv(qp.copy(), compute_Pb=1)
    o = orc.ric_sv(qp.copy(), compute_Pb=1)
    nux = [qp.nux(k) for k in range(N + 1)]
    eu = max(float(np.max(np.abs(g[0][k][:nux[k]] - o[0][k][:nux[k]]))) for k in range(N + 1))
    ep = max(float(np.max(np.abs(g[1][k][:nx] - o[1][k][:nx]))) for k in range(N))
    eb = max(float(np.max(np.abs(g[2][k][:nx] - o[2][k][:nx]))) for k in range(N))
    print(f'sv N={N} nx={nx} nu={nu}: ux {eu:.3e} pi {ep:.3e} Pb {eb:.3e}  ({time.time()-t0:.2f}s)', flush=True)
    b, q = bq_from_qp(qp)
    rng = np.random.default_rng(1)
    b2 = [x + rng.standard_normal(x.shape) for x in b]; q2 = [x + rng.standard_normal(x.shape) for x in q]
    mg = gpu.ric_trf(qp.copy()); mo = orc.ric_trf(qp.copy())
    G = gpu.ric_trs(qp.copy(), mg, b=b2, q=q2); O = orc.ric_trs(qp.copy(), mo, b=b2, q=q2)
    eu = max(float(np.max(np.abs(G[0][k][:nux[k]] - O[0][k][:nux[k]]))) for k in range(N + 1))
    ep = max(float(np.max(np.abs(G[1][k][:nx] - O[1][k][:nx]))) for k in range(N))
    print(f'trf+trs: ux {eu:.3e} pi {ep:.3e}', flush=True)
    qp = mass_spring_qp(N, nx, nu, boxes=True)
    G = gpu.ipm(qp.copy()); O = orc.ipm(qp.copy())
    eu = max(float(np.max(np.abs(G['ux'][k][:nux[k]] - O['ux'][k][:nux[k]]))) for k in range(N + 1))
    ep = max(float(np.max(np.abs(G['pi'][k][:nx] - O['pi'][k][:nx]))) for k in range(N))
    print(f'ipm: ret {G["ret"]}/{O["ret"]} kk {G["kk"]}/{O["kk"]} ux {eu:.3e} pi {ep:.3e}', flush=True)
    if G['kk'] == O['kk']:
        print('   stat maxdiff', float(np.max(np.abs(G['stat'] - O['stat']))))
    print('   gpu stat', G['stat'].reshape(-1, 5)[:3])
    print('   orc stat', O['stat'].reshape(-1, 5)[:3])
