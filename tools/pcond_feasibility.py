import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from hpmpc_amd.shard import make_shard
from hpmpc_amd.pcond import PcondSolver
for sc in (1.0, 0.5, 0.3, 0.2):
    qp = make_shard(200, 24, 6, 0, 1, 512, boxes=True, x0_scale=sc)
    s = PcondSolver(qp, 20); s.solve_ipm(k_max=50); torch.cuda.synchronize()
    ret = s.ret2.cpu().numpy(); kk = s.kk2.cpu().numpy()
    print(sc, {int(v): int((ret == v).sum()) for v in np.unique(ret)}, "mean kk", kk.mean(), "conv kk", kk[ret == 0].mean() if (ret == 0).any() else 0, flush=True)
