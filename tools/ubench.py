"""Per-kernel timing of the batched entry points (N=100 nx=12 nu=4, batch 1024 unless overridden)."""
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hpmpc_amd.batch import BatchSolver
from hpmpc_amd.ocp import mass_spring_qp
N, nx, nu, B = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (100, 12, 4, 1024)))
qp = mass_spring_qp(N, nx, nu, boxes=False, batch=B, time_variant=True, seed=1)
s = BatchSolver(qp, k_max=1)
b = torch.zeros((B, N + 1, 16), dtype=torch.float64, device='cuda')
q = torch.zeros((B, N + 1, 16), dtype=torch.float64, device='cuda')
def timeit(f, reps=20):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
res = {}
res['sv'] = timeit(lambda: s.ric_sv())
res['sv_noPi'] = timeit(lambda: s.ric_sv(compute_pi=0))
res['trf'] = timeit(lambda: s.ric_trf())
res['trs'] = timeit(lambda: s.ric_trs(b, q, compute_Pb=1))
res['trs_noPb'] = timeit(lambda: s.ric_trs(b, q, compute_Pb=0))
for k, v in res.items():
    print(f"{k:10s} {v*1e3:9.1f} us/launch  {v*1e3/N:7.2f} us/stage  {B/(v*1e-3)/1e6:7.3f} M/s", flush=True)
qp2 = mass_spring_qp(N, nx, nu, boxes=True, batch=B, time_variant=True, seed=1)
s2 = BatchSolver(qp2, k_max=50)
t = timeit(lambda: s2.ipm(), reps=3)
kk = s2.kk.cpu().numpy()
print(f"ipm {t:.2f} ms  sum_kk {kk.sum()} max_kk {kk.max()} mean {kk.mean():.2f} -> {kk.sum()/(t*1e-3)/1e6:.3f} M IP-iter/s; per-iter latency {t/kk.max()*1e3:.1f} us")
