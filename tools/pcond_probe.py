"""Per-kernel timing of the partial-condensing pipeline at configs[4] (512 x N=200 nx=24 nu=6 -> N2=20)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hpmpc_amd.ocp import mass_spring_qp
from hpmpc_amd.pcond import PcondSolver

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
qp = mass_spring_qp(200, 24, 6, boxes=False, batch=B, time_variant=True, seed=3)
s = PcondSolver(qp, 20)
for _ in range(2):
    s.solve()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
R = 5
tot = [0.0, 0.0, 0.0]
for _ in range(R):
    ev[0].record(); s.condense(); ev[1].record(); s.riccati(); ev[2].record(); s.expand(); ev[3].record()
    torch.cuda.synchronize()
    for i in range(3):
        tot[i] += ev[i].elapsed_time(ev[i + 1])
print(f"batch {B}: condense {tot[0]/R:.3f} ms  riccati {tot[1]/R:.3f} ms  expand {tot[2]/R:.3f} ms  "
      f"-> {B / (sum(tot)/R) * 1e3:.0f} pipelines/s")
