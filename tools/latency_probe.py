"""Latency of a lone QP (configs[1], N=100 nx=12 nu=4): device time per pass of the batched passes on a batch of
one, the one-launch solo kernel, a queue of one; then the HK_STAMPS per-phase breakdown of Riccati sv stage 50 for
a batch of 1 and of 1024 (needs hpmpc_amd/lib/libhpmpc_mi355x_stamps.so, build.py build_stamps)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.ocp import mass_spring_qp  # noqa: E402

one = mass_spring_qp(100, 12, 4, batch=1)
s = BatchSolver(one, k_max=50)
st = torch.cuda.current_stream()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


pm = s.ipm_profiled()
kk = int(s.kk[0].item())
print(f"lone QP: kk {kk}; batched passes (device ms, summed over k_max launches): "
      + " ".join(f"{n} {v:.3f}" for n, v in zip(["init", "fact", "pred", "corr", "update"], pm)))
t_batch = timed(s.ipm)
Q = s.queue(1, 1)
t_queue = timed(Q.run)
t_solo = timed(s.ipm_solo)
print(f"batch API {t_batch:.3f} ms | queue of one {t_queue:.3f} ms | solo {t_solo:.3f} ms "
      f"({t_solo * 1e3 / kk:.1f} us per IP iteration)")
for B in (1, 1024):
    qp = mass_spring_qp(100, 12, 4, boxes=False, batch=B, time_variant=True, seed=1)
    sb = BatchSolver(qp, k_max=1)
    t = timed(lambda: sb.ric_sv(), reps=20)
    print(f"riccati sv batch {B}: {t * 1e3:.1f} us per launch ({t * 1e3 / 101:.2f} us per stage)")
