"""Batch vs problem-queue throughput on the benchmark workload (diagnostic)."""
import os
import sys
import time

import torch

from hpmpc_amd.batch import BatchSolver
from hpmpc_amd.shard import make_shard

qp = make_shard(100, 12, 4, 0, 1, 1024)
s = BatchSolver(qp, k_max=50)
s.ipm()
torch.cuda.synchronize()
it_batch = int(s.kk.sum())
t0 = time.perf_counter()
for _ in range(3):
    s.ipm()
torch.cuda.synchronize()
tb = (time.perf_counter() - t0) / 3
print(f"batch: {tb*1e3:.2f} ms/batch  {it_batch/tb/1e6:.3f} M IP-iter/s", flush=True)
for steps in [int(x) for x in sys.argv[1:]] or [10]:
    for slots in [int(x) for x in os.environ.get("QP_SLOTS", "1024 2048").split()]:
        Q = s.queue(steps * 1024, slots)
        Q.run()
        torch.cuda.synchronize()
        its = int(Q.kk.sum())
        t0 = time.perf_counter()
        _, ticks = Q.run()
        torch.cuda.synchronize()
        tq = time.perf_counter() - t0
        pm, _ = Q.run(profiled=True)
        torch.cuda.synchronize()
        print(f"queue steps {steps} slots {slots}: {tq*1e3:.2f} ms = {tq/steps*1e3:.2f} ms/batch, ticks {ticks}, "
              f"{its/tq/1e6:.3f} M IP-iter/s; pass ms {[round(x,2) for x in pm]} per-tick fact "
              f"{pm[1]/ticks*1e3:.1f} us upd {pm[4]/ticks*1e3:.1f} us", flush=True)
