"""hk_pcond alone at configs[4] (512 x N=200 nx=24 nu=6 -> 20 blocks; no boxes and the boxed IPM leg's data): ms per
launch, median of 5 rounds of 20.  The variant follows HPMPC_MI355X_PCOND_GL (read once per process): run once per
setting for an A/B (tools/gpu_steps.sh)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpmpc_amd.pcond as hp  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
for boxes in (False, True):
    s = hp.PcondSolver(make_shard(200, 24, 6, 0, 1, B, boxes=boxes, x0_scale=0.2), 20)
    s.condense()
    torch.cuda.synchronize()
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            s.condense()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 20)
    print(f"PCOND_GL={os.environ.get('HPMPC_MI355X_PCOND_GL', 'default')} boxes={boxes} batch {B}: "
          f"{float(np.median(res)):.4f} ms per condensing launch", flush=True)
