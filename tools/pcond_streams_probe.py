"""configs[4] (512 x N=200 nx=24 nu=6 condensed into 20 blocks) with S batches in flight: K pipelines (condense ->
condensed Riccati -> expand) issued round-robin on S streams, each stream with its own PcondSolver buffers; and the
same for the condensed IPM with boxes (condense -> wide IPM -> expand).
    python3 tools/pcond_streams_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.pcond import PcondSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def rate(sols, streams, K, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        j = i % len(sols)
        with torch.cuda.stream(streams[j]):
            fn(sols[j])
    torch.cuda.synchronize()
    return K * sols[0].nprob / (time.perf_counter() - t0)


def main():
    B = 512
    sts = [torch.cuda.Stream() for _ in range(3)]
    qp = make_shard(200, 24, 6, 0, 1, B, boxes=False)
    sols = [PcondSolver(qp, 20) for _ in range(3)]
    for S in (1, 2, 3, 1):
        rate(sols[:S], sts[:S], 4, lambda s: s.solve())
        v = max(rate(sols[:S], sts[:S], 20, lambda s: s.solve()) for _ in range(2))
        print(f"pcond solve streams={S}: {v:.0f} solves/s", flush=True)
    del sols
    qb = make_shard(200, 24, 6, 0, 1, B, boxes=True, x0_scale=0.2)
    sols = [PcondSolver(qb, 20) for _ in range(2)]
    for S in (1, 2, 1):
        rate(sols[:S], sts[:S], 2, lambda s: s.solve_ipm(k_max=50))
        v = rate(sols[:S], sts[:S], 4, lambda s: s.solve_ipm(k_max=50))
        it = float(sols[0].kk2.sum().item())
        print(f"pcond ipm streams={S}: {v:.0f} solves/s = {v * it / B:.0f} IP-iter/s", flush=True)


if __name__ == "__main__":
    main()
