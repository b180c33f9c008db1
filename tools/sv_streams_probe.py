"""Riccati sv (d_back_ric_rec_sv_tv_res, nb = 0) throughput with S batches in flight: K steps of one batch of 1024
each, issued round-robin on S streams (each stream its own solver buffers), against one stream.  One wave per problem
and 1024 problems fill one wave per SIMD; a second batch in flight is a second wave on every SIMD.
    python3 tools/sv_streams_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def rate(solvers, streams, K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        j = i % len(solvers)
        with torch.cuda.stream(streams[j]):
            solvers[j].ric_sv()
    torch.cuda.synchronize()
    return K * solvers[0].nprob / (time.perf_counter() - t0)


def main():
    K = 40
    for (N, nx, nu) in ((100, 12, 4), (50, 8, 3)):
        qp = make_shard(N, nx, nu, 0, 1, 1024, boxes=False)
        sol = [BatchSolver(qp, k_max=1) for _ in range(4)]
        sts = [torch.cuda.Stream() for _ in range(4)]
        for S in (1, 2, 3, 4, 1):
            rate(sol[:S], sts[:S], 8)
            v = max(rate(sol[:S], sts[:S], K) for _ in range(3))
            print(f"N={N} nx={nx} nu={nu} streams={S}: {v / 1e6:.3f} M fact/s", flush=True)
        ref = sol[0].ux.clone()
        for s in sol[1:]:
            assert torch.equal(s.ux, ref)


if __name__ == "__main__":
    main()
