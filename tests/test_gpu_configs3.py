"""configs[3] (BASELINE.json): 4096 x N=100 nx=12 nu=4 full IPM sharded over 8 GPUs, at its per-rank shape.

Each rank solves its 512-problem block of the global batch through the problem queue at the bench's slot count
(bench.py --gpus 8 --global-batch 4096: slots = max(2 x 512, 2048)).  Here, on one GPU, the blocks of ranks 0 and 7
are solved exactly as those ranks would and checked three ways:
* problem data are a function of the global index only (hpmpc_amd.shard): the rank's block is bitwise the same
  problems as the corresponding rows of a world-1 batch, and its results are bitwise those of that batch's solve;
* a queue of two passes over the block gives bitwise the batched solve (entry q solves problem q % 512);
* sampled problems, including non-converged ones, match the CPU oracle at the IPM gates.
"""
import os

import numpy as np
import pytest

from helpers import TOL_IPM, compare_ipm

pytestmark = pytest.mark.gpu
N, NX, NU, WORLD, PER = 100, 12, 4, 8, 512
SLOTS = max(2 * PER, 2048)


@pytest.fixture(autouse=True)
def _queue_ticks_to_the_end(monkeypatch):
    """The rank block is compared bitwise with the world-1 batched solve: no multi-wave drain (test_gpu_parity.py
    test_queue_drain_matches_oracle covers it)."""
    monkeypatch.setenv("HPMPC_MI355X_QUEUE_DRAIN", "0")


def _solve_queue(qp, nq):
    import torch

    from hpmpc_amd.batch import BatchSolver

    s = BatchSolver(qp, k_max=50)
    Q = s.queue(nq, SLOTS)
    Q.run()
    torch.cuda.synchronize()
    return s, Q


@pytest.mark.parametrize("rank", [0, 7])
def test_configs3_rank_block(oracle, rank):
    import torch

    from hpmpc_amd.batch import BatchSolver, pack_batch
    from hpmpc_amd.shard import global_block, make_shard, shard_range

    qp = make_shard(N, NX, NU, rank, WORLD, PER)
    start, stop = shard_range(rank, WORLD, PER)
    # the world-1 batch that holds these global problems (1024 problems, the rank's block in one half)
    w0 = (start // 1024) * 1024
    big = global_block(N, NX, NU, w0, w0 + 1024)
    rows = slice(start - w0, stop - w0)
    for a, b in zip(pack_batch(qp), pack_batch(big)):
        np.testing.assert_array_equal(a, b[rows])

    s, Q = _solve_queue(qp, 2 * PER)
    kk, ret = Q.kk.cpu().numpy(), Q.ret.cpu().numpy()
    # two passes over the block: the same problem solved in another slot is bitwise the same
    for name in ("ux", "pi", "lam", "t", "kk", "ret"):
        a = getattr(Q, name)
        assert torch.equal(a[:PER], a[PER:]), name
    # and bitwise the world-1 batch's solve of the same global problems
    sb = BatchSolver(big, k_max=50)
    sb.ipm()
    torch.cuda.synchronize()
    for name in ("ux", "pi", "lam", "t", "kk", "ret"):
        assert torch.equal(getattr(Q, name)[:PER], getattr(sb, name)[rows]), name
    assert (ret[:PER] == 0).sum() > 0.85 * PER and kk.max() <= 50

    # sampled problems against the oracle: first / last of the block and non-converged ones
    ux, pi, lam, t = (getattr(Q, n).cpu().numpy() for n in ("ux", "pi", "lam", "t"))
    bad = [int(p) for p in np.nonzero(ret[:PER] != 0)[0][:3]]
    for p in [0, PER // 2, PER - 1] + bad:
        one = qp.problem(p)
        r = oracle.ipm(one, k_max=50)
        got = dict(kk=int(kk[p]), ret=int(ret[p]), ux=[ux[p, k] for k in range(N + 1)],
                   pi=[pi[p, k] for k in range(N)], lam=[lam[p, k] for k in range(N + 1)],
                   t=[t[p, k] for k in range(N + 1)])
        # a diverging infeasible draw (ret 2, lam -> 1e30) compares by ret and kk only (helpers.compare_ipm)
        compare_ipm(one, got, r, tol=TOL_IPM, allow_divergent=bool(ret[p] == 2))
