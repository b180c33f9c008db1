"""World-size-2 gloo run of the multi-GPU decomposition (CPU): each rank builds its own block of the
global batch and solves it with no data collective; the reductions bench.py uses (max time, sum of
iteration counts) must give the same totals as one process solving the whole batch.
The per-rank solver here is the CPU oracle (the bench uses the HIP library on the same shard)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from hpmpc_amd.shard import Reducer, make_shard, shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, NX, NU, PER_RANK, WORLD = 12, 4, 1, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(qp):
    from hpmpc_amd.cabi import HpmpcAPI, load

    orc = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")
    return [orc.ipm(qp.problem(p), k_max=30) for p in range(qp.batch)]


def _worker(rank, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    red = Reducer(dist, "cpu")
    qp = make_shard(N, NX, NU, rank, WORLD, PER_RANK)
    res = _solve(qp)
    kk = sum(r["kk"] for r in res)
    red.barrier()
    tot = red.sum(kk)
    mx = red.max(float(rank + 1))
    out[rank] = (tot, mx, [r["ux"][1][:NU + NX].tolist() for r in res])
    dist.destroy_process_group()


def test_shard_ranges_partition_the_batch():
    got = [shard_range(r, 4, 5) for r in range(4)]
    assert got == [(0, 5), (5, 10), (10, 15), (15, 20)]


def test_gloo_world2_matches_single_process():
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(port, out), nprocs=WORLD, join=True)
        out = dict(out)
    # single process: the same blocks, built and solved in turn
    kk_single = 0
    for r in range(WORLD):
        res = _solve(make_shard(N, NX, NU, r, WORLD, PER_RANK))
        kk_single += sum(x["kk"] for x in res)
        np.testing.assert_allclose(np.array(out[r][2]), np.array([x["ux"][1][:NU + NX] for x in res]), rtol=0,
                                   atol=0)
    for r in range(WORLD):
        assert out[r][0] == kk_single
        assert out[r][1] == float(WORLD)
    # rank blocks differ (global x0 seeds), i.e. ranks did not solve the same problems
    assert not np.allclose(out[0][2], out[1][2])
