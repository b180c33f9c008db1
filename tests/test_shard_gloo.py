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


def test_shard_data_depend_on_global_index_only():
    """Global problem p is bitwise the same QP in a world-1 batch and in any rank's block of any split
    (configs[3]: 4096 over 8 ranks is the same problem set as 4096 on one GPU)."""
    from hpmpc_amd.batch import pack_batch

    whole = pack_batch(make_shard(8, 12, 4, 0, 1, 16))
    for world in (2, 4, 8):
        per = 16 // world
        for r in range(world):
            blk = pack_batch(make_shard(8, 12, 4, r, world, per))
            for a, b in zip(whole, blk):
                np.testing.assert_array_equal(a[r * per:(r + 1) * per], b)
    # and the problems of a batch differ from one another
    assert not np.array_equal(whole[0][1], whole[0][2])


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


# ---------------------------------------------------------------- scatter mode
def _solve_block(qp):
    """Solve a received block problem by problem; pack the results like the device API's outputs."""
    import torch

    res = _solve(qp)
    B, N = qp.batch, qp.N
    ux = torch.zeros((B, N + 1, 16), dtype=torch.float64)
    pi = torch.zeros((B, N + 1, 16), dtype=torch.float64)
    kk = torch.zeros(B, dtype=torch.int32)
    ret = torch.zeros(B, dtype=torch.int32)
    for p, r in enumerate(res):
        for k in range(N + 1):
            n = qp.nux(k)
            ux[p, k, :n] = torch.from_numpy(np.asarray(r["ux"][k][:n]))
            if k < N:
                m = int(qp.nx[k + 1])
                pi[p, k, :m] = torch.from_numpy(np.asarray(r["pi"][k][:m]))
        kk[p], ret[p] = r["kk"], r["ret"]
    return [ux, pi, kk, ret]


def _scatter_worker(rank, port, out):
    import torch
    import torch.distributed as dist

    from hpmpc_amd.batch import pack_batch, unpack_batch
    from hpmpc_amd.ocp import mass_spring_qp
    from hpmpc_amd.shard import gather_to_root, scatter_from_root

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    template = mass_spring_qp(N, NX, NU)  # sizes and idxb only: every rank knows the problem class
    shapes = [a.shape[1:] for a in pack_batch(make_shard(N, NX, NU, 0, 1, 1))]
    local = [torch.zeros((PER_RANK,) + tuple(s), dtype=torch.float64) for s in shapes]
    blocks = None
    if rank == 0:  # rank 0 holds the whole global batch, block r for rank r
        blocks = [[torch.from_numpy(a) for a in pack_batch(make_shard(N, NX, NU, r, WORLD, PER_RANK))]
                  for r in range(WORLD)]
    scatter_from_root(dist, rank, WORLD, local, blocks)
    qp = unpack_batch(template, *local)
    got = gather_to_root(dist, rank, WORLD, _solve_block(qp))
    if rank == 0:
        out["res"] = [[t.numpy().copy() for t in g] for g in got]
    out[rank] = [t.numpy().copy() for t in local]
    dist.destroy_process_group()


def test_gloo_world2_scatter_solve_gather_matches_single_process():
    """Rank 0 scatters the blocks of the global batch, each rank solves its block, the results are
    gathered on rank 0: bit for bit what one process solving every block produces."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    from hpmpc_amd.batch import pack_batch

    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_scatter_worker, args=(port, out), nprocs=WORLD, join=True)
        out = dict(out)
    for r in range(WORLD):
        blk = make_shard(N, NX, NU, r, WORLD, PER_RANK)
        # the scattered data are the rank's block, unchanged
        for a, b in zip(out[r], pack_batch(blk)):
            np.testing.assert_array_equal(a, b)
        ref = [t.numpy() for t in _solve_block(blk)]
        for a, b in zip(out["res"][r], ref):
            np.testing.assert_array_equal(a, b)
    assert not np.array_equal(out["res"][0][0], out["res"][1][0])


def test_bench_launches_world2_ranks():
    """`bench.py --gpus 2` starts two ranks (torch.distributed.run child) that reach init_process_group
    with world size 2 before any GPU call (--check-launch: gloo, no device)."""
    import json
    import subprocess
    import sys

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--check-launch"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1] and all(x["world"] == 2 for x in lines), lines
