"""Data-parallel sharding of a batch of independent QPs over ranks.

Problems are independent, so a solve has no exchange step: each rank owns a contiguous block of the
global batch.  Two ways to get a block onto its rank:

* seed mode -- every rank generates its own block from the global per-problem seeds (no data-path
  collective at all);
* scatter mode -- rank 0 holds the whole batch and sends each rank its block with point-to-point sends
  (one batched isend/irecv group: over xGMI every rank-0 -> rank-r transfer has its own link), and the
  results (ux, pi, kk, ret) come back to rank 0 the same way (gather_to_root).

The timing collectives are the barrier and two scalar reductions (max of elapsed time, sum of iteration
counts).  The same code runs over RCCL (backend "nccl", device tensors) on the GPU box and over gloo
(CPU tensors) in the multi-process CPU tests.
"""
from __future__ import annotations

import numpy as np

from .ocp import OCPQP, batch_x0, mass_spring_qp


def split_batch(global_batch: int, world: int) -> int:
    """Problems per rank for a fixed global batch (strong scaling): contiguous equal blocks."""
    if global_batch <= 0 or global_batch % world:
        raise ValueError(f"global batch {global_batch} does not split evenly over {world} ranks")
    return global_batch // world


def scatter_from_root(dist, rank: int, world: int, local, blocks=None):
    """Rank 0 sends blocks[r] (a list of tensors) to rank r and copies blocks[0] into its own `local`;
    every other rank receives into `local` (preallocated tensors of the same shapes and dtypes).  One
    batch_isend_irecv group, so rank 0's sends to different ranks proceed concurrently."""
    if world == 1 or dist is None:
        if blocks is not None:
            for dst, src in zip(local, blocks[0]):
                dst.copy_(src)
        return
    ops = []
    if rank == 0:
        assert blocks is not None and len(blocks) == world
        for r in range(1, world):
            assert len(blocks[r]) == len(local)
            ops += [dist.P2POp(dist.isend, t.contiguous(), r) for t in blocks[r]]
        for dst, src in zip(local, blocks[0]):
            dst.copy_(src)
    else:
        ops = [dist.P2POp(dist.irecv, t, 0) for t in local]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def gather_to_root(dist, rank: int, world: int, local):
    """The inverse of scatter_from_root: rank 0 returns [local of rank 0, ..., of rank world-1] (fresh
    tensors for the remote ranks), the others send theirs and return None."""
    if world == 1 or dist is None:
        return [list(local)]
    if rank == 0:
        out = [list(local)] + [[t.new_empty(t.shape) for t in local] for _ in range(1, world)]
        ops = [dist.P2POp(dist.irecv, out[r][i], r) for r in range(1, world) for i in range(len(local))]
    else:
        out = None
        ops = [dist.P2POp(dist.isend, t.contiguous(), 0) for t in local]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return out


def shard_range(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """Global problem indices [start, stop) owned by `rank` (weak scaling: per_rank fixed)."""
    assert 0 <= rank < world and per_rank > 0
    return rank * per_rank, (rank + 1) * per_rank


SHARD_SEED = 1


def make_shard(N: int, nx: int, nu: int, rank: int, world: int, per_rank: int, *, boxes: bool = True,
               time_variant: bool = True, x0_scale: float = 1.0) -> OCPQP:
    """The rank's block of the benchmark workload, a function of the global problem indices only: x0 of
    global problem p comes from PCG64(20261015+p) (problem 0 = the reference drivers' x0) and its
    time-variant stage perturbations from PCG64([SHARD_SEED, p]).  So global problem p is bitwise the same QP
    whether it is solved in a world-1 batch or in rank r's block of an 8-GPU split (configs[3]), and a
    strong-scaling curve compares identical inputs (BASELINE.json north_star)."""
    start, stop = shard_range(rank, world, per_rank)
    return global_block(N, nx, nu, start, stop, boxes=boxes, time_variant=time_variant, x0_scale=x0_scale)


def global_block(N: int, nx: int, nu: int, start: int, stop: int, *, boxes: bool = True,
                 time_variant: bool = True, x0_scale: float = 1.0) -> OCPQP:
    """Global problems [start, stop) of the benchmark workload (see make_shard); x0_scale shrinks the initial
    states (the configs[4] IPM leg, whose N = 200 horizon makes most x0 ~ U(-2.5, 2.5) draws box-infeasible)."""
    X0 = x0_scale * batch_x0(nx, stop - start, start=start)
    return mass_spring_qp(N, nx, nu, boxes=boxes, batch=stop - start, x0=X0, time_variant=time_variant,
                          seed=SHARD_SEED, problem_ids=np.arange(start, stop))


class Reducer:
    """Barrier + scalar max/sum over ranks; a no-op group of one when `dist` is None."""

    def __init__(self, dist=None, device="cpu"):
        self.dist = dist
        self.device = device

    def _all_reduce(self, x: float, op) -> float:
        if self.dist is None:
            return float(x)
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        return self._all_reduce(x, None if self.dist is None else self.dist.ReduceOp.MAX)

    def min(self, x: float) -> float:
        return self._all_reduce(x, None if self.dist is None else self.dist.ReduceOp.MIN)

    def sum(self, x: float) -> float:
        return self._all_reduce(x, None if self.dist is None else self.dist.ReduceOp.SUM)


COUPLED_SEED = 7


def coupled_shard(N: int, nx: int, nu: int, rank: int, world: int, per_rank: int, *, boxes: bool = True) -> OCPQP:
    """The benchmark block (make_shard) with strongly coupled stage Hessians: every stage's [R S'; S Q] becomes
    diag(R, Q) + G G' / nux with G ~ N(0, 1) (nux x nux) from PCG64([COUPLED_SEED, p]) for global problem p (the
    random_qp style of the parity tests).  The blocks stay positive definite (lambda_min >= 1) but are far from
    diagonally dominant, so Gershgorin's bound on them is negative: the workload of the clamp certificate's
    shifted-Cholesky bound (hk_riccati.h cert_g_shift; VERDICT r4 item 5, bench.py 'coupled')."""
    from .ocp import pack_lib4_batch, unpack_lib4

    qp = make_shard(N, nx, nu, rank, world, per_rank, boxes=boxes)
    start, stop = shard_range(rank, world, per_rank)
    G = np.empty((stop - start, N + 1, nx + nu, nx + nu))
    for i, p in enumerate(range(start, stop)):
        G[i] = np.random.Generator(np.random.PCG64([COUPLED_SEED, p])).standard_normal(G.shape[1:])
    for k in range(N + 1):
        nux = qp.nux(k)
        M = np.stack([unpack_lib4(qp.RSQrq[k][i], nux + 1, nux) for i in range(stop - start)])
        Gk = G[:, k, :nux, :nux]
        M[:, :nux, :nux] += Gk @ np.swapaxes(Gk, 1, 2) / max(nux, 1)
        qp.RSQrq[k] = pack_lib4_batch(M)
    return qp
