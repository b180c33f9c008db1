"""Data-parallel sharding of a batch of independent QPs over ranks.

Problems are independent, so a solve has no exchange step: each rank owns a contiguous block of the
global batch, generates that block itself from the global per-problem seeds (no scatter), and the
only collectives are the barrier and two scalar reductions (max of elapsed time, sum of iteration
counts).  The same code runs over RCCL (backend "nccl", device tensors) on the GPU box and over gloo
(CPU tensors) in the multi-process CPU tests.
"""
from __future__ import annotations

from .ocp import OCPQP, batch_x0, mass_spring_qp


def shard_range(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """Global problem indices [start, stop) owned by `rank` (weak scaling: per_rank fixed)."""
    assert 0 <= rank < world and per_rank > 0
    return rank * per_rank, (rank + 1) * per_rank


def make_shard(N: int, nx: int, nu: int, rank: int, world: int, per_rank: int, *, boxes: bool = True,
               time_variant: bool = True) -> OCPQP:
    """The rank's block of the benchmark workload.  x0 of global problem p comes from PCG64(20261015+p)
    (problem 0 = the reference drivers' x0); the time-variant stage perturbations of a block come
    from PCG64(1 + rank)."""
    start, stop = shard_range(rank, world, per_rank)
    X0 = batch_x0(nx, stop)[start:stop]
    return mass_spring_qp(N, nx, nu, boxes=boxes, batch=per_rank, x0=X0, time_variant=time_variant,
                          seed=1 + rank)


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

    def sum(self, x: float) -> float:
        return self._all_reduce(x, None if self.dist is None else self.dist.ReduceOp.SUM)
