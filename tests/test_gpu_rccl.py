"""RCCL (torch.distributed "nccl" on ROCm) on the device, world size 1: the bench's Reducer (barrier, max / min / sum
of scalars as CUDA tensors) and the scatter / gather helpers run through a real RCCL communicator.  The world-2
data path itself is covered over gloo on the CPU (test_shard_gloo.py); an 8-GPU run is the driver's."""
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_reducer_and_scatter_world1():
    import torch
    import torch.distributed as dist

    from hpmpc_amd.shard import Reducer, gather_to_root, scatter_from_root

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        red = Reducer(dist, "cuda")
        red.barrier()
        assert red.sum(3.5) == 3.5 and red.max(-2.0) == -2.0 and red.min(7.0) == 7.0
        # the rank-0 scatter / gather of a block of device tensors (world 1: a local copy each way)
        src = [torch.arange(12, dtype=torch.float64, device="cuda"), torch.ones(5, dtype=torch.int32, device="cuda")]
        local = [torch.empty_like(t) for t in src]
        scatter_from_root(dist, 0, 1, local, [src])
        assert all(torch.equal(a, b) for a, b in zip(local, src))
        out = gather_to_root(dist, 0, 1, local)
        assert len(out) == 1 and all(torch.equal(a, b) for a, b in zip(out[0], src))
        # one real collective on a device tensor
        x = torch.full((4,), 2.0, dtype=torch.float64, device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        assert torch.equal(x, torch.full_like(x, 2.0))
    finally:
        dist.destroy_process_group()
