#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (one counter group per pass, see tools/gpu_round.sh):
1 GiB calibration copy (known bytes), then the benchmark's IPM (N=100 nx=12 nu=4, batch 1024: a
problem queue of 8 batches through the bench's 8192 resident slots with its multi-wave drain, run twice), two
Riccati sv launches at that shape, two at configs[2] (1024 x N=50 nx=8 nu=3), and the configs[4]
partial-condensing pipeline (512 x N=200 nx=24 nu=6 -> 20 blocks: hk_pcond, hk_wide_sv, hk_pexpand) twice.
Prints kk_sum (iterations per queue run) and kk_pass (those the pass kernels ran, i.e. minus the drained ones)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    n = (1 << 30) // 8
    x = torch.rand(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    cal = C.CDLL(os.path.join(ROOT, "hpmpc_amd", "lib", "libhbm_calib.so"))
    cal.calib_run.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        assert cal.calib_run(x.data_ptr(), y.data_ptr(), n, s) == 0
    torch.cuda.synchronize()
    del x, y
    qp = make_shard(100, 12, 4, 0, 1, 1024)
    sol = BatchSolver(qp, k_max=50)
    ric = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024, boxes=False), k_max=1)
    ric2 = BatchSolver(make_shard(50, 8, 3, 0, 1, 1024, boxes=False), k_max=1)
    Q = sol.queue(8 * 1024, 8192)
    drained = 0
    for _ in range(2):
        Q.run()
        torch.cuda.synchronize()
        drained += Q.drained()[0]
    for _ in range(2):
        ric.ric_sv()
    for _ in range(2):
        ric2.ric_sv()
    torch.cuda.synchronize()
    kk = int(Q.kk.sum().item())
    print("kk_sum", kk)
    print("kk_pass", kk - drained // 2)
    if "--no-pcond" not in sys.argv:
        from hpmpc_amd.ocp import mass_spring_qp
        from hpmpc_amd.pcond import PcondSolver

        pc = PcondSolver(mass_spring_qp(200, 24, 6, boxes=False, batch=512, time_variant=True, seed=4), 20)
        for _ in range(2):
            pc.solve()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
