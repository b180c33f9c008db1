"""Run tools/ldpat_ubench.hip: cycles per 16-load iteration by address pattern, for one wave and for a full grid
(1024 / 2048 waves, each over its own 40 KB region, so HBM traffic and contention are like the stage kernels').

Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ldpat_ubench.hip -o hpmpc_amd/lib/libldpat_ubench.so
"""
import ctypes as C
import os
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "hpmpc_amd", "lib", "libldpat_ubench.so"))
L.ldpat_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_longlong, C.c_void_p]
stride = 640 * 8  # doubles per wave: 8 rotating 5 KB blocks
names = ["contiguous b64", "lib4 tile b64 (RSQrq)", "lib4 trans b64 (BAbt)", "contiguous b128"]
st = torch.cuda.current_stream().cuda_stream
for grid in (1, 1024, 2048):
    buf = torch.rand(grid * stride + 4096, dtype=torch.float64, device="cuda")
    out = torch.zeros(grid * 64, dtype=torch.float64, device="cuda")
    cyc = torch.zeros(1, dtype=torch.int64, device="cuda")
    for p in range(4):
        iters = 200
        for _ in range(2):
            L.ldpat_run(buf.data_ptr(), out.data_ptr(), cyc.data_ptr(), p, iters, grid, stride, st)
        torch.cuda.synchronize()
        t = time.perf_counter()
        L.ldpat_run(buf.data_ptr(), out.data_ptr(), cyc.data_ptr(), p, iters, grid, stride, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        c = int(cyc.item())
        print(f"grid {grid:5d}  {names[p]:24s} {c / iters:8.1f} cyc/iter (wave 0)   wall {dt * 1e6 / iters:7.2f} us/iter")
