"""Achievable HBM bandwidth with the solver kernels' own access pattern (and, beside it, 16-B loads and several loads in
flight per thread: what a wider stage fetch could reach) (8-B raw buffer loads / stores per lane, 512 B
per wave instruction, tools/hbm_calib.hip): 1 GiB copy (read + write) and 1 GiB read, far beyond the 256 MiB
Infinity Cache.  The reference point for the measured traffic of the pass kernels (profiles/pmc_hk_ipm.json)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

cal = C.CDLL(os.path.join(ROOT, "hpmpc_amd", "lib", "libhbm_calib.so"))
for f in (cal.calib_run, cal.calib_read_run):
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
n = (1 << 30) // 8
x = torch.rand(n, dtype=torch.float64, device="cuda")
y = torch.empty(n, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
out = {}
for name, fn, nbytes in (("copy", cal.calib_run, 2 * n * 8), ("read", cal.calib_read_run, n * 8)):
    fn(x.data_ptr(), y.data_ptr(), n, C.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        assert fn(x.data_ptr(), y.data_ptr(), n, C.c_void_p(s.cuda_stream)) == 0
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    out[name] = {"ms": ms, "GBps": nbytes / ms / 1e6}
# load width and loads in flight per thread (hbm_calib.hip probe_run): 8-B vs 16-B raw buffer ops per lane, one or
# four independent loads per thread and iteration, over the same 1 GiB (y holds one partial sum per thread)
cal.probe_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_void_p]
names = ["read8_u1", "read8_u4", "read16_u1", "read16_u4", "copy8_u4", "copy16_u4"]
for grid in (2048, 8192):
    for w, name in enumerate(names):
        nbytes = (2 if name.startswith("copy") else 1) * n * 8
        assert cal.probe_run(w, x.data_ptr(), y.data_ptr(), n, grid, C.c_void_p(s.cuda_stream)) == 0
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            cal.probe_run(w, x.data_ptr(), y.data_ptr(), n, grid, C.c_void_p(s.cuda_stream))
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = float(np.median(ts))
        out[f"{name}_grid{grid}"] = {"ms": ms, "GBps": nbytes / ms / 1e6}
print(json.dumps(out))
