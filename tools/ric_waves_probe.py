"""Riccati sv batches: the one-wave kernel (HPMPC_MI355X_RIC_WAVES=1) against the two-wave kernel (hk_ric2.hip),
same process, alternating, at the benchmark batches (1024 x N=100 nx=12 nu=4; configs[2] 1024 x N=50 nx=8 nu=3), a
lone problem and two batches' worth.  Prints us per launch and M fact/s per variant (median of 5 rounds of 20).

--stamps: the diagnostic build (hpmpc_amd/lib/libhpmpc_mi355x_stamps.so, -DHK_STAMPS): cycles of problem 0's sweeps
(one-wave: backward / forward; two-wave: per wave, and wave 0's backward step by segment)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS = "--stamps" in sys.argv
if STAMPS:
    os.environ["HPMPC_MI355X_LIB"] = os.environ.get("HPMPC_STAMPS_LIB") or os.path.join(
        ROOT, "hpmpc_amd", "lib", "libhpmpc_mi355x_stamps.so")
import numpy as np
import torch

from hpmpc_amd.batch import BatchSolver, lib
from hpmpc_amd.shard import make_shard


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def set_waves(w):
    os.environ["HPMPC_MI355X_RIC_WAVES"] = str(w)


CONFIGS = [(100, 12, 4, 1024), (50, 8, 3, 1024), (100, 12, 4, 1), (100, 12, 4, 2048)]
if STAMPS:
    dbg = torch.zeros(64, dtype=torch.int64, device="cuda")
    lib().hpmpc_mi355x_debug_buffer.argtypes = [C.c_void_p]
    lib().hpmpc_mi355x_debug_buffer(dbg.data_ptr())
    for (N, nx, nu, B) in CONFIGS[:3]:
        s = BatchSolver(make_shard(N, nx, nu, 0, 1, B, boxes=False), k_max=1)
        for w in (1, 2):
            set_waves(w)
            s.ric_sv(compute_pi=1)
            torch.cuda.synchronize()
            dbg.zero_()
            s.ric_sv(compute_pi=1)
            torch.cuda.synchronize()
            t = dbg.cpu().numpy()
            if w == 1:
                print(f"N={N} nx={nx} nu={nu} batch={B} 1-wave: backward {t[60]} ({t[60] / (N + 1):.0f}/stage) "
                      f"forward {t[61]} ({t[61] / N:.0f}/stage) cycles", flush=True)
            else:
                print(f"N={N} nx={nx} nu={nu} batch={B} 2-wave (cycles; work / barrier wait): backward w0 {t[0]} / "
                      f"{t[1]} ({t[0] / (N + 1):.0f} / {t[1] / (N + 1):.0f} per step), w1 {t[2]} / {t[3]}; forward w0 "
                      f"{t[4]} / {t[5]}, w1 {t[6]} / {t[7]}; w0 step: dispatch {t[8] / (N + 1):.0f} tile+cert "
                      f"{t[9] / (N + 1):.0f} chol {t[10] / (N + 1):.0f} whole {t[11] / (N + 1):.0f}", flush=True)
    os.environ.pop("HPMPC_MI355X_RIC_WAVES", None)
    sys.exit(0)

SPLIT = "--split" in sys.argv  # one-wave entry points: sv, sv without pi, trf (backward without the row), trs
if SPLIT:
    import torch as _t
    os.environ["HPMPC_MI355X_RIC_WAVES"] = "1"
    for (N, nx, nu, B) in CONFIGS[:3]:
        s = BatchSolver(make_shard(N, nx, nu, 0, 1, B, boxes=False), k_max=1)
        bb = _t.zeros((B, N + 1, 16), dtype=_t.float64, device="cuda")
        res = {n: float(np.median([timeit(f) for _ in range(3)])) for n, f in (
            ("sv", lambda: s.ric_sv(compute_pi=1)), ("sv_nopi", lambda: s.ric_sv(compute_pi=0)),
            ("trf", lambda: s.ric_trf()), ("trs", lambda: s.ric_trs(bb, bb, compute_Pb=0)))}
        print(f"N={N} nx={nx} nu={nu} batch={B} one-wave us: " + " ".join(f"{k} {v * 1e3:.1f}" for k, v in res.items()),
              flush=True)
    sys.exit(0)

for (N, nx, nu, B) in CONFIGS:
    s = BatchSolver(make_shard(N, nx, nu, 0, 1, B, boxes=False), k_max=1)
    res = {1: [], 2: []}
    for _ in range(5):
        for w in (1, 2):
            set_waves(w)
            res[w].append(timeit(lambda: s.ric_sv(compute_pi=1)))
    os.environ.pop("HPMPC_MI355X_RIC_WAVES", None)
    line = f"N={N} nx={nx} nu={nu} batch={B}:"
    for w in (1, 2):
        ms = float(np.median(res[w]))
        line += f"  {w}-wave {ms * 1e3:8.1f} us ({B / (ms * 1e-3) / 1e6:6.3f} M fact/s)"
    print(line, flush=True)
