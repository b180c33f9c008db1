"""How often the P form's clamp certificate fails (hk_riccati.h cert_ok) on the benchmark workload: the headline
queue (N=100 nx=12 nu=4, 1024 problems, the IPM end game included) and the Riccati sv, through the diagnostic build
(libhpmpc_mi355x_stamps.so, HK_STAMPS counters: P-form stages tested / failed at the build's allowance 1e-11 and at
1e-12, 1e-13; backward sweeps and the sweeps with at least one failed stage).  Run with HPMPC_MI355X_LIB pointing
at the stamps build.  The coupled workload (hpmpc_amd.shard.coupled_shard: stage Hessians that are not diagonally
dominant) measures the shifted-Cholesky bound (hk_riccati.h cert_g_shift).  The counters live in the one-wave
kernels: the Riccati legs run with HPMPC_MI355X_RIC_WAVES=1."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import LIBPATH, BatchSolver  # noqa: E402
from hpmpc_amd.shard import coupled_shard, make_shard  # noqa: E402

lib = C.CDLL(LIBPATH)
f = lib.hpmpc_mi355x_diag_xfac
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 6)()


def stat(reset=True):
    torch.cuda.synchronize()
    assert f(buf, 1 if reset else 0) == 0
    return [int(x) for x in buf]


os.environ["HPMPC_MI355X_RIC_WAVES"] = "1"
out = {}
stat()
for name, gen in (("", make_shard), ("coupled_", coupled_shard)):
    qp = gen(100, 12, 4, 0, 1, 1024)
    s = BatchSolver(qp, k_max=50)
    Q = s.queue(4 * 1024, 2048)
    Q.run()
    st = stat()
    out[name + "ipm_queue_4x1024"] = {"stages": st[0], "fail_1e-11": st[1], "fail_1e-12": st[2], "fail_1e-13": st[3],
                                      "sweeps": st[4], "sweeps_with_fail": st[5], "sum_kk": int(Q.kk.sum().item()),
                                      "fail_frac": st[1] / max(st[0], 1)}
    del Q, s
    qr = gen(100, 12, 4, 0, 1, 1024, boxes=False)
    r = BatchSolver(qr, k_max=1)
    r.ric_sv()
    st = stat()
    out[name + "riccati_sv_1024"] = {"stages": st[0], "fail_1e-11": st[1], "fail_1e-12": st[2], "fail_1e-13": st[3],
                                     "sweeps": st[4], "sweeps_with_fail": st[5], "fail_frac": st[1] / max(st[0], 1)}
print(json.dumps(out))
