"""CPU-side checks of the drop-in boundary and the host logic (no GPU compute is launched here).

* libhpmpc_mi355x.so loads and exports every function include/hpmpc_mi355x.h declares;
* the reference-named entry points reject what the GPU path does not support with the documented
  error code before touching the device (ng > 0, stages wider than the 16-wide tile);
* lib4 packing helpers, the synthetic workload generator and the roofline byte/flop formulas.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from hpmpc_amd import batch
from hpmpc_amd.ocp import (OCPQP, batch_x0, default_x0, lib4_size, mass_spring_qp, pack_lib4, pack_lib4_batch,
                           unpack_lib4)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hpmpc_mi355x.h")
EUNSUPPORTED = -10


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n not in ("defined",)))


@pytest.fixture(scope="module")
def hiplib():
    if not os.path.exists(batch.LIBPATH):
        from hpmpc_amd.build import build_hip

        build_hip()
    return C.CDLL(batch.LIBPATH, mode=os.RTLD_LOCAL)


def test_header_declares_reference_entry_points():
    names = header_functions()
    for ref in ("d_back_ric_rec_sv_tv_res", "d_back_ric_rec_trf_tv_res", "d_back_ric_rec_trs_tv_res",
                "d_back_ric_rec_sv_tv_work_space_size_bytes", "d_back_ric_rec_sv_tv_memory_space_size_bytes",
                "d_ip2_res_mpc_hard_tv", "d_ip2_res_mpc_hard_tv_work_space_size_bytes",
                "d_ip2_res_mpc_hard_tv_single_newton_step", "d_kkt_solve_new_rhs_res_mpc_hard_tv",
                "d_res_res_mpc_hard_tv", "d_ip2_mpc_hard_tv", "d_kkt_solve_new_rhs_mpc_hard_tv", "d_res_mpc_hard_tv",
                "d_part_cond", "d_part_cond_compute_problem_size", "d_part_cond_memory_space_size_bytes",
                "d_part_expand_solution", "fortran_order_d_ip_ocp_hard_tv", "c_order_d_ip_ocp_hard_tv",
                "hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes", "fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv",
                "c_order_d_solve_kkt_new_rhs_ocp_hard_tv"):
        assert ref in names, ref
    assert len(names) >= 19, names


def test_library_exports_every_declared_symbol(hiplib):
    missing = [n for n in header_functions() if not hasattr(hiplib, n)]
    assert not missing, missing


def test_library_exports_nothing_else(hiplib):
    """A shim linked beside the reference archive must not leak internal symbols into the caller's namespace:
    the dynamic symbol table is exactly the header's functions (build: -fvisibility=hidden + exports.map)."""
    import shutil
    import subprocess

    if shutil.which("nm") is None:
        pytest.skip("nm not available")
    out = subprocess.run(["nm", "-D", "--defined-only", batch.LIBPATH], check=True, capture_output=True,
                         text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if len(ln.split()) >= 3}
    assert exported == set(header_functions()), sorted(exported ^ set(header_functions()))


def test_every_reference_citation_resolves():
    """Each prototype cites the reference declaration it replaces; the cited headers exist in the
    reference layout (checked by name only: the reference tree is not needed at run time)."""
    text = open(HEADER).read()
    cites = re.findall(r"/\* (include/\w+\.h):(\d+)", text)
    assert len(cites) >= 10
    assert {c[0] for c in cites} <= {"include/lqcp_solvers.h", "include/mpc_solvers.h", "include/c_interface.h"}


def test_version_string(hiplib):
    hiplib.hpmpc_mi355x_version.restype = C.c_char_p
    assert b"gfx950" in hiplib.hpmpc_mi355x_version()


def _sizes(qp):
    iv = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    return iv(qp.nx), iv(qp.nu), iv(qp.nb), iv(qp.ng)


def test_plan_rejects_unsupported_sizes(hiplib):
    L = hiplib
    L.hpmpc_mi355x_plan_create.restype = C.c_void_p
    L.hpmpc_mi355x_plan_create.argtypes = [C.c_int] + [C.c_void_p] * 5
    for nx, nu in ((20, 4), (12, 8), (13, 4)):  # nu+nx > 16 or round_up(nu,4)+nx > 16
        N = 3
        nxv = np.array([0] + [nx] * N, dtype=np.int32)
        nuv = np.array([nu] * N + [0], dtype=np.int32)
        z = np.zeros(N + 1, dtype=np.int32)
        idx = (C.POINTER(C.c_int) * (N + 1))()
        p = L.hpmpc_mi355x_plan_create(N, nxv.ctypes.data, nuv.ctypes.data, z.ctypes.data, C.cast(idx, C.c_void_p),
                                       z.ctypes.data)
        assert not p
        assert L.hpmpc_mi355x_last_error() == EUNSUPPORTED


def test_plan_rejects_too_many_constraints(hiplib):
    """Box and general constraints share one 32-slot vector per stage: round_up(nb,4) + round_up(ng,4)
    <= 16, checked on the host before any device allocation."""
    L = hiplib
    L.hpmpc_mi355x_plan_create.restype = C.c_void_p
    L.hpmpc_mi355x_plan_create.argtypes = [C.c_int] + [C.c_void_p] * 5
    N = 3
    nxv = np.array([0] + [12] * N, dtype=np.int32)
    nuv = np.array([4] * N + [0], dtype=np.int32)
    nbv = np.array([4, 10, 10, 6], dtype=np.int32)
    ngv = np.array([0, 0, 8, 0], dtype=np.int32)  # stage 2: 12 + 8 > 16
    idx_arrs = [np.arange(n, dtype=np.int32) for n in nbv]
    idx = (C.POINTER(C.c_int) * (N + 1))(*[a.ctypes.data_as(C.POINTER(C.c_int)) for a in idx_arrs])
    p = L.hpmpc_mi355x_plan_create(N, nxv.ctypes.data, nuv.ctypes.data, nbv.ctypes.data, C.cast(idx, C.c_void_p),
                                   ngv.ctypes.data)
    assert not p
    assert L.hpmpc_mi355x_last_error() == EUNSUPPORTED


def test_size_queries_are_host_only(hiplib):
    from hpmpc_amd.cabi import HpmpcAPI

    api = HpmpcAPI(hiplib, "")
    qp = mass_spring_qp(100, 12, 4)
    ws = api.ipm_ws_size(qp)
    assert ws % 64 == 0 and ws >= 8 * 101 * (352 + 9 * 16 + 8 * 32)
    w, m = api.ric_sizes(qp)
    assert m >= 8 * 101 * 352 and w >= 0


# ---------------------------------------------------------------- lib4 / workload generator
@pytest.mark.parametrize("m,n", [(1, 1), (4, 4), (5, 3), (17, 16), (13, 12), (20, 12)])
def test_lib4_roundtrip(m, n):
    rng = np.random.default_rng(m * 100 + n)
    A = rng.standard_normal((m, n))
    buf = pack_lib4(A)
    assert buf.size == lib4_size(m, n)
    np.testing.assert_array_equal(unpack_lib4(buf, m, n), A)
    # element (i,j) at (i/4)*4*sd + i%4 + 4*j  (include/block_size.h, blas_d_lib4.c:5659-5672)
    sd = (n + 1) // 2 * 2
    for i, j in ((m - 1, n - 1), (0, n - 1), (m - 1, 0)):
        assert buf[(i // 4) * 4 * sd + i % 4 + 4 * j] == A[i, j]


def test_pack_lib4_batch_matches_single():
    rng = np.random.default_rng(7)
    M = rng.standard_normal((5, 17, 12))
    B = pack_lib4_batch(M)
    for p in range(5):
        np.testing.assert_array_equal(B[p], pack_lib4(M[p]))


def test_workload_generator_shapes():
    qp = mass_spring_qp(100, 12, 4, batch=8, time_variant=True, seed=1)
    assert qp.nb.tolist() == [4] + [10] * 99 + [6]
    assert qp.nx[0] == 0 and qp.nu[100] == 0
    one = qp.problem(3)
    assert isinstance(one, OCPQP) and one.batch is None
    X0 = batch_x0(12, 8)
    np.testing.assert_array_equal(X0[0], default_x0(12))
    assert np.all(np.abs(X0[1:]) <= 2.5)


def test_roofline_formulas_match_survey():
    """flop_sv(N=100,nx=12,nu=4) = 843.5k.  Bytes are summed over the real stage
    shapes (nx[0]=0, nu[N]=0), slightly below the survey's uniform-stage 441.6 KB estimate."""
    assert abs(batch.flops_sv(100, 12, 4) - 843.5e3) < 0.5e3
    assert abs(batch.flops_sv(50, 8, 3) - 144.8e3) < 0.5e3
    qp = mass_spring_qp(100, 12, 4, boxes=False)
    b = batch.algorithmic_bytes_per_sv(qp)
    assert 0.98 * 441.6e3 < b <= 441.6e3
    qpb = mass_spring_qp(100, 12, 4)
    bi = batch.algorithmic_bytes_per_ip_iter(qpb)
    assert 0.97 * 1318e3 < bi <= 1318e3 * 1.01


def test_batch_solver_refuses_without_gpu():
    """No CPU fallback: the batched front end raises when there is no HIP device."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        batch.BatchSolver(mass_spring_qp(5, 4, 1, batch=2))


def test_noidxb_size_matches_idxb_size(hiplib):
    """hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes_noidxb (c_interface.h:60): boxes given by count (nbu inputs, nbx
    states) need the work space of any index set with those counts, full space and partially condensed (host only)."""
    N = 12
    nx = np.array([0] + [6] * N, dtype=np.int32)
    nu = np.array([2] * N + [0], dtype=np.int32)
    nbu = np.array([2] * N + [0], dtype=np.int32)
    nbx = np.array([0] + [3] * N, dtype=np.int32)
    nb = (nbu + nbx).astype(np.int32)
    ng = np.zeros(N + 1, dtype=np.int32)
    rng = np.random.default_rng(0)
    idx = []
    for k in range(N + 1):
        u = rng.permutation(int(nu[k]))[: nbu[k]] if nu[k] else np.zeros(0, int)
        x = int(nu[k]) + rng.permutation(int(nx[k]))[: nbx[k]] if nx[k] else np.zeros(0, int)
        idx.append(np.ascontiguousarray(np.r_[u, x], dtype=np.int32))
    P = C.POINTER(C.c_int)
    idxp = (P * (N + 1))(*[a.ctypes.data_as(P) for a in idx])
    f = hiplib.hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes
    g = hiplib.hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes_noidxb
    ip = lambda a: a.ctypes.data_as(P)
    for N2 in (N, 4, 3):
        a = f(N, ip(nx), ip(nu), ip(nb), idxp, ip(ng), N2)
        b = g(N, ip(nx), ip(nu), ip(nb), ip(nbx), ip(nbu), ip(ng), N2)
        assert a == b > 0, (N2, a, b)


@pytest.mark.parametrize("fill", ["zeros", "garbage"])
def test_kkt_wrapper_refuses_unwritten_work0(fill):
    """fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv on a work space no IPM wrapper has written -- what
    test_problems/test_d_ip_hard.c:892 does (its IPM call at :849 is commented out, work1 comes straight from malloc):
    an error code (HPMPC_MI355X_EUNSUPPORTED via hpmpc_mi355x_last_error) and untouched outputs, decided on the host
    before any device work."""
    import sys

    from hpmpc_amd.cabi import HpmpcAPI, load

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import iface_oracle

    P = iface_oracle.random_iface_problem(8, [4] * 9, [2] * 8, [2] * 9, [1] * 9, seed=3)
    api = HpmpcAPI(load(batch.LIBPATH))
    wsz = api.fn("hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes")(
        C.c_int(8), *(np.ascontiguousarray(P[k], dtype=np.int32).ctypes.data_as(C.POINTER(C.c_int))
                      for k in ("nx", "nu", "nb")),
        (C.POINTER(C.c_int) * 9)(*[np.ascontiguousarray(i, dtype=np.int32).ctypes.data_as(C.POINTER(C.c_int))
                                   for i in P["hidxb"]]),
        np.ascontiguousarray(P["ng"], dtype=np.int32).ctypes.data_as(C.POINTER(C.c_int)), C.c_int(8))
    work0 = np.zeros(wsz // 8 + 16)
    if fill == "garbage":
        work0[:] = np.random.default_rng(1).standard_normal(work0.size) * 1e3
    r = api.kkt_ocp(P, work0)
    assert api.lib.hpmpc_mi355x_last_error() == EUNSUPPORTED
    assert all(not np.any(x) for x in r["x"]) and all(not np.any(u) for u in r["u"])


def test_plan_rejects_horizon_beyond_lds_tables(hiplib):
    """the tile kernels keep 104 B of stage tables per stage in LDS (+ 256 B); a horizon whose tables exceed
    the 160 KiB of one workgroup is refused when the plan is created, before any device allocation (N <= 1571)."""
    L = hiplib
    L.hpmpc_mi355x_plan_create.restype = C.c_void_p
    L.hpmpc_mi355x_plan_create.argtypes = [C.c_int] + [C.c_void_p] * 5
    N = 1572
    nxv = np.array([0] + [4] * N, dtype=np.int32)
    nuv = np.array([2] * N + [0], dtype=np.int32)
    z = np.zeros(N + 1, dtype=np.int32)
    idx = (C.POINTER(C.c_int) * (N + 1))()
    p = L.hpmpc_mi355x_plan_create(N, nxv.ctypes.data, nuv.ctypes.data, z.ctypes.data, C.cast(idx, C.c_void_p),
                                   z.ctypes.data)
    assert not p
    assert L.hpmpc_mi355x_last_error() == EUNSUPPORTED
