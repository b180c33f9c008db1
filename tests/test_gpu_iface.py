"""The include/c_interface.h wrappers on the HIP path.

The goldens (iface_*, run through test_gpu_parity.py) pin the column-major wrapper against the restatement
oracle/iface_oracle.py over the reference's own low-level entry points.  These cases add the row-major
twin, random problems against the restatement over the oracle, warm start, the KKT re-solve in both orders, and
the partially condensed path whose condensed stages exceed the narrow tile (solved by the wide-stage IPM).
Tolerances as the IPM goldens: ux/pi/lam 1e-10 with identical kk; residual norms 1e-9 absolute.
"""
import os
import sys

import numpy as np
import pytest

from helpers import TOL_IPM

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import iface_oracle as IO  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = [
    # N, nx, nu, nb_u, nb_x, ng, N2
    (10, [0] + [4] * 10, [2] * 10, 2, 2, None, 10),
    (12, [0] + [4] * 12, [1] * 12, 1, 2, None, 4),
    (9, [3] * 10, [2] * 9, 1, 1, [0] * 9 + [2], 9),
    (20, [0] + [12] * 20, [4] * 20, 4, 6, None, 20),
]


def _cmp(a, b, keys=("u", "x", "pi", "lam")):
    for key in keys:
        for k, (g, r) in enumerate(zip(a[key], b[key])):
            g, r = np.asarray(g), np.asarray(r)
            if r.size:
                e = float(np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r))))
                assert e <= TOL_IPM, (key, k, e)
    np.testing.assert_allclose(a["inf_norm_res"], b["inf_norm_res"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_N2_{c[6]}" for c in CASES])
def test_ip_ocp_both_orders_vs_oracle(product, oracle, case):
    N, nx, nu, bu, bx, ng, N2 = case
    P = IO.random_iface_problem(N, nx, nu, bu, bx, ng, seed=N + 100)
    ref = IO.ip_ocp(oracle, P, N2, mu_tol=1e-10)
    for order in ("F", "C"):
        got = product.ip_ocp(P, N2, order=order, mu_tol=1e-10)
        assert (got["status"], got["kk"]) == (ref["status"], ref["kk"]), order
        _cmp(got, ref)


def test_ip_ocp_warm_start_and_auto_mu0(product, oracle):
    P = IO.random_iface_problem(15, [0] + [6] * 15, [3] * 15, 3, 3, None, seed=8)
    cold = IO.ip_ocp(oracle, P, 15, mu0=-1.0, mu_tol=1e-10)
    got = product.ip_ocp(P, 15, mu0=-1.0, mu_tol=1e-10)
    assert got["kk"] == cold["kk"]
    _cmp(got, cold)
    warm = dict(u=[0.9 * v for v in cold["u"]], x=[0.9 * v for v in cold["x"]])
    a = product.ip_ocp(P, 15, mu_tol=1e-10, warm=warm)
    b = IO.ip_ocp(oracle, P, 15, mu_tol=1e-10, warm=warm)
    assert (a["status"], a["kk"]) == (b["status"], b["kk"])
    _cmp(a, b)


@pytest.mark.parametrize("order", ["F", "C"])
def test_kkt_new_rhs_wrapper(product, oracle, order):
    P = IO.random_iface_problem(10, [0] + [4] * 10, [2] * 10, 2, 2, None, seed=5)
    P2 = IO.new_rhs(P, seed=6)
    r = product.ip_ocp(P, 10, order=order, mu_tol=1e-10)
    got = product.kkt_ocp(P2, r["work0"], order=order)
    _cmp(got, IO.kkt_ocp(oracle, P, P2, mu_tol=1e-10))


@pytest.mark.parametrize("case", [(10, [0] + [8] * 10, [4] * 10, 2, 2, None, 2),
                                  (40, [0] + [12] * 40, [4] * 40, 4, 6, None, 4),
                                  (30, [0] + [24] * 30, [6] * 30, 3, 5, None, 3)],
                         ids=["N10_N2_2", "N40_N2_4", "N30_nx24_nu6_N2_3"])
def test_condensed_ipm_beyond_the_tile(product, oracle, case):
    """N2 < N with condensed stages wider than the narrow tile (nu2 + nx2 = 5*4 + 8 .. 10*6 + 24): the wrapper
    condenses (inner state boxes become general constraints), runs the wide-stage IPM (hk_wide_ipm) on the
    condensed problem and expands, in both orders, against the restatement over the oracle."""
    N, nx, nu, bu, bx, ng, N2 = case
    P = IO.random_iface_problem(N, nx, nu, bu, bx, ng, seed=N + 7)
    ref = IO.ip_ocp(oracle, P, N2, mu_tol=1e-10)
    assert ref["status"] == 0
    for order in ("F", "C"):
        got = product.ip_ocp(P, N2, order=order, mu_tol=1e-10)
        assert (got["status"], got["kk"]) == (ref["status"], ref["kk"]), order
        _cmp(got, ref)


# ---------------------------------------------------------------------------- legacy uniform-size wrappers
# fortran_order_d_ip_mpc_hard_tv / c_order_ twin and their KKT re-solves (include/c_interface.h:45-53): the goldens
# (iface_mpc_*, through test_gpu_parity.py) pin the column-major wrapper; these add the row-major twin on the same
# goldens and random problems against oracle/iface_oracle.py ip_mpc / kkt_mpc over the CPU oracle.
MPC_CASES = [  # N, nx, nu, nb, ng, ngN, time_invariant, seed
    (10, 4, 2, 6, 0, 0, 0, 310),
    (12, 3, 2, 4, 2, 1, 1, 301),
    (20, 12, 4, 10, 0, 0, 0, 320),
    (8, 5, 2, 5, 2, 2, 1, 308),
]


def _cmp_mpc(a, b):
    for key in ("u", "x", "pi", "lam", "t"):
        g, r = np.asarray(a[key]), np.asarray(b[key])
        e = float(np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r)))) if r.size else 0.0
        assert e <= TOL_IPM, (key, e)
    np.testing.assert_allclose(a["inf_norm_res"], b["inf_norm_res"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("case", MPC_CASES, ids=[f"N{c[0]}_nx{c[1]}_ti{c[6]}" for c in MPC_CASES])
def test_ip_mpc_both_orders_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng, ngN, ti, seed = case
    M = IO.random_mpc_problem(N, nx, nu, nb, ng, ngN, ti, seed=seed)
    ref = IO.ip_mpc(oracle, M, mu_tol=1e-8)
    assert ref["status"] == 0
    for order in ("F", "C"):
        got = product.ip_mpc(M, order=order, mu_tol=1e-8)
        assert (got["status"], got["kk"]) == (ref["status"], ref["kk"]), order
        _cmp_mpc(got, ref)


def test_ip_mpc_input_equality_quirk(product, oracle):
    """An input with lb == ub: the wrapper folds it into b, zeroes its B column and gives the box the bounds
    [lb + 1e3, ub - 1e3] (fortran_order_interface.c:2695-2705), which this IPM's [lb | ub] convention reads as an
    empty box -- the reference's own wrapper diverges (ret 2, mu ~1e16).  Held here: the same status and iteration
    count as the restatement, u / x to the IPM gate, u[1] = lb on every stage (the wrapper's equality fix)."""
    M = IO.random_mpc_problem(10, 4, 2, 6, 0, 0, 0, seed=310, eq=(1,))
    ref = IO.ip_mpc(oracle, M, mu_tol=1e-8)
    got = product.ip_mpc(M, mu_tol=1e-8)
    assert (got["status"], got["kk"]) == (ref["status"], ref["kk"])
    for key in ("u", "x"):
        e = float(np.max(np.abs(got[key] - ref[key]) / np.maximum(1.0, np.abs(ref[key]))))
        assert e <= 1e-10, (key, e)
    np.testing.assert_array_equal(got["u"][1::2], M["lb"][1:60:6])


@pytest.mark.parametrize("order", ["F", "C"])
def test_kkt_mpc_both_orders_vs_oracle(product, oracle, order):
    M = IO.random_mpc_problem(12, 3, 2, 4, 2, 1, 0, seed=303)
    M2 = IO.mpc_new_rhs(M, seed=403)
    ref = IO.kkt_mpc(oracle, M, M2, mu_tol=1e-8, order=order)
    r = product.ip_mpc(M, order=order, mu_tol=1e-8)
    got = product.kkt_mpc(M2, r["work0"], order=order)
    for key in ("u", "x", "pi", "lam", "t"):  # a Newton system at complementarity mu: the KKT gate
        e = float(np.max(np.abs(got[key] - ref[key]) / np.maximum(1.0, np.abs(ref[key]))))
        assert e <= 1e-8, (key, e)
    np.testing.assert_allclose(got["inf_norm_res"], ref["inf_norm_res"], rtol=0, atol=1e-8)


def test_ip_mpc_goldens_row_major(product):
    """The row-major twins on the column-major goldens (same problems, each stage block transposed in memory)."""
    from hpmpc_amd.golden import load_all
    from helpers import check_iface, run_iface_mpc

    cases = load_all("iface_mpc")
    assert len(cases) >= 7
    for c in cases:
        check_iface(c, run_iface_mpc(product, c, order="C"))


def test_kkt_wrapper_refuses_after_failed_ipm():
    """the wrapper tags work0 as holding an IPM factor only after a successful solve.  In the diagnostic
    build (libhpmpc_mi355x_stamps.so) with HPMPC_MI355X_MW_FAULT=1 the multi-wave IPM kernel drops a hand-over and the
    solve returns -20 (HPMPC_MI355X_EMW) without copying anything out; the KKT re-solve on that work0 must then refuse
    (HPMPC_MI355X_EUNSUPPORTED) and leave its outputs untouched.  A child process (the library is chosen at import)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "hpmpc_amd", "lib", "libhpmpc_mi355x_stamps.so")
    assert os.path.exists(lib), "diagnostic build missing (hpmpc_amd/build.py build_stamps, run by build())"
    code = r"""
import sys, numpy as np
sys.path.insert(0, "oracle")
import iface_oracle as IO
from hpmpc_amd.batch import LIBPATH
from hpmpc_amd.cabi import HpmpcAPI, load
api = HpmpcAPI(load(LIBPATH))
P = IO.random_iface_problem(10, [0] + [4] * 10, [2] * 10, 2, 2, None, seed=5)
r = api.ip_ocp(P, 10, mu_tol=1e-10)
assert r["status"] == -20, r["status"]
got = api.kkt_ocp(IO.new_rhs(P, seed=6), r["work0"])
assert api.lib.hpmpc_mi355x_last_error() == -10, api.lib.hpmpc_mi355x_last_error()
assert all(not np.any(v) for key in ("u", "x", "pi", "lam") for v in got[key])
print("refused")
"""
    env = dict(os.environ, HPMPC_MI355X_LIB=lib, HPMPC_MI355X_MW_FAULT="1", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0 and "refused" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
