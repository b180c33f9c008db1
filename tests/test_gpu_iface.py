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
