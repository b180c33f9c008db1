"""The alternate IPM of mpc_solvers/d_ip2_hard.c on the HIP path against the oracle.

d_ip2_mpc_hard_tv (d_ip2_hard.c:88) is the phase-1 Mehrotra loop run to mu_tol, d_kkt_solve_new_rhs_mpc_hard_tv
(:626) its KKT re-solve and d_res_mpc_hard_tv (mpc_solvers/d_res_ip_hard.c:38) the plain residuals.  The
reference's own pins are the ipm2/kkt2/res2 goldens (test_gpu_parity.py); these cases add varying stage sizes,
arbitrary box subsets and dense general constraints.  Tolerances (tests/helpers.py TOL_KKT2): without the residual
correction the last Newton systems carry Hessian terms lam/t ~ 1/mu_tol, so a different (MFMA) summation order
moves ux/pi/t by up to eps / mu_tol (measured at mu_tol 1e-8, N=20 nx=12 nu=4 nb=10: ux 6e-10, the KKT re-solve's
pi 6e-8).  These cases run to mu_tol 1e-6 and hold ux/pi/t to 1e-8, lam to 1e-4.
"""
import numpy as np
import pytest

from helpers import TOL_KKT2, TOL_RIC, random_qp

pytestmark = pytest.mark.gpu

CASES = [
    # N, nx, nu, nb, ng
    (8, [0] + [6] * 8, [2] * 8 + [0], [1] + [3] * 7 + [3], None),
    (7, [0, 3, 5, 5, 2, 7, 12, 9], [2, 4, 1, 3, 6, 4, 4, 0], [1, 3, 2, 0, 4, 5, 6, 3], None),
    (20, [0] + [12] * 20, [4] * 20 + [0], [4] + [10] * 19 + [6], None),
    (10, [0] + [8] * 10, [3] * 10 + [0], [2] + [3] * 9 + [4], [0] + [2] * 9 + [8]),
    (5, [0, 6, 9, 9, 5, 7], [3, 2, 4, 1, 3, 0], [0, 4, 2, 3, 0, 2], [3, 0, 5, 2, 7, 4]),
]


def _valid(qp, key, k):
    if key == "ux":
        return np.arange(qp.nux(k))
    if key == "pi":
        return np.arange(int(qp.nx[k + 1]))
    nb, pnb, ng, png = int(qp.nb[k]), qp.pnb(k), int(qp.ng[k]), qp.png(k)
    return np.r_[0:nb, pnb:pnb + nb, 2 * pnb:2 * pnb + ng, 2 * pnb + png:2 * pnb + png + ng].astype(int)


def _cmp(qp, a, b, tols):
    for key, tol in tols.items():
        if key == "stat":
            continue
        n = qp.N if key == "pi" else qp.N + 1
        e = 0.0
        for k in range(n):
            i = _valid(qp, key, k)
            if i.size:
                e = max(e, float(np.max(np.abs(a[key][k][i] - b[key][k][i]) / np.maximum(1.0, np.abs(b[key][k][i])))))
        assert e <= tol, (key, e, tol)


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_ipm2_kkt2_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=13 * N + 5, ng=ng)
    kw = dict(k_max=40, mu_tol=1e-6, res=False)
    a = product.ipm(qp.copy(), **kw)
    b = oracle.ipm(qp.copy(), **kw)
    assert (a["kk"], a["ret"]) == (b["kk"], b["ret"])
    _cmp(qp, a, b, TOL_KKT2)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-5, atol=1e-12)
    # re-solve with new b, q and bounds on the factor the IPM left in its workspace
    rng = np.random.default_rng(N)
    b2 = [np.concatenate([0.1 * rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    q2 = [np.concatenate([0.1 * rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    d2 = [x * (1.0 + 0.05 * rng.random(x.shape)) for x in qp.d]
    ka = product.kkt_new_rhs_plain(qp.copy(), a["work"], b2, q2, d2, a["ux"])
    kb = oracle.kkt_new_rhs_plain(qp.copy(), b["work"], b2, q2, d2, b["ux"])
    _cmp(qp, ka, kb, TOL_KKT2)


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_res_plain_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=3 * N + 2, ng=ng)
    rng = np.random.default_rng(7 + N)
    b = [rng.standard_normal(int(qp.nx[k + 1]) + 8) for k in range(N)]
    q = [rng.standard_normal(qp.nux(k) + 8) for k in range(N + 1)]
    ux = [rng.standard_normal(qp.nux(k) + 8) for k in range(N + 1)]
    pi = [rng.standard_normal(int(qp.nx[k + 1]) + 8) for k in range(N)]
    lam = [rng.random(qp.d[k].size) + 0.1 for k in range(N + 1)]
    t = [rng.random(qp.d[k].size) + 0.1 for k in range(N + 1)]
    ra = product.residuals_plain(qp, b, q, ux, pi, lam, t)
    rb = oracle.residuals_plain(qp, b, q, ux, pi, lam, t)
    assert abs(ra["mu"] - rb["mu"]) <= TOL_RIC * max(1.0, abs(rb["mu"]))
    for key, n, ln in (("rq", N + 1, qp.nux), ("rb", N, lambda k: int(qp.nx[k + 1]))):
        for k in range(n):
            m = ln(k)
            np.testing.assert_allclose(ra[key][k][:m], rb[key][k][:m], rtol=TOL_RIC, atol=TOL_RIC)
    for k in range(N + 1):
        i = _valid(qp, "rd", k)
        np.testing.assert_allclose(ra["rd"][k][i], rb["rd"][k][i], rtol=TOL_RIC, atol=TOL_RIC)


def test_ipm2_unconstrained_leaves_iterate(product, oracle):
    """Without constraints d_ip2_mpc_hard_tv runs one sv into its workspace and returns kk = 0 with the
    caller's ux untouched (d_ip2_hard.c:282-291); the KKT re-solve then solves on that factor."""
    qp = random_qp(12, [0] + [8] * 12, [3] * 12 + [0], seed=3)
    a = product.ipm(qp.copy(), k_max=10, res=False)
    b = oracle.ipm(qp.copy(), k_max=10, res=False)
    assert a["kk"] == b["kk"] == 0 and a["ret"] == b["ret"] == 0
    for k in range(13):
        assert not np.any(a["ux"][k])
    rng = np.random.default_rng(1)
    b2 = [rng.standard_normal(16) for _ in range(12)]
    q2 = [rng.standard_normal(16) for _ in range(13)]
    d2 = [x.copy() for x in qp.d]
    ka = product.kkt_new_rhs_plain(qp.copy(), a["work"], b2, q2, d2, a["ux"])
    kb = oracle.kkt_new_rhs_plain(qp.copy(), b["work"], b2, q2, d2, b["ux"])
    _cmp(qp, ka, kb, dict(ux=TOL_RIC * 10, pi=TOL_RIC * 10))
