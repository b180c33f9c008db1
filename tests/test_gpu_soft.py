"""Soft-constraint IPM d_ip2_mpc_soft_tv on the HIP path against the oracle.

The reference's own outputs pin the oracle (tests/golden/soft_*.npz, run through test_gpu_parity.py as well);
these cases add sizes and options the goldens do not cover: warm start, iteration caps, time-variant data,
non-uniform soft sets, and the configurations the product rejects.  Tolerance TOL_SOFT (tests/helpers.py):
the end game of these problems is rounding-sensitive (the reference's own FMA build drifts from its default
build by the same amounts), so the cases stop at mu_tol >= 1e-6.
"""
import numpy as np
import pytest

from helpers import TOL_SOFT
from hpmpc_amd.soft import mass_spring_soft

pytestmark = pytest.mark.gpu
EUNSUPPORTED = -10


def _cmp(sq, a, b):
    assert a["ret"] == b["ret"] and a["kk"] == b["kk"], (a["ret"], a["kk"], b["ret"], b["kk"])
    N = sq.N
    if a["kk"]:
        e = np.max(np.abs(a["stat"] - b["stat"]) / np.maximum(1.0, np.abs(b["stat"])))
        assert e <= TOL_SOFT["stat"], e
    for k in range(N + 1):
        n = sq.nux(k)
        e = np.max(np.abs(a["ux"][k][:n] - b["ux"][k][:n]) / np.maximum(1.0, np.abs(b["ux"][k][:n])))
        assert e <= TOL_SOFT["ux"], (k, e)
        if k < N:
            m = int(sq.nx[k + 1])
            e = np.max(np.abs(a["pi"][k][:m] - b["pi"][k][:m]) / np.maximum(1.0, np.abs(b["pi"][k][:m])),
                       initial=0.0)
            assert e <= TOL_SOFT["pi"], (k, e)
        nb, ns = int(sq.nb[k]), int(sq.ns[k])
        pnb, pns = (nb + 3) // 4 * 4, (ns + 3) // 4 * 4
        idx = np.concatenate([np.arange(nb), np.arange(pnb, pnb + nb)] +
                             [np.arange(2 * pnb + s * pns, 2 * pnb + s * pns + ns) for s in range(4)]).astype(int)
        for key in ("lam", "t"):
            if idx.size:
                g, r = a[key][k][idx], b[key][k][idx]
                e = np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r)))
                assert e <= TOL_SOFT[key], (key, k, e)


CASES = [
    ("ms_N30_nx8_nu2", dict(N=30, nx=8, nu=2), dict(mu_tol=1e-5)),
    ("tv_N20_nx12_nu3", dict(N=20, nx=12, nu=3, time_variant=True, seed=3, Q_diag=1.0, Zq=2.0, zl=5.0),
     dict(mu_tol=1e-6)),
    ("kmax6_N25_nx4_nu2", dict(N=25, nx=4, nu=2, Q_diag=0.5), dict(k_max=6, mu_tol=1e-6)),
    ("hardN_N16_nx12_nu4", dict(N=16, nx=12, nu=4, hard_last=6, Q_diag=1.0), dict(mu_tol=1e-6)),
    ("N1_nx4_nu2", dict(N=1, nx=4, nu=2, Q_diag=1.0), dict(mu_tol=1e-6)),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_soft_vs_oracle(product, oracle, case):
    _, mk, kw = case
    sq = mass_spring_soft(**mk)
    args = dict(k_max=50, mu0=100.0, mu_tol=1e-8, alpha_min=1e-8)
    args.update(kw)
    _cmp(sq, product.ipm_soft(sq.copy(), **args), oracle.ipm_soft(sq.copy(), **args))


def test_soft_warm_start(product, oracle):
    sq = mass_spring_soft(12, 8, 3, Q_diag=1.0, Zq=1.0)
    rng = np.random.default_rng(4)
    ux0 = [0.05 * rng.standard_normal(sq.nux(k) + 4) for k in range(sq.N + 1)]
    args = dict(k_max=50, mu0=50.0, mu_tol=1e-6, alpha_min=1e-8, warm_start=1, ux=ux0)
    _cmp(sq, product.ipm_soft(sq.copy(), **args), oracle.ipm_soft(sq.copy(), **args))


def test_soft_rejects_unsupported(product):
    """ng > 0, and nx = 6 (the reference reads b_k past BAbt_k with its stride round_up(nx, 4))."""
    sq = mass_spring_soft(6, 6, 2)
    assert product.ipm_soft(sq.copy(), k_max=10)["ret"] == EUNSUPPORTED
    sq = mass_spring_soft(6, 8, 2)
    sq.ng = sq.ng.copy()
    sq.ng[3] = 1
    assert product.ipm_soft(sq.copy(), k_max=10)["ret"] == EUNSUPPORTED


SOFT_RES = [
    # (N, nx, nu, kwargs of mass_spring_soft)
    (15, 20, 4, dict(Q_diag=1.0, Zq=0.3)),          # wide stages (nu + nx > 16)
    (6, 4, 1, dict(hard_last=1, time_variant=True)),  # hard boxes at stage N (the soft index reads them)
    (9, 12, 4, dict(soft=False, Q_diag=0.5)),        # hard boxes only
]


@pytest.mark.parametrize("N,nx,nu,kw", SOFT_RES, ids=[f"N{c[0]}_nx{c[1]}_nu{c[2]}" for c in SOFT_RES])
def test_soft_residuals_vs_oracle(product, oracle, N, nx, nu, kw):
    """d_res_mpc_soft_tv (hk_soft_res) against the oracle at random iterates, beyond the soft_res goldens."""
    from helpers import check_soft_res
    from hpmpc_amd.golden import Case

    sq = mass_spring_soft(N, nx, nu, **kw)
    rng = np.random.default_rng(N * nx)
    ux, pi, lam, t = sq.alloc_solution()
    for k in range(N + 1):
        ux[k][:sq.nux(k)] = rng.standard_normal(sq.nux(k))
        lam[k][:sq.ncv(k)] = 0.1 + rng.random(sq.ncv(k))
        t[k][:sq.ncv(k)] = 0.1 + rng.random(sq.ncv(k))
        if k < N:
            pi[k][:nx] = rng.standard_normal(nx)
    q = [np.concatenate([rng.standard_normal(sq.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ref = oracle.residuals_soft(sq.copy(), q, ux, pi, lam, t)
    got = product.residuals_soft(sq.copy(), q, ux, pi, lam, t)
    like = Case.__new__(Case)
    like.name, like.qp, like.out = f"softres_N{N}_nx{nx}", sq, ref
    like.inp = dict(ns=[sq.ns.astype(np.float64)], Z=sq.Z, z=sq.z)
    check_soft_res(like, got)
