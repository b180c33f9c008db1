"""The IPM on stages beyond the 16-wide register tile (hk_wide_ipm.hip) against the CPU oracle.

The reference pins this path through the `ipmw_*` / `kktw_*` / `resw_*` / `res2w_*` / `ipm2w_*` / `kkt2w_*` /
`newtonw_*` / `iface_condw_*` / `iface_fullw_*` goldens of tests/golden (run by test_gpu_parity.py); the cases
here add what those do not cover: varying stage sizes across the tile boundary, odd sizes, x-only boxes, dense
general constraints at every stage (more than 16 slots), N = 1, warm start, the KKT re-solves and residual
routines on random problems, a single Newton step, the alternate IPM, the unconstrained shortcut, an
infeasible problem (alpha_min exit), and the size checks of the wide path.
Tolerances as SURVEY.md §8c: IPM identical kk / ret and 1e-10 relative, Riccati-level outputs 1e-12.
"""
import numpy as np
import pytest

from helpers import TOL_IPM, TOL_KKT2, TOL_RIC, compare_ipm, random_qp

pytestmark = pytest.mark.gpu
EUNSUPPORTED = -10


def tol_cond(mu):
    """Gate for outputs of Newton systems solved at complementarity mu: their Hessian terms lam/t reach ~1/mu, so
    two correct solvers whose sums run in different orders (16x16x4 MFMA tiles here, sequential loops in the
    oracle and in the reference's 4x4 kernels) differ by up to ~eps/mu.  100 eps / mu, never below TOL_IPM."""
    return max(TOL_IPM, 100 * np.finfo(float).eps / mu)


CASES = [
    # N, nx per stage, nu per stage, nb per stage, ng per stage
    (10, [0] + [24] * 10, [6] * 10 + [0], [6] + [18] * 9 + [12], None),                      # configs[4] stage shape
    (8, [0, 14, 20, 9, 30, 17, 12, 25, 11], [5, 3, 7, 2, 6, 4, 9, 1, 0], [3, 10, 5, 11, 20, 6, 12, 4, 7], None),
    (6, [0] + [20] * 6, [4] * 6 + [0], [4] + [0] * 5 + [20], [5] + [22] * 5 + [9]),          # general > 16 slots
    (12, [0] + [8] * 12, [3] * 12 + [0], [3] + [11] * 11 + [8], [1] + [9] * 11 + [10]),     # narrow stages, many slots
    (1, [0, 40], [20, 0], [10, 30], [3, 17]),                                                 # N = 1, 60-wide stage 0
    (5, [24, 24, 24, 24, 24, 24], [6] * 5 + [0], [30] * 5 + [24], [2] * 6),                  # x0 as a variable
]


def _rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)), initial=0.0))


def _ng(case):
    return case[4]


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_wide_ipm_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=97 * N + len(nx), ng=ng)
    a = product.ipm(qp.copy(), k_max=60)
    b = oracle.ipm(qp.copy(), k_max=60)
    assert b["ret"] == 0, b["ret"]
    compare_ipm(qp, a, b, tol=TOL_IPM)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-8, atol=1e-13)
    # KKT re-solve with new right-hand sides from the persisted factor and iterate.  At the converged iterate
    # (mu ~ 1e-12) that Newton system carries lam/t ~ 1e12 and amplifies the 1e-13 differences the two IPMs'
    # summation orders leave (MFMA tiles vs sequential loops) to ~1e-3, so the re-solve is compared on the
    # iterate of a run stopped at mu_tol = 1e-6 (lam/t ~ 1e6).
    a = product.ipm(qp.copy(), k_max=60, mu_tol=1e-6)
    b = oracle.ipm(qp.copy(), k_max=60, mu_tol=1e-6)
    compare_ipm(qp, a, b, tol=TOL_IPM)
    rng = np.random.default_rng(N + 3)
    bb = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    qq = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ka = product.kkt_new_rhs(qp.copy(), a["work"], bb, qq)
    kb = oracle.kkt_new_rhs(qp.copy(), b["work"], bb, qq)
    ka.update(kk=0, ret=0)
    kb.update(kk=0, ret=0)
    compare_ipm(qp, ka, kb, tol=tol_cond(1e-6))


@pytest.mark.parametrize("case", CASES[:4], ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES[:4])])
def test_wide_residuals_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=5 * N + 1, ng=ng)
    rng = np.random.default_rng(N)
    b = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    q = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ux = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    pi = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    lam = [0.5 + rng.random(qp.nconstr(k) + 8) for k in range(N + 1)]
    t = [0.5 + rng.random(qp.nconstr(k) + 8) for k in range(N + 1)]
    for plain in (False, True):
        fa = product.residuals_plain if plain else product.residuals
        fb = oracle.residuals_plain if plain else oracle.residuals
        ra = fa(qp.copy(), b, q, ux, pi, lam, t)
        rb = fb(qp.copy(), b, q, ux, pi, lam, t)
        for k in range(N + 1):
            assert _rel(ra["rq"][k][: qp.nux(k)], rb["rq"][k][: qp.nux(k)]) <= TOL_RIC, (plain, k)
            if k < N:
                m = int(qp.nx[k + 1])
                assert _rel(ra["rb"][k][:m], rb["rb"][k][:m]) <= TOL_RIC, (plain, k)
            nbk, pnb, ngk, png = int(qp.nb[k]), qp.pnb(k), int(qp.ng[k]), qp.png(k)
            idx = np.r_[0:nbk, pnb:pnb + nbk, 2 * pnb:2 * pnb + ngk, 2 * pnb + png:2 * pnb + png + ngk].astype(int)
            assert _rel(ra["rd"][k][idx], rb["rd"][k][idx]) <= TOL_RIC, (plain, k)
            if not plain:
                assert _rel(ra["rm"][k][idx], rb["rm"][k][idx]) <= TOL_RIC, k
        assert abs(ra["mu"] - rb["mu"]) <= TOL_RIC * max(1.0, abs(rb["mu"])), plain


@pytest.mark.parametrize("case", [CASES[0], CASES[2]], ids=["box", "general"])
def test_wide_alternate_ipm_vs_oracle(product, oracle, case):
    """d_ip2_mpc_hard_tv (phase-1 loop to mu_tol) on wide stages.  Without the residual correction its last
    Newton systems carry lam/t ~ 1/mu_tol: ux / pi / t are gated by tol_cond(mu_tol), lam by TOL_KKT2's 1e-4 (the
    gate the oracle meets against the reference build on such systems).  The reference pins this routine at
    TOL_IPM2 through the ipm2w_* goldens."""
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=13 * N + 2, ng=ng)
    a = product.ipm(qp.copy(), k_max=60, mu_tol=1e-8, res=False)
    b = oracle.ipm(qp.copy(), k_max=60, mu_tol=1e-8, res=False)
    assert a["kk"] == b["kk"] and a["ret"] == b["ret"]
    for key in ("ux", "pi", "t", "lam"):
        for k in range(len(b[key])):
            n = qp.nux(k) if key == "ux" else (int(qp.nx[k + 1]) if key == "pi" else qp.nconstr(k))
            if key in ("t", "lam"):
                nbk, pnb, ngk, png = int(qp.nb[k]), qp.pnb(k), int(qp.ng[k]), qp.png(k)
                idx = np.r_[0:nbk, pnb:pnb + nbk, 2 * pnb:2 * pnb + ngk, 2 * pnb + png:2 * pnb + png + ngk].astype(int)
                assert _rel(a[key][k][idx], b[key][k][idx]) <= (TOL_KKT2["lam"] if key == "lam" else tol_cond(1e-8)), (key, k)
            else:
                assert _rel(a[key][k][:n], b[key][k][:n]) <= tol_cond(1e-8), (key, k)


def test_wide_single_newton_vs_oracle(product, oracle):
    qp = random_qp(8, [0] + [22] * 8, [5] * 8 + [0], [5] + [14] * 7 + [10], seed=21)
    r = oracle.ipm(qp.copy(), k_max=60)
    rng = np.random.default_rng(8)
    ux0 = [0.9 * x for x in r["ux"]]
    pi0 = [0.9 * x for x in r["pi"]]
    lam0 = [np.concatenate([1 + 0.1 * rng.random(2 * int(n)), np.zeros(4)]) for n in qp.nb]
    t0 = [np.concatenate([0.5 + 0.1 * rng.random(2 * int(n)), np.zeros(4)]) for n in qp.nb]
    a = product.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=2, mu0=0.1)
    b = oracle.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=2, mu0=0.1)
    compare_ipm(qp, a, b)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-9, atol=1e-14)


def test_wide_warm_start_and_unconstrained(product, oracle):
    qp = random_qp(9, [0] + [18] * 9, [6] * 9 + [0], [6] + [9] * 9, seed=33)
    rng = np.random.default_rng(1)
    ux0 = [0.1 * rng.standard_normal(qp.nux(k) + 4) for k in range(10)]
    a = product.ipm(qp.copy(), k_max=50, warm_start=1, ux=ux0)
    b = oracle.ipm(qp.copy(), k_max=50, warm_start=1, ux=ux0)
    compare_ipm(qp, a, b)
    # no constraints: mu_scal == 0, one Riccati solve (d_ip2_res_hard.c:428-450)
    qp = random_qp(9, [0] + [18] * 9, [6] * 9 + [0], None, seed=34)
    a = product.ipm(qp.copy(), k_max=50)
    b = oracle.ipm(qp.copy(), k_max=50)
    assert a["kk"] == 0 and a["ret"] == 0
    compare_ipm(qp, a, b)


def test_wide_infeasible_alpha_min(product, oracle):
    """Contradictory general constraints (lg > ug on one row): the step length collapses and both stop with
    ret 2 at the same iteration."""
    qp = random_qp(6, [0] + [20] * 6, [4] * 6 + [0], [4] + [6] * 6, seed=51, ng=[0, 3, 3, 3, 3, 3, 0])
    for k in (2, 3):
        pnb, png = qp.pnb(k), qp.png(k)
        qp.d[k][2 * pnb] = 1.0          # lg_0 =  1
        qp.d[k][2 * pnb + png] = -1.0   # ug_0 = -1
    a = product.ipm(qp.copy(), k_max=40)
    b = oracle.ipm(qp.copy(), k_max=40)
    assert a["kk"] == b["kk"] and a["ret"] == b["ret"], (a["kk"], b["kk"], a["ret"], b["ret"])


def test_wide_size_checks(product):
    """Stages beyond the wide kernels' limits, duplicate box indices and nb > nu+nx return EUNSUPPORTED."""
    qp = random_qp(3, [0, 70, 70, 70], [4, 4, 4, 0], [2, 2, 2, 2], seed=1)  # nx > 64
    assert product.ipm(qp.copy(), k_max=5)["ret"] == EUNSUPPORTED
    qp = random_qp(3, [0] + [20] * 3, [4] * 3 + [0], [4, 6, 6, 6], seed=2)
    qp.idxb[1][1] = qp.idxb[1][0]
    assert product.ipm(qp.copy(), k_max=5)["ret"] == EUNSUPPORTED


@pytest.mark.parametrize("case", [CASES[2], CASES[3], CASES[4]], ids=["wide_general", "narrow_slots", "N1"])
def test_wide_riccati_general_vs_oracle(product, oracle, case):
    """d_back_ric_rec_sv_tv_res / _trf_tv_res / _trs_tv_res with general constraints on the wide path (DCt diag(Qx_g)
    DCt' as MFMA tiles, DCt qx_g in the solve), box terms as the reference's in-place side effects."""
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=3 * N + 2, ng=ng)
    rng = np.random.default_rng(N + 11)

    def vec(k, scale, off):
        v = np.zeros(qp.pnb(k) + qp.png(k) + 8)
        v[: qp.nb[k]] = off + scale * rng.random(int(qp.nb[k]))
        v[qp.pnb(k): qp.pnb(k) + qp.ng[k]] = off + scale * rng.random(int(qp.ng[k]))
        return v

    bd = [vec(k, 1.0, 1.0) for k in range(N + 1)]
    Qx = [vec(k, 1.0, 0.5) for k in range(N + 1)]
    qx = [vec(k, 2.0, -1.0) for k in range(N + 1)]
    qa, qb = qp.copy(), qp.copy()
    ua, pa, Pa, _ = product.ric_sv(qa, bd=bd, Qx=Qx, qx=qx, compute_pi=1, compute_Pb=1)
    ub, pb, Pbb, _ = oracle.ric_sv(qb, bd=bd, Qx=Qx, qx=qx, compute_pi=1, compute_Pb=1)
    for k in range(N + 1):
        assert _rel(ua[k][: qp.nux(k)], ub[k][: qp.nux(k)]) <= TOL_RIC, k
        np.testing.assert_array_equal(qa.RSQrq[k], qb.RSQrq[k])  # the reference's side effects on RSQrq
        if k < N:
            m = int(qp.nx[k + 1])
            assert _rel(pa[k][:m], pb[k][:m]) <= TOL_RIC, k
            assert _rel(Pa[k][:m], Pbb[k][:m]) <= TOL_RIC, k
    mem_a = product.ric_trf(qp.copy(), bd=bd, Qx=Qx)
    mem_b = oracle.ric_trf(qp.copy(), bd=bd, Qx=Qx)
    b = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    q = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ta = product.ric_trs(qp.copy(), mem_a, b=b, q=q, qx=qx)
    tb = oracle.ric_trs(qp.copy(), mem_b, b=b, q=q, qx=qx)
    for k in range(N + 1):
        assert _rel(ta[0][k][: qp.nux(k)], tb[0][k][: qp.nux(k)]) <= TOL_RIC, k
        if k < N:
            m = int(qp.nx[k + 1])
            assert _rel(ta[1][k][:m], tb[1][k][:m]) <= TOL_RIC, k
