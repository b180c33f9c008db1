"""General constraints lg <= D_k ux_k <= ug (ng > 0) on the HIP path against the oracle.

The reference's own pin for this branch is the golden `ipm_ng_N30_nx8_nu3` (terminal D = I, run
through test_gpu_parity.py); these cases add dense random D at inner stages, at stage 0 (u only), next
to boxes, and through every entry point that takes DCt (sv/trf/trs with given Qx/qx, the residuals,
the IPM and the KKT re-solve).  Tolerances as SURVEY.md §8c: Riccati 1e-12, IPM identical kk / 1e-10.
"""
import numpy as np
import pytest

from helpers import TOL_IPM, TOL_RIC, compare_ipm, random_qp

pytestmark = pytest.mark.gpu

CASES = [
    # N, nx, nu, nb, ng
    (6, [0] + [4] * 6, [2] * 6 + [0], [1] + [2] * 5 + [2], [2] + [3] * 5 + [4]),
    (10, [0] + [8] * 10, [3] * 10 + [0], [2] + [3] * 9 + [4], [0] + [2] * 9 + [8]),
    (12, [0] + [12] * 12, [4] * 12 + [0], [4] + [6] * 11 + [6], [1] + [0, 3] * 5 + [4, 8]),
    (5, [0, 6, 9, 9, 5, 7], [3, 2, 4, 1, 3, 0], [0, 4, 2, 3, 0, 2], [3, 0, 5, 2, 7, 4]),
]


def fma_oracle():
    import os

    from hpmpc_amd.cabi import HpmpcAPI, load

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return HpmpcAPI(load(os.path.join(root, "oracle", "liboracle_fma.so")), "orc_")


def _rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)), initial=0.0))


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_ipm_general_vs_oracle(product, oracle, case):
    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=7 * N + 1, ng=ng)
    a = product.ipm(qp.copy(), k_max=40)
    b = oracle.ipm(qp.copy(), k_max=40)
    compare_ipm(qp, a, b, tol=TOL_IPM)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-8, atol=1e-13)
    # the KKT re-solve with new right-hand sides from the persisted factor and iterate
    rng = np.random.default_rng(N)
    bb = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    qq = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ka = product.kkt_new_rhs(qp.copy(), a["work"], bb, qq)
    kb = oracle.kkt_new_rhs(qp.copy(), b["work"], bb, qq)
    # The re-solve runs on the last iteration's Newton system, whose lam / t ~ 1 / mu terms lift summation-order
    # differences: the gate is the GATES rule of test_gpu_parity.py, max(TOL_IPM, 4 x the spread of the oracle's own
    # builds) -- the same restatement compiled with -mfma -ffp-contract=fast (oracle/liboracle_fma.so).  Measured: 3.3e-11
    # in lam on the N6 case (so gate 1.3e-10; the GPU's P-form records give 1.05e-10 there), <= 1e-19 on the others.
    bf = fma_oracle().ipm(qp.copy(), k_max=40)
    kf = fma_oracle().kkt_new_rhs(qp.copy(), bf["work"], bb, qq)
    for key, size in (("ux", qp.nux), ("lam", qp.nconstr), ("t", qp.nconstr)):
        spread = max(_rel(kf[key][k][:size(k)], kb[key][k][:size(k)]) for k in range(N + 1))
        gate = max(TOL_IPM, 4 * spread)
        err = max(_rel(ka[key][k][:size(k)], kb[key][k][:size(k)]) for k in range(N + 1))
        assert err <= gate, (key, err, gate)
        # regression pin: the largest error measured since the P-form records is 1.05e-10 (N6, lam), at
        # 0.81 of its gate; an error above 1.5e-10 is a regression even where a wider oracle spread would admit it
        assert err <= max(TOL_IPM, 1.5e-10), (key, err, "above the pinned P-form error")


@pytest.mark.parametrize("case", CASES[:3], ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES[:3])])
def test_riccati_general_vs_oracle(product, oracle, case):
    """sv / trf + trs with given box and general Hessian / gradient terms (Qx, qx = [box | general])."""
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
    ua, pa, Pa, ma = product.ric_sv(qp.copy(), bd=bd, Qx=Qx, qx=qx, compute_pi=1, compute_Pb=1)
    ub, pb, Pbb, mb = oracle.ric_sv(qp.copy(), bd=bd, Qx=Qx, qx=qx, compute_pi=1, compute_Pb=1)
    for k in range(N + 1):
        assert _rel(ua[k][: qp.nux(k)], ub[k][: qp.nux(k)]) <= TOL_RIC, k
        if k < N:
            m = int(qp.nx[k + 1])
            assert _rel(pa[k][:m], pb[k][:m]) <= TOL_RIC, k
            assert _rel(Pa[k][:m], Pbb[k][:m]) <= TOL_RIC, k
    # trf then trs with new right-hand sides
    mem_a = product.ric_trf(qp.copy(), bd=bd, Qx=Qx)
    mem_b = oracle.ric_trf(qp.copy(), bd=bd, Qx=Qx)
    b = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    q = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    ta = product.ric_trs(qp.copy(), mem_a, b=b, q=q, qx=qx)
    tb = oracle.ric_trs(qp.copy(), mem_b, b=b, q=q, qx=qx)
    for k in range(N + 1):
        assert _rel(ta[0][k][: qp.nux(k)], tb[0][k][: qp.nux(k)]) <= TOL_RIC, k


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_residuals_general_vs_oracle(product, oracle, case):
    from hpmpc_amd.cabi import bq_from_qp

    N, nx, nu, nb, ng = case
    qp = random_qp(N, nx, nu, nb, seed=5 * N + 3, ng=ng)
    rng = np.random.default_rng(N + 3)
    b, q = bq_from_qp(qp)
    ux = [np.concatenate([rng.standard_normal(qp.nux(k)), np.zeros(8)]) for k in range(N + 1)]
    pi = [np.concatenate([rng.standard_normal(int(qp.nx[k + 1])), np.zeros(8)]) for k in range(N)]
    lam = [0.1 + rng.random(qp.nconstr(k) + 4) for k in range(N + 1)]
    t = [0.1 + rng.random(qp.nconstr(k) + 4) for k in range(N + 1)]
    ra = product.residuals(qp, b, q, ux, pi, lam, t)
    rb = oracle.residuals(qp, b, q, ux, pi, lam, t)
    for k in range(N + 1):
        assert _rel(ra["rq"][k][: qp.nux(k)], rb["rq"][k][: qp.nux(k)]) <= 1e-12, k
        nbk, pnb, ngk, png = int(qp.nb[k]), qp.pnb(k), int(qp.ng[k]), qp.png(k)
        idx = np.r_[0:nbk, pnb:pnb + nbk, 2 * pnb:2 * pnb + ngk, 2 * pnb + png:2 * pnb + png + ngk].astype(int)
        assert _rel(ra["rd"][k][idx], rb["rd"][k][idx]) <= 1e-12, k
        assert _rel(ra["rm"][k][idx], rb["rm"][k][idx]) <= 1e-12, k
    assert abs(ra["mu"] - rb["mu"]) <= 1e-12 * max(1.0, abs(rb["mu"]))


def test_batched_entry_rejects_general_constraints():
    """The batched device API carries no DCt array: a plan with ng > 0 is refused loudly."""
    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.ocp import mass_spring_qp

    qp = mass_spring_qp(6, 4, 1, batch=2)
    qp.ng = np.array([0] * 6 + [4], dtype=np.int32)
    s = BatchSolver(qp, k_max=5)
    with pytest.raises(RuntimeError):
        s.ipm()
