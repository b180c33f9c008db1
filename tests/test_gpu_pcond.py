"""Partial condensing and the wide-stage Riccati on the HIP path against the oracle.

The reference's own pins are the pcond / pcond_sv goldens (run through test_gpu_parity.py): d_part_cond /
d_part_expand_solution outputs of the reference c99 build where it is right (nu <= 4), and its direct Riccati
solution at the configs[4] size (N=200 nx=24 nu=6 -> 20 blocks), which condense -> sv -> expand must
reproduce.  These cases add the nu > 4 condensing (where the oracle, not the reference build, is the
checker -- DESIGN.md), boxes that become general constraints, wide stages of arbitrary sizes through
d_back_ric_rec_sv_tv_res, and the batched device pipeline.  Tolerances: Riccati 1e-12;
condensed pipeline vs direct solve 1e-11.
"""
import os

import numpy as np
import pytest

from hpmpc_amd.cabi import HpmpcAPI, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from helpers import TOL_PCOND_SV, TOL_RIC, check_pcond, pcond_sv, random_qp

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)), initial=0.0))


WIDE = [
    # N, nx, nu, nb
    (4, [0] + [20] * 4, [6] * 4 + [0], None),
    (3, [0, 24, 24, 24], [60, 60, 60, 0], None),
    (5, [7, 30, 12, 17, 9, 25], [3, 11, 40, 2, 5, 0], None),
    (6, [0] + [18] * 6, [5] * 6 + [0], [3] + [6] * 5 + [4]),
]


@pytest.mark.parametrize("case", WIDE, ids=[f"N{c[0]}_{i}" for i, c in enumerate(WIDE)])
def test_wide_sv_vs_oracle(product, oracle, case):
    """d_back_ric_rec_sv_tv_res with nu+nx > 16 (the wide-stage path), with box terms and update rows."""
    N, nx, nu, nb = case
    qp = random_qp(N, nx, nu, nb, seed=41 + N)
    rng = np.random.default_rng(N)
    kw = dict(compute_pi=1, compute_Pb=1)
    if nb is not None:
        kw.update(bd=[rng.random(max(int(n), 1)) + 0.5 for n in qp.nb], Qx=[rng.random(max(int(n), 1)) for n in qp.nb],
                  qx=[rng.standard_normal(max(int(n), 1)) for n in qp.nb],
                  update_b=1, b=[rng.standard_normal(int(qp.nx[k + 1]) + 8) for k in range(N)],
                  update_q=1, q=[rng.standard_normal(qp.nux(k) + 8) for k in range(N + 1)])
    q1, q2 = qp.copy(), qp.copy()
    u1, p1, b1, _ = product.ric_sv(q1, **kw)
    u2, p2, b2, _ = oracle.ric_sv(q2, **kw)
    for k in range(N + 1):
        assert _rel(u1[k][:qp.nux(k)], u2[k][:qp.nux(k)]) <= TOL_RIC, k
        if k < N:
            m = int(qp.nx[k + 1])
            assert _rel(p1[k][:m], p2[k][:m]) <= TOL_RIC and _rel(b1[k][:m], b2[k][:m]) <= TOL_RIC, k
        np.testing.assert_array_equal(q1.RSQrq[k], q2.RSQrq[k])
        if k < N:
            np.testing.assert_array_equal(q1.BAbt[k], q2.BAbt[k])


@pytest.mark.parametrize("case", WIDE, ids=[f"N{c[0]}_{i}" for i, c in enumerate(WIDE)])
def test_wide_trf_trs_vs_oracle(product, oracle, case):
    """d_back_ric_rec_trf_tv_res once, then d_back_ric_rec_trs_tv_res for several right-hand sides, on wide
    stages; the last trial passes Pb in (compute_Pb = 0)."""
    N, nx, nu, nb = case
    qp = random_qp(N, nx, nu, nb, seed=73 + N)
    rng = np.random.default_rng(7 * N)
    bd = [rng.random(max(int(n), 1)) + 0.5 for n in qp.nb]
    Qx = [rng.random(max(int(n), 1)) for n in qp.nb]
    res = []
    for api in (product, oracle):
        q0 = qp.copy()
        mem = api.ric_trf(q0, bd=bd, Qx=Qx)
        outs = []
        for trial in range(3):
            r2 = np.random.default_rng(200 + trial)
            b = [r2.standard_normal(int(qp.nx[k + 1]) + 8) for k in range(N)]
            q = [r2.standard_normal(qp.nux(k) + 8) for k in range(N + 1)]
            qx = [r2.standard_normal(max(int(n), 1)) for n in qp.nb]
            kw = dict(compute_pi=1, compute_Pb=1)
            if trial == 2:
                kw = dict(compute_pi=1, compute_Pb=0,
                          Pb=[r2.standard_normal(int(qp.nx[k + 1]) + 8) for k in range(N)])
            outs.append(api.ric_trs(q0, mem, b=b, q=q, qx=qx, **kw))
        res.append((outs, q0))
    (o1, g1), (o2, g2) = res
    for k in range(N + 1):
        np.testing.assert_array_equal(g1.RSQrq[k], g2.RSQrq[k])
    for (u1, p1, b1), (u2, p2, b2) in zip(o1, o2):
        for k in range(N + 1):
            assert _rel(u1[k][:qp.nux(k)], u2[k][:qp.nux(k)]) <= TOL_RIC, k
            if k < N:
                m = int(qp.nx[k + 1])
                assert _rel(p1[k][:m], p2[k][:m]) <= TOL_RIC and _rel(b1[k][:m], b2[k][:m]) <= TOL_RIC, k


PCOND = [
    # N, nx, nu, N2, boxes
    (40, 12, 6, 8, True),     # nu > 4: the reference c99 build is wrong here, the oracle is the checker
    (30, 24, 6, 3, False),
    (23, 10, 5, 5, True),     # uneven blocks (first R1 blocks one stage longer)
    (10, 6, 3, 1, True),      # a single block
]


@pytest.mark.parametrize("case", PCOND, ids=[f"N{c[0]}_nu{c[2]}_N2_{c[3]}" for c in PCOND])
def test_pcond_entry_points_vs_oracle(product, oracle, case):
    """d_part_cond + d_part_expand_solution through the C ABI against the oracle (condensed data and the
    expansion of random condensed-space vectors)."""
    from hpmpc_amd.golden import Case
    from hpmpc_amd.ocp import mass_spring_qp

    N, nx, nu, N2, boxes = case
    qp = mass_spring_qp(N, nx, nu, boxes=boxes)
    c, _ = oracle.part_cond(qp.copy(), N2)
    rng = np.random.default_rng(N)
    rv = lambda n: np.concatenate([rng.standard_normal(n), np.zeros(8)])
    u2 = [rv(c.nux(k)) for k in range(N2 + 1)]
    p2 = [rv(int(c.nx[k + 1])) for k in range(N2)]
    lam2 = [np.abs(rv(c.nconstr(k))) for k in range(N2 + 1)]
    t2 = [np.abs(rv(c.nconstr(k))) for k in range(N2 + 1)]
    e = oracle.part_expand(qp, c, u2, p2, lam2, t2)
    case_like = Case.__new__(Case)
    case_like.name, case_like.qp = f"pcond_N{N}_nu{nu}", qp
    case_like.out = dict(BAbt2=c.BAbt, RSQrq2=c.RSQrq[:N2], DCt2=c.DCt[:N2] if c.DCt else [], d2=c.d[:N2],
                         idxb2=[i.astype(np.float64) for i in c.idxb[:N2]], nx2=c.nx, nu2=c.nu, nb2=c.nb, ng2=c.ng,
                         ux=e["ux"], pi=e["pi"], lam=e["lam"], t=e["t"])
    gc, _ = product.part_cond(qp.copy(), N2)
    ge = product.part_expand(qp, gc, u2, p2, lam2, t2)
    check_pcond(case_like, dict(cqp=gc, ux=ge["ux"], pi=ge["pi"], lam=ge["lam"], t=ge["t"]))


COND_PARTS = [
    # N, nx, nu, s0, T: blocks of time-variant boxed mass-spring problems
    (200, 24, 6, 40, 10),   # a configs[4] block (nu > 4: the oracle is the checker)
    (30, 12, 5, 0, 6),      # first block (nx_0 = 0)
    (12, 18, 7, 4, 2),
    (20, 30, 3, 5, 7),      # nx > 16
]


@pytest.mark.parametrize("case", COND_PARTS, ids=[f"N{c[0]}_nx{c[1]}_nu{c[2]}_T{c[4]}" for c in COND_PARTS])
def test_cond_parts_vs_oracle(product, oracle, case):
    """d_cond_BAbt / d_cond_RSQrq / d_cond_DCtd alone (one hk_pcond phase each) against the oracle's restatement
    of the same building blocks, on shapes the c99 reference build gets wrong (nu > 4) or the goldens lack; the
    checks are the goldens' (check_cond_parts): same elements written, values to 1e-12."""
    from hpmpc_amd.golden import Case
    from hpmpc_amd.ocp import mass_spring_qp
    from helpers import COND_FILL, check_cond_parts, sub_block

    N, nx, nu, s0, T = case
    qp = mass_spring_qp(N, nx, nu, boxes=True, batch=1, time_variant=True, seed=N + T).problem(0)
    b = sub_block(qp, s0, T)
    G, B2 = oracle.cond_BAbt(b.copy(), fill=COND_FILL)
    R2 = oracle.cond_RSQrq(b.copy(), G, fill=COND_FILL)
    DCt2, d2, idxb2, _ = oracle.cond_DCtd(b.copy(), G, fill=COND_FILL)
    like = Case.__new__(Case)
    like.name, like.qp, like.args = f"cond_parts_{case}", b, dict(fill=COND_FILL)
    like.out = dict(Gamma=G, BAbt2=B2, RSQrq2=R2, DCt2=DCt2, d2=d2, idxb2=idxb2.astype(np.float64))
    pG, pB2 = product.cond_BAbt(b.copy(), fill=COND_FILL)
    pR2 = product.cond_RSQrq(b.copy(), G, fill=COND_FILL)
    pD, pd2, pidx, _ = product.cond_DCtd(b.copy(), G, fill=COND_FILL)
    check_cond_parts(like, dict(Gamma=pG, BAbt2=pB2, RSQrq2=pR2, DCt2=pD, d2=pd2, idxb2=pidx))


def test_pcond_sv_pipeline_nu6(product, oracle):
    """condense -> wide sv -> expand through the C ABI == the oracle's direct Riccati (nu = 6)."""
    from hpmpc_amd.ocp import mass_spring_qp

    qp = mass_spring_qp(40, 12, 6, boxes=False)
    got = pcond_sv(product, qp.copy(), 8)
    u, p, _, _ = oracle.ric_sv(qp.copy(), compute_pi=1, compute_Pb=0)
    for k in range(41):
        assert _rel(got["ux"][k][:qp.nux(k)], u[k][:qp.nux(k)]) <= TOL_PCOND_SV, k
        if k < 40:
            assert _rel(got["pi"][k][:12], p[k][:12]) <= TOL_PCOND_SV, k


@pytest.mark.parametrize("N,nx,nu,N2,batch", [(40, 12, 6, 8, 16), (200, 24, 6, 20, 512)])
def test_pcond_batch_pipeline(oracle, N, nx, nu, N2, batch):
    """The batched device pipeline (configs[4] at full size: 512 x N=200 nx=24 nu=6 -> 20 blocks): sampled
    problems equal the oracle's direct Riccati solution; repeated and split launches are bitwise identical."""
    import torch

    from hpmpc_amd.ocp import mass_spring_qp
    from hpmpc_amd.pcond import PcondSolver

    qp = mass_spring_qp(N, nx, nu, boxes=False, batch=batch, time_variant=True, seed=3)
    s = PcondSolver(qp, N2)
    s.solve()
    torch.cuda.synchronize()
    ux1 = s.ux.clone()
    s.ux.zero_()
    h = batch // 2
    for p0, cnt in ((0, h), (h, batch - h)):
        s.condense(p0, cnt)
        s.riccati(p0, cnt)
        s.expand(p0, cnt)
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux1)
    for p in sorted({0, 1, batch // 2, batch - 1}):
        U, Pi = s.solution(p)
        u, pi, _, _ = oracle.ric_sv(qp.problem(p), compute_pi=1, compute_Pb=0)
        for k in range(N + 1):
            assert _rel(U[k], u[k][:qp.nux(k)]) <= TOL_PCOND_SV, (p, k)
            if k < N:
                assert _rel(Pi[k], pi[k][:nx]) <= TOL_PCOND_SV, (p, k)


@pytest.mark.parametrize("N,nx,nu,N2,B", [(40, 12, 4, 4, 8), (60, 24, 6, 6, 4)], ids=["N40_nu4", "N60_nx24_nu6"])
def test_pcond_ipm_batch_pipeline(oracle, N, nx, nu, N2, B):
    """The IPM on a partially condensed batch (configs[4] with boxes): hk_pcond (inner state boxes become the
    condensed problem's general constraints) -> the batched wide-stage IPM (hpmpc_mi355x_wide_ipm_batch) ->
    hk_pexpand, against the oracle's d_part_cond -> d_ip2_res_mpc_hard_tv -> d_part_expand_solution problem by
    problem: identical iteration counts and return codes, the expanded point close to the oracle's and meeting the
    original problem's KKT conditions as tightly."""
    from hpmpc_amd.ocp import mass_spring_qp

    _pcond_ipm_vs_oracle(oracle, mass_spring_qp(N, nx, nu, boxes=True, batch=B, time_variant=True, seed=N), N2,
                         range(B))


def test_pcond_ipm_full_size(oracle):
    """configs[4] with boxes at its full size: 512 x N=200 nx=24 nu=6 condensed into 20 blocks (ng2 = 108 general
    constraints per inner block), the whole batch in one wide-IPM launch; split launches are bitwise the whole
    batch's, and sampled problems -- converged ones and non-converged ones -- match the oracle's pipeline."""
    import torch

    from hpmpc_amd.shard import global_block

    bq = global_block(200, 24, 6, 0, 512)
    s = _pcond_ipm_vs_oracle(oracle, bq, 20, [])
    ux1, kk1, ret1 = s.ux.clone(), s.kk2.clone(), s.ret2.clone()
    s.ux.zero_()
    s.condense(0, 200)
    s.condense(200, 312)
    s.ipm(k_max=60, p0=0, count=300)
    s.ipm(k_max=60, p0=300, count=212)
    s.expand()
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux1) and torch.equal(s.kk2, kk1) and torch.equal(s.ret2, ret1)
    ret = ret1.cpu().numpy()
    conv, bad = np.nonzero(ret == 0)[0], np.nonzero(ret != 0)[0]
    assert conv.size > 0
    sample = sorted({int(conv[0]), int(conv[-1]), int(conv[conv.size // 2])} | {int(p) for p in bad[:2]})
    _pcond_ipm_vs_oracle(oracle, bq, 20, sample, solver=s)


def _pcond_ipm_vs_oracle(oracle, bq, N2, problems, solver=None):
    from hpmpc_amd.cabi import bq_from_qp
    from hpmpc_amd.pcond import PcondSolver

    N, nx = bq.N, int(bq.nx[1])
    s = solver
    if s is None:
        s = PcondSolver(bq, N2)
        s.solve_ipm(k_max=60)
    import torch

    torch.cuda.synchronize()
    kk, ret = s.kk2.cpu().numpy(), s.ret2.cpu().numpy()
    # no reference golden exists at these shapes (the reference's own condensing is wrong at nu > 4), so
    # the gates come from the build spread of the oracle pipeline itself, per problem and quantity: the same
    # restatement built with -mfma -ffp-contract=fast (oracle/liboracle_fma.so), gate = max(1e-10, 4 x spread) -- the
    # rule of test_gpu_parity.py GATES.  Measured (tools/pcond_ipm_err.py): the GPU point sits at the builds' own
    # spread, 1e-14..1e-13 on well-conditioned problems and up to ~1e-8 where the last Newton systems carry
    # lam / t ~ 1/mu and the condensed inner-state boxes enter as general constraints.
    ofma = HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle_fma.so")), "orc_")
    for p in problems:
        qp = bq.problem(p)
        es = []
        for o in (oracle, ofma):
            c, _ = o.part_cond(qp.copy(), N2)
            r = o.ipm(c.copy(), k_max=60)
            es.append((r, o.part_expand(qp, c, r["ux"], r["pi"], r["lam"], r["t"])))
        (r, e), (_, e2) = es
        assert (int(kk[p]), int(ret[p])) == (r["kk"], r["ret"]), (p, kk[p], r["kk"], ret[p], r["ret"])
        if r["ret"] != 0:  # N60_nx24: three of four problems are box-infeasible (ret 1 / 2, |pi| 1e16..1e33): the
            continue  # matching (kk, ret) is the check, the diverged iterates carry no comparable digits
        U, Pi = s.solution(p)
        Lm, T = s.multipliers(p)
        box = [np.r_[0:int(qp.nb[k]), qp.pnb(k):qp.pnb(k) + int(qp.nb[k])].astype(int) for k in range(N + 1)]
        views = {"ux": (U, e["ux"], e2["ux"], [slice(0, qp.nux(k)) for k in range(N + 1)]),
                 "pi": (Pi, e["pi"], e2["pi"], [slice(0, int(qp.nx[k + 1])) for k in range(N)]),
                 "lam": (Lm, e["lam"], e2["lam"], box), "t": (T, e["t"], e2["t"], box)}
        for key, (got, ref, alt, sel) in views.items():
            err = spread = 0.0
            for k, ix in enumerate(sel):
                g_, r_, a_ = np.asarray(got[k])[ix], np.asarray(ref[k])[ix], np.asarray(alt[k])[ix]
                w = np.maximum(1.0, np.abs(r_))
                err = max(err, float(np.max(np.abs(g_ - r_) / w, initial=0.0)))
                spread = max(spread, float(np.max(np.abs(a_ - r_) / w, initial=0.0)))
            assert err <= max(1e-10, 4.0 * spread), (p, key, err, spread)
        # and the GPU point satisfies the ORIGINAL problem's KKT conditions (d_res_mpc_hard_tv) as well as the
        # oracle's own point does
        b, q = bq_from_qp(qp)
        pad = lambda xs: [np.r_[np.asarray(x, dtype=np.float64), np.zeros(8)] for x in xs]
        rg = oracle.residuals_plain(qp, b, q, pad(U), pad(Pi), pad(Lm), pad(T))
        ro = oracle.residuals_plain(qp, b, q, pad(e["ux"]), pad(e["pi"]), pad(e["lam"]), pad(e["t"]))
        for key in ("rq", "rb", "rd"):
            got = max(float(np.max(np.abs(x), initial=0)) for x in rg[key])
            ref = max(float(np.max(np.abs(x), initial=0)) for x in ro[key])
            assert got <= max(10 * ref, 1e-9), (p, key, got, ref)
    return s


@pytest.mark.parametrize("coupled", [False, True], ids=["mass_spring", "coupled"])
def test_pcond_pform_matches_cholesky_route(coupled):
    """hk_pcond's P form (W W' = [BAbt | e] X^ [BAbt | e]' on stages whose clamp certificate holds) against the
    reference's route on every stage (HPMPC_MI355X_PCOND_PFORM=0: state-block Cholesky, W = BAbt L + l, W W'):
    the condensed data agree to rounding (1e-12 relative), on the benchmark's data (every certificate holds) and on
    coupled, non-diagonally-dominant stage Hessians (the Gershgorin certificate fails and the stages fall back)."""
    import os

    import torch

    from hpmpc_amd.pcond import PcondSolver
    from hpmpc_amd.shard import coupled_shard, make_shard

    gen = coupled_shard if coupled else make_shard
    qp = gen(60, 24, 6, 0, 1, 16, boxes=True)
    out = []
    for pf in (None, "0"):
        if pf is None:
            os.environ.pop("HPMPC_MI355X_PCOND_PFORM", None)
        else:
            os.environ["HPMPC_MI355X_PCOND_PFORM"] = pf
        try:
            s = PcondSolver(qp, 6)
            s.condense()
            torch.cuda.synchronize()
            out.append([t.clone() for t in (s.BAbt2, s.RSQrq2, s.DCt2, s.d2)])
        finally:
            os.environ.pop("HPMPC_MI355X_PCOND_PFORM", None)
    for a, b in zip(*out):
        scale = float(b.abs().max()) or 1.0
        assert float((a - b).abs().max()) <= 1e-12 * scale


def test_pcond_pform_wide_state_stage():
    """A time-varying block whose stage s has nx_s = 32 after a stage with nu + nx = 30: the P form's
    T = X^ [BAbt | e]' would need a third 16-row tile (nx + 1 = 33 rows), more than its one-tile-per-wave gemm covers,
    so such a stage takes the Cholesky route; the condensed data match the Cholesky route everywhere to rounding."""
    import os

    import torch

    from hpmpc_amd.pcond import PcondSolver
    from helpers import random_qp, stack_qps as stack

    N = 8
    nx = [0, 24, 24, 32, 32, 24, 24, 24, 24]
    nu = [6] * (N + 1)
    qps = [random_qp(N, nx, nu, nb=[0] * (N + 1), seed=300 + i, coupling=0.05) for i in range(4)]
    qp = stack(qps)
    out = []
    for pf in (None, "0"):
        if pf is None:
            os.environ.pop("HPMPC_MI355X_PCOND_PFORM", None)
        else:
            os.environ["HPMPC_MI355X_PCOND_PFORM"] = pf
        try:
            s = PcondSolver(qp, 2)
            s.condense()
            torch.cuda.synchronize()
            out.append([t.clone() for t in (s.BAbt2, s.RSQrq2, s.d2)])
        finally:
            os.environ.pop("HPMPC_MI355X_PCOND_PFORM", None)
    for a, b in zip(*out):
        scale = float(b.abs().max()) or 1.0
        assert float((a - b).abs().max()) <= 1e-12 * scale


@pytest.mark.parametrize("shape", ["bench", "coupled", "tv"])
def test_pcond_deferred_cross_terms_bitwise(shape):
    """hk_pcond's full condensing runs d_cond_RSQrq first and forms each stage's cross term M_s = Gamma_{s-1} pL_s[x, u]
    and its general constraints later, while d_cond_BAbt has Gamma_{s-1} in LDS (no Gamma through the HBM scratch).  Same
    operations on the same operands as the reference's order (HPMPC_MI355X_PCOND_DM=0): the condensed problem is bitwise
    the same, on the benchmark data, on coupled stage Hessians (Cholesky route) and with time-varying stage sizes."""
    import os

    import torch

    from hpmpc_amd.pcond import PcondSolver
    from hpmpc_amd.shard import coupled_shard, make_shard
    from helpers import stack_qps

    if shape == "bench":
        qp, N2 = make_shard(60, 24, 6, 0, 1, 16, boxes=True), 6
    elif shape == "coupled":
        qp, N2 = coupled_shard(60, 24, 6, 0, 1, 16, boxes=True), 6
    else:
        N = 13
        nx = [0, 5, 9, 24, 7, 12, 12, 3, 16, 10, 8, 8, 20, 6]
        nu = [3, 2, 6, 1, 4, 4, 5, 2, 3, 6, 2, 3, 1, 0]
        nb = [2, 4, 8, 3, 5, 9, 7, 2, 6, 8, 4, 5, 9, 3]
        qp, N2 = stack_qps([random_qp(N, nx, nu, nb=nb, seed=700 + i, coupling=0.1) for i in range(6)]), 4
    out = []
    for dm in ("1", "0"):
        os.environ["HPMPC_MI355X_PCOND_DM"] = dm
        try:
            s = PcondSolver(qp, N2)
            s.condense()
            torch.cuda.synchronize()
            out.append([t.clone() for t in (s.BAbt2, s.RSQrq2, s.DCt2, s.d2)])
        finally:
            os.environ.pop("HPMPC_MI355X_PCOND_DM", None)
    for name, a, b in zip(("BAbt2", "RSQrq2", "DCt2", "d2"), *out):
        assert torch.equal(a, b), name
