"""Parity of the HIP path (libhpmpc_mi355x.so on the MI355X) with the reference.

* every golden vector of the real reference (tests/golden) through the reference-named C ABI;
* the CPU oracle on seeded problems the goldens do not cover (varying stage sizes, arbitrary box
  index sets, aliased stage buffers, warm start, N = 1);
* the batched device API against the oracle problem by problem, and at the benchmark's full size
  (N=100 nx=12 nu=4, batch 1024) through size-independent properties: launch splitting and repeat
  runs are bit-identical, and converged problems satisfy the KKT conditions.

Tolerances: Riccati outputs 1e-12, IPM iterates 1e-10 relative to max(1,|ref|), with
identical iteration counts and return codes.
"""
import os

import numpy as np
import pytest

from hpmpc_amd.golden import load_all
from hpmpc_amd.ocp import mass_spring_qp
from helpers import XCLAMP, TOL_IPM, TOL_RIC, check_case, compare_ipm, random_qp, run_case

pytestmark = pytest.mark.gpu
EUNSUPPORTED = -10

CASES = load_all()
# headline-batch problems with a per-problem gate from the reference's build spread, by global problem id
GATES = {int(c.args["problem"]): c for c in CASES if "gate" in c.args and "problem" in c.args}


@pytest.fixture(autouse=True)
def _queue_ticks_to_the_end(monkeypatch):
    """Queue results in this module are compared bitwise with the batched solve, so the queue ticks to the end: the
    multi-wave drain (hk_ipm_qdrain_mw, HPMPC_MI355X_QUEUE_DRAIN) agrees with it to rounding only, and
    test_queue_drain_matches_oracle turns it back on."""
    monkeypatch.setenv("HPMPC_MI355X_QUEUE_DRAIN", "0")


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_golden_through_c_abi(product, case):
    check_case(case, run_case(product, case))


# The reference's inner-stage x-pivot clamp (kernel_dpotrf_c99_lib4.c:555-640): a state whose Hessian diagonal is
# d <= 1e-15 with cross terms `off` and gradient r.  The P form keeps its cheap record only on stages that pass the
# clamp certificate (hk_riccati.h cert_ok); these stages fail it and are factorised as the reference does, so the
# product returns the reference's clamped answer (the goldens sv_xclamp_* above, at 1e-12) and the oracle's on
# every other variant, through every kernel family.
# (a pivot just above the clamp, d = 2e-15, is left out: there the reference's own builds spread by 1e-11 -- its
# pivot is the difference of two rounding-level terms; the last two variants fail the certificate without a clamp)
# (the list lives in helpers.py: tests/golden/make_golden.py xclamp_ipm generates the IPM gates of these variants)
# IPM gates of the clamp problems (N=20, boxes): the GATES rule, max(default, 4 x the spread of the reference's own
# builds c99 / fma / X64_AVX / X64_AVX2), generated with the c99 answer by tests/golden/make_golden.py xclamp_ipm
# (ipm_xclamp_* goldens, which the golden sweep above also checks).  Only (1e-16, 1e-9, 0.5) carries one: it does not
# converge within k_max = 50 (ret 1 in every build) and the builds end 4.7e-5 apart; the others agree to <= 7e-14.
XCLAMP_IPM_TOL = {(float(c.args["xclamp_d"]), float(c.args["xclamp_off"]), float(c.args["xclamp_r"])): float(c.args["gate"])
                  for c in CASES if "xclamp_d" in c.args}


@pytest.mark.parametrize("d,off,r", XCLAMP, ids=[f"d{x[0]:g}_off{x[1]:g}_r{x[2]:g}" for x in XCLAMP])
def test_inner_x_pivot_clamp_riccati(product, oracle, d, off, r):
    from helpers import xclamp_qp

    qp = xclamp_qp(N=12, nx=8, nu=3, d=d, off=off, r=r)
    out = []
    for api in (product, oracle):
        ux, pi, Pb, _ = api.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
        mem = api.ric_trf(qp.copy())
        rng = np.random.default_rng(3)
        b = [rng.standard_normal(8) for _ in range(12)]
        q = [rng.standard_normal(11) for _ in range(13)]
        out.append((ux, pi, Pb) + api.ric_trs(qp.copy(), mem, b=b, q=q, compute_pi=1, compute_Pb=1))
    for k in range(13):
        n = qp.nux(k)
        for i in (0, 3):
            np.testing.assert_allclose(out[0][i][k][:n], out[1][i][k][:n], rtol=TOL_RIC, atol=TOL_RIC)
        if k < 12:
            for i in (1, 2, 4, 5):
                np.testing.assert_allclose(out[0][i][k][:8], out[1][i][k][:8], rtol=TOL_RIC, atol=TOL_RIC)


def test_inner_x_pivot_clamp_ipm(product, oracle):
    """The clamp inside the IPM: the drop-in call (the multi-wave solo kernel), the batched passes (fixed-shape
    class (3, 8)) and the single-wave solo kernel, each against the oracle problem by problem."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.ocp import OCPQP
    from helpers import xclamp_qp

    qps = [xclamp_qp(N=20, nx=8, nu=3, d=d, off=off, r=r, boxes=True) for d, off, r in XCLAMP]
    tols = [XCLAMP_IPM_TOL.get(v) for v in XCLAMP]
    for one, tol in zip(qps, tols):
        compare_ipm(one, product.ipm(one.copy(), k_max=50), oracle.ipm(one.copy(), k_max=50), tol=tol or TOL_IPM)
    q0 = qps[0]
    qp = OCPQP(q0.N, q0.nx, q0.nu, q0.nb, q0.ng, q0.idxb, [np.stack([q.BAbt[k] for q in qps]) for k in range(q0.N)],
               [np.stack([q.RSQrq[k] for q in qps]) for k in range(q0.N + 1)],
               [np.stack([q.d[k] for q in qps]) for k in range(q0.N + 1)], [], len(qps))
    s = BatchSolver(qp, k_max=50)
    old = os.environ.get("HPMPC_MI355X_SOLO")
    try:
        for mode in ("batch", "1"):
            if mode == "batch":
                s.ipm()
            else:
                os.environ["HPMPC_MI355X_SOLO"] = mode
                s.ipm_solo()
            torch.cuda.synchronize()
            g = {n: getattr(s, n).cpu().numpy() for n in ("ux", "pi", "lam", "t", "kk", "ret")}
            for p, (one, tol) in enumerate(zip(qps, tols)):
                got = dict(kk=int(g["kk"][p]), ret=int(g["ret"][p]), ux=[g["ux"][p, k] for k in range(q0.N + 1)],
                           pi=[g["pi"][p, k] for k in range(q0.N)], lam=[g["lam"][p, k] for k in range(q0.N + 1)],
                           t=[g["t"][p, k] for k in range(q0.N + 1)])
                compare_ipm(one, got, oracle.ipm(one.copy(), k_max=50), tol=tol or TOL_IPM)
    finally:
        if old is None:
            os.environ.pop("HPMPC_MI355X_SOLO", None)
        else:
            os.environ["HPMPC_MI355X_SOLO"] = old


SIZES = [
    # (N, nx per stage, nu per stage, nb per stage)
    (1, [0, 4], [2, 0], [2, 2]),
    (2, [0, 1, 1], [1, 1, 0], [1, 2, 1]),
    (7, [0, 3, 5, 5, 2, 7, 12, 9], [2, 4, 1, 3, 6, 4, 4, 0], [1, 3, 2, 0, 4, 5, 6, 3]),
    (12, [0] + [8] * 12, [8] * 12 + [0], [3] * 13),
    (20, [0] + [12] * 20, [4] * 20 + [0], [0] * 21),
    (9, [0] + [16] * 9, [4] + [0] * 9, [0] + [2] * 9),
    (5, [0, 12, 12, 11, 12, 12], [3, 3, 2, 4, 3, 0], [2, 15, 3, 10, 5, 12]),
]


@pytest.mark.parametrize("N,nx,nu,nb", SIZES, ids=[f"N{s[0]}_{i}" for i, s in enumerate(SIZES)])
def test_ipm_random_sizes_vs_oracle(product, oracle, N, nx, nu, nb):
    qp = random_qp(N, nx, nu, nb, seed=N * 31 + len(nx))
    a = product.ipm(qp.copy(), k_max=40)
    b = oracle.ipm(qp.copy(), k_max=40)
    compare_ipm(qp, a, b)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-9, atol=1e-14)


@pytest.mark.parametrize("N,nx,nu,nb", SIZES, ids=[f"N{s[0]}_{i}" for i, s in enumerate(SIZES)])
def test_riccati_random_sizes_vs_oracle(product, oracle, N, nx, nu, nb):
    qp = random_qp(N, nx, nu, nb, seed=N * 17 + 1)
    rng = np.random.default_rng(N)
    bd = [rng.random(max(int(n), 1)) + 0.5 for n in qp.nb]
    Qx = [rng.random(max(int(n), 1)) for n in qp.nb]
    qx = [rng.standard_normal(max(int(n), 1)) for n in qp.nb]
    out = []
    for api in (product, oracle):
        q1 = qp.copy()
        ux, pi, Pb, _ = api.ric_sv(q1, bd=bd, Qx=Qx, qx=qx, compute_pi=1, compute_Pb=1)
        out.append((ux, pi, Pb, q1))
    (u1, p1, b1, q1), (u2, p2, b2, q2) = out
    for k in range(N + 1):
        n = qp.nux(k)
        np.testing.assert_allclose(u1[k][:n], u2[k][:n], rtol=TOL_RIC, atol=TOL_RIC)
        if k < N:
            m = int(qp.nx[k + 1])
            np.testing.assert_allclose(p1[k][:m], p2[k][:m], rtol=TOL_RIC, atol=TOL_RIC)
            np.testing.assert_allclose(b1[k][:m], b2[k][:m], rtol=TOL_RIC, atol=TOL_RIC)
        # the in-place side effects on the caller's RSQrq (box diagonal / gradient) are the reference's
        np.testing.assert_array_equal(q1.RSQrq[k], q2.RSQrq[k])


def test_trf_trs_reuse_factor(product, oracle):
    qp = random_qp(10, [0] + [6] * 10, [3] * 10 + [0], [2] * 11, seed=5)
    rng = np.random.default_rng(5)
    bd = [rng.random(2) + 1.0 for _ in range(11)]
    Qx = [rng.random(2) for _ in range(11)]
    res = []
    for api in (product, oracle):
        mem = api.ric_trf(qp.copy(), bd=bd, Qx=Qx)
        outs = []
        for trial in range(3):  # several right-hand sides against one factorisation
            r2 = np.random.default_rng(100 + trial)
            b = [r2.standard_normal(8) for _ in range(10)]
            q = [r2.standard_normal(12) for _ in range(11)]
            qx = [r2.standard_normal(4) for _ in range(11)]
            outs.append(api.ric_trs(qp.copy(), mem, b=b, q=q, qx=qx, compute_pi=1, compute_Pb=1))
        res.append(outs)
    for (u1, p1, b1), (u2, p2, b2) in zip(*res):
        for k in range(11):
            np.testing.assert_allclose(u1[k][:qp.nux(k)], u2[k][:qp.nux(k)], rtol=TOL_RIC, atol=TOL_RIC)
            if k < 10:
                np.testing.assert_allclose(p1[k][:6], p2[k][:6], rtol=TOL_RIC, atol=TOL_RIC)
                np.testing.assert_allclose(b1[k][:6], b2[k][:6], rtol=TOL_RIC, atol=TOL_RIC)


def test_aliased_time_invariant_buffers(product, oracle):
    """The reference drivers pass the SAME buffer for every inner stage (test_d_ip_hard.c:420-440)."""
    qp = mass_spring_qp(25, 8, 3)
    for k in range(2, 25):
        qp.BAbt[k] = qp.BAbt[1]
    for k in range(2, 25):
        qp.RSQrq[k] = qp.RSQrq[1]
        qp.d[k] = qp.d[1]
    a = product.ipm(qp, k_max=50)
    b = oracle.ipm(qp, k_max=50)
    compare_ipm(qp, a, b)


def test_warm_start_and_kkt_resolve(product, oracle):
    qp = random_qp(15, [0] + [6] * 15, [2] * 15 + [0], [2] + [3] * 15, seed=11)
    ux0 = [np.random.default_rng(k).standard_normal(12) * 0.1 for k in range(16)]
    a = product.ipm(qp.copy(), k_max=30, warm_start=1, ux=ux0)
    b = oracle.ipm(qp.copy(), k_max=30, warm_start=1, ux=ux0)
    compare_ipm(qp, a, b)
    rng = np.random.default_rng(2)
    b2 = [rng.standard_normal(8) for _ in range(15)]
    q2 = [rng.standard_normal(12) for _ in range(16)]
    ka = product.kkt_new_rhs(qp.copy(), a["work"], b2, q2)
    kb = oracle.kkt_new_rhs(qp.copy(), b["work"], b2, q2)
    ka.update(kk=0, ret=0)
    kb.update(kk=0, ret=0)
    compare_ipm(qp, ka, kb)


def test_single_newton_steps(product, oracle):
    qp = mass_spring_qp(12, 8, 3)
    rng = np.random.default_rng(4)
    r = oracle.ipm(qp.copy(), k_max=50)
    ux0 = [0.9 * x for x in r["ux"]]
    pi0 = [0.9 * x for x in r["pi"]]
    lam0 = [np.concatenate([1 + 0.1 * rng.random(2 * int(n)), np.zeros(4)]) for n in qp.nb]
    t0 = [np.concatenate([0.5 + 0.1 * rng.random(2 * int(n)), np.zeros(4)]) for n in qp.nb]
    a = product.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=1, mu0=0.1)
    b = oracle.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=1, mu0=0.1)
    compare_ipm(qp, a, b)
    np.testing.assert_allclose(a["stat"], b["stat"], rtol=1e-9, atol=1e-14)


# ------------------------------------------------------------------ batched device API
@pytest.fixture(scope="module")
def small_batch():
    return mass_spring_qp(30, 8, 3, batch=64, time_variant=True, seed=9)


def test_batch_ipm_vs_oracle(oracle, small_batch):
    import torch

    from hpmpc_amd.batch import BatchSolver

    qp = small_batch
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    torch.cuda.synchronize()
    kk, ret = s.kk.cpu().numpy(), s.ret.cpu().numpy()
    ux, pi, lam, t = (x.cpu().numpy() for x in (s.ux, s.pi, s.lam, s.t))
    from helpers import DIVERGENT_SKIPS

    skips0 = len(DIVERGENT_SKIPS)
    for p in range(qp.batch):
        one = qp.problem(p)
        r = oracle.ipm(one, k_max=50)
        got = dict(kk=int(kk[p]), ret=int(ret[p]), ux=[ux[p, k] for k in range(31)],
                   pi=[pi[p, k] for k in range(30)], lam=[lam[p, k] for k in range(31)],
                   t=[t[p, k] for k in range(31)])
        # infeasible draws of x0 diverge (ret 2, lam -> 1e33) in the oracle and on the GPU alike: kk/ret only
        compare_ipm(one, got, r, allow_divergent=True)
    # this seeded batch has exactly one infeasible (diverging) problem, p = 59 (oracle and reference: kk 16,
    # ret 2, lam -> 3e33); nothing else may take the divergence escape
    n_div = len(DIVERGENT_SKIPS) - skips0
    assert n_div <= 1, n_div


def test_batch_riccati_vs_oracle(oracle):
    import torch

    from hpmpc_amd.batch import BatchSolver

    qp = mass_spring_qp(50, 8, 3, boxes=False, batch=32, time_variant=True, seed=2)
    s = BatchSolver(qp, k_max=1)
    s.ric_sv(compute_pi=1, compute_Pb=1)
    torch.cuda.synchronize()
    ux, pi, Pb = (x.cpu().numpy() for x in (s.ux, s.pi, s.Pb))
    for p in range(qp.batch):
        u2, p2, b2, _ = oracle.ric_sv(qp.problem(p), compute_pi=1, compute_Pb=1)
        for k in range(51):
            n = qp.nux(k)
            np.testing.assert_allclose(ux[p, k, :n], u2[k][:n], rtol=TOL_RIC, atol=TOL_RIC)
            if k < 50:
                np.testing.assert_allclose(pi[p, k, :8], p2[k][:8], rtol=TOL_RIC, atol=TOL_RIC)
                np.testing.assert_allclose(Pb[p, k, :8], b2[k][:8], rtol=TOL_RIC, atol=TOL_RIC)
    # trf + trs with new right-hand sides == sv with those rows
    s.ric_trf()
    rng = np.random.default_rng(0)
    b = torch.from_numpy(rng.standard_normal((32, 51, 16))).cuda()
    q = torch.from_numpy(rng.standard_normal((32, 51, 16))).cuda()
    s.ric_trs(b, q)
    torch.cuda.synchronize()
    ux = s.ux.cpu().numpy()
    for p in (0, 7, 31):
        one = qp.problem(p)
        mem = oracle.ric_trf(one)
        u2, _, _ = oracle.ric_trs(one, mem, b=[b[p, k].cpu().numpy().copy() for k in range(50)],
                                  q=[q[p, k].cpu().numpy().copy() for k in range(51)])
        for k in range(51):
            n = qp.nux(k)
            np.testing.assert_allclose(ux[p, k, :n], u2[k][:n], rtol=TOL_RIC, atol=TOL_RIC)


def test_full_size_properties():
    """N=100 nx=12 nu=4 batch=1024 (the benchmark workload): split launches and repeats are bitwise
    identical; converged problems satisfy primal feasibility and complementarity."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    qp = make_shard(100, 12, 4, 0, 1, 1024)
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    torch.cuda.synchronize()
    ux1, kk1, ret1 = s.ux.clone(), s.kk.clone(), s.ret.clone()
    lam, t = s.lam.cpu().numpy(), s.t.cpu().numpy()
    s.ux.zero_()
    s.ipm(p0=0, count=300)
    s.ipm(p0=300, count=724)
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux1) and torch.equal(s.kk, kk1) and torch.equal(s.ret, ret1)
    ret = ret1.cpu().numpy()
    kk = kk1.cpu().numpy()
    assert (ret == 0).sum() > 900 and kk.max() <= 50
    ux = ux1.cpu().numpy()
    d = s.d.cpu().numpy()
    conv = np.nonzero(ret == 0)[0]
    for k in range(101):
        nbk, pnb = int(qp.nb[k]), qp.pnb(k)
        v = ux[conv][:, k, qp.idxb[k]]
        lb, ub = d[conv, k, :nbk], d[conv, k, pnb:pnb + nbk]
        assert np.all(v >= lb - 1e-8) and np.all(v <= ub + 1e-8)
        lt = lam[conv, k, :nbk] * t[conv, k, :nbk] + lam[conv, k, pnb:pnb + nbk] * t[conv, k, pnb:pnb + nbk]
        assert np.all(lt < 1e-8)
    # exact parity for a sample spread over the batch
    from hpmpc_amd.cabi import HpmpcAPI, load
    import os

    orc = HpmpcAPI(load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                                      "liboracle.so")), "orc_")
    lamt = s.lam.cpu().numpy(), s.t.cpu().numpy()
    pi = s.pi.cpu().numpy()
    from helpers import DIVERGENT_SKIPS

    skips0 = len(DIVERGENT_SKIPS)
    unconverged = tuple(int(p) for p in np.nonzero(ret != 0)[0][:2])
    # the ill-conditioned problems with their own reference-spread gates (ipm_gate_* goldens): against the
    # reference's answer at that gate
    for p, case in GATES.items():
        got = dict(kk=int(kk[p]), ret=int(ret[p]), ux=[ux[p, k] for k in range(101)], pi=[pi[p, k] for k in range(100)],
                   lam=[lamt[0][p, k] for k in range(101)], t=[lamt[1][p, k] for k in range(101)])
        check_case(case, got | {"stat": case.out["stat"]})
    for p in (0, 1, 511, 1023) + unconverged:
        one = qp.problem(int(p))
        r = orc.ipm(one, k_max=50)
        got = dict(kk=int(kk[p]), ret=int(ret[p]), ux=[ux[p, k] for k in range(101)],
                   pi=[pi[p, k] for k in range(100)], lam=[lamt[0][p, k] for k in range(101)],
                   t=[lamt[1][p, k] for k in range(101)])
        # only the deliberately sampled non-converged problems may be divergent (compare kk/ret only)
        compare_ipm(one, got, r, tol=TOL_IPM, allow_divergent=p in unconverged and ret[p] == 2)
    assert len(DIVERGENT_SKIPS) - skips0 <= len(unconverged)


# ------------------------------------------------------------------ problem queue (continuous batching)
def _queue_equals_batch(s, Q, nq):
    import torch

    idx = torch.arange(nq, device=s.ux.device) % s.nprob
    for name in ("ux", "pi", "lam", "t", "kk", "ret", "stat"):
        a, b = getattr(Q, name), getattr(s, name)[idx]
        assert torch.equal(a, b), name


@pytest.mark.parametrize("n_slots,nq", [(16, 197), (64, 64), (100, 37)])
def test_queue_matches_batch(small_batch, n_slots, nq):
    """Every queue entry q is bitwise the batched solve of problem q % nprob, whatever the slot
    count (fewer slots than entries, equal, more slots than entries)."""
    import torch

    from hpmpc_amd.batch import BatchSolver

    s = BatchSolver(small_batch, k_max=50)
    s.ipm()
    Q = s.queue(nq, n_slots)
    pass_ms, ticks = Q.run(profiled=True)
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, nq)
    assert Q.finished() == nq and Q.idle()
    kk = s.kk.cpu().numpy()
    assert ticks >= int(kk.max()) and pass_ms[1] > 0.0
    Q.run()  # a second run over the same buffers gives the same answers
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, nq)


@pytest.mark.parametrize("lanes", [3, 4])
def test_queue_lanes_match_batch(monkeypatch, lanes):
    """A queue split into lanes (each a queue over its own slots on its own stream, forked from and joined back into
    the caller's, all handing out entries from one counter): every entry is bitwise the batched solve of its problem,
    with an uneven split of the slots, and the caller's stream sees every lane's results."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    monkeypatch.setenv("HPMPC_MI355X_QUEUE_LANES", str(lanes))
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    s.ipm()
    Q = s.queue(5001, 4096)
    assert len(Q.lanes()) == lanes
    pass_ms, ticks = Q.run(profiled=True)
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, 5001)
    assert Q.finished() == 5001 and Q.idle() and Q.drained() == (0, 0)
    assert ticks >= lanes * int(s.kk.max().item()) and pass_ms[1] > 0.0
    Q.ux.zero_()
    Q.run()  # unprofiled: the results land on the caller's stream (the lanes are joined back into it)
    _queue_equals_batch(s, Q, 5001)


def test_queue_back_to_back_on_two_streams(small_batch):
    """Two queue runs issued back to back from one thread on different streams, without a synchronise in
    between: each call's finished-count polling state is its own, so neither sees the other's count."""
    import torch

    from hpmpc_amd.batch import BatchSolver

    s = BatchSolver(small_batch, k_max=50)
    s.ipm()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    Q1, Q2 = s.queue(97, 16), s.queue(131, 32)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        Q1.run()
    with torch.cuda.stream(s2):
        Q2.run()
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q1, 97)
    _queue_equals_batch(s, Q2, 131)


@pytest.mark.parametrize("shape", ["ms_N30", "tv_N100", "random"])
def test_solo_matches_batch(oracle, shape):
    """The latency path (hpmpc_mi355x_ipm_solo: each problem's whole solve in one launch).
    * HPMPC_MI355X_SOLO=1, the single-wave solo kernel: the batched passes' bodies in one launch, bitwise the batched
      solve (fixed-shape classes and the generic kernels);
    * the default, one problem per four-wave workgroup (hk_ipm_solo_mw): the same routines on the same operands, but
      hipcc contracts a * b + c into FMAs differently once the bodies are split over waves (built with
      -ffp-contract=on the two are bitwise equal, measured), and at mu_tol = 1e-12 the last Newton systems
      (lam / t ~ 1 / mu) lift a last-bit difference to ~1e-9 in pi: identical iteration counts and return codes as
      the batched solve, and every problem held to the CPU oracle at the IPM gate (helpers.compare_ipm) -- except the
      ill-conditioned tv_N100 problem 5 (kk 15), which both kernels meet against the reference's own answer at the
      gate of that problem (4 x the spread of the reference's builds, golden ipm_gate_p5)."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    if shape == "ms_N30":
        qp = mass_spring_qp(30, 8, 3, batch=16, time_variant=True, seed=9)
    elif shape == "tv_N100":
        qp = make_shard(100, 12, 4, 0, 1, 8)
    else:
        from hpmpc_amd.ocp import OCPQP

        one = random_qp(9, [0] + [7] * 9, [3] * 9 + [0], [2] + [5] * 8 + [3], seed=5)
        qp = OCPQP(one.N, one.nx, one.nu, one.nb, one.ng, one.idxb, [a[None].repeat(3, 0) for a in one.BAbt],
                   [a[None].repeat(3, 0) for a in one.RSQrq], [a[None].repeat(3, 0) for a in one.d], [], 3)
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    torch.cuda.synchronize()
    ref = {n: getattr(s, n).clone() for n in ("ux", "pi", "lam", "t", "kk", "ret", "stat")}
    old = os.environ.get("HPMPC_MI355X_SOLO")
    try:
        os.environ["HPMPC_MI355X_SOLO"] = "1"
        for n in ("ux", "pi", "lam", "t"):
            getattr(s, n).zero_()
        s.ipm_solo()
        torch.cuda.synchronize()
        for n, v in ref.items():
            assert torch.equal(getattr(s, n), v), n
        os.environ["HPMPC_MI355X_SOLO"] = "0"
        for n in ("ux", "pi", "lam", "t"):
            getattr(s, n).zero_()
        s.ipm_solo()
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("HPMPC_MI355X_SOLO", None)
        else:
            os.environ["HPMPC_MI355X_SOLO"] = old
    assert torch.equal(s.kk, ref["kk"]) and torch.equal(s.ret, ref["ret"])
    N = qp.N

    def view(src, p):
        g = {n: (src[n].cpu().numpy() if hasattr(src[n], "cpu") else src[n]) for n in ("ux", "pi", "lam", "t", "kk",
                                                                                         "ret")}
        return dict(kk=int(g["kk"][p]), ret=int(g["ret"][p]), ux=[g["ux"][p, k] for k in range(N + 1)],
                    pi=[g["pi"][p, k] for k in range(N)], lam=[g["lam"][p, k] for k in range(N + 1)],
                    t=[g["t"][p, k] for k in range(N + 1)])

    mw = {n: getattr(s, n) for n in ("ux", "pi", "lam", "t", "kk", "ret")}
    for p in range(qp.batch):
        one = qp.problem(p)
        if shape == "tv_N100" and p in GATES:
            # an ill-conditioned problem (kk 15 at mu_tol 1e-12): both kernels against the reference's answer at the
            # gate its own builds set (ipm_gate_p5, make_golden.py gates())
            for src in (ref, mw):
                check_case(GATES[p], view(src, p) | {"stat": GATES[p].out["stat"]})
            continue
        r = oracle.ipm(one, k_max=50)
        div = bool(int(ref["ret"][p]) == 2)
        compare_ipm(one, view(ref, p), r, allow_divergent=div)
        compare_ipm(one, view(mw, p), r, allow_divergent=div)


def test_queue_unconstrained_entries_finish_at_init():
    """nb = 0 problems are solved by one sv inside the refill (kk = 0): the queue drains without
    any iteration doing work."""
    import torch

    from hpmpc_amd.batch import BatchSolver

    qp = mass_spring_qp(20, 8, 3, boxes=False, batch=8, time_variant=True, seed=4)
    s = BatchSolver(qp, k_max=10)
    s.ipm()
    Q = s.queue(40, 4)
    Q.run()
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, 40)
    assert int(Q.kk.max()) == 0


def test_queue_full_size_matches_batch():
    """The benchmark workload (N=100 nx=12 nu=4, 1024 problems) through a queue of two batches."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    qp = make_shard(100, 12, 4, 0, 1, 1024)
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    Q = s.queue(2048)
    _, ticks = Q.run()
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, 2048)
    # two batches back to back would take 2 x 50 iterations; the queue needs far fewer
    assert ticks < 100


def test_queue_drain_matches_oracle(oracle, monkeypatch):
    """The queue's drain: once every entry is handed out and at most HPMPC_MI355X_QUEUE_DRAIN slots still iterate,
    the survivors finish on the multi-wave kernel (one four-wave workgroup each).  The benchmark workload, two batches
    through 2048 slots: every entry's ret equals the batched solve's, entries that never reached the drain are bitwise
    the batched solve, and every entry that finished in the drain (results to rounding: the multi-wave bodies contract
    a few products differently, hk_mw.h) meets the CPU oracle at the IPM gate -- the headline's ill-conditioned
    problems at their reference-spread gates (GATES), the others at max(TOL_IPM, 4 x the oracle's -mfma build spread)
    (the GATES rule), a divergent infeasible draw by ret and kk +-2."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.cabi import HpmpcAPI, load
    from hpmpc_amd.shard import make_shard

    oracle_fma = HpmpcAPI(load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                                            "liboracle_fma.so")), "orc_")
    monkeypatch.setenv("HPMPC_MI355X_QUEUE_DRAIN", "256")
    qp = make_shard(100, 12, 4, 0, 1, 1024)
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    Q = s.queue(2048, 2048)
    pass_ms, ticks = Q.run(profiled=True)
    torch.cuda.synchronize()
    assert len(Q.lanes()) == 2 and Q.finished() == 2048 and Q.idle()
    idx = torch.arange(2048, device=s.ux.device) % 1024
    assert torch.equal(Q.ret, s.ret[idx])
    same = torch.ones(2048, dtype=torch.bool, device=s.ux.device)
    for n in ("ux", "pi", "lam", "t", "kk"):
        a, b = getattr(Q, n), getattr(s, n)[idx]
        same &= (a == b).reshape(2048, -1).all(dim=1)
    drained = [int(q) for q in torch.nonzero(~same).flatten()]
    assert 0 < len(drained) < 400, len(drained)  # the drain ran, on the survivors only
    g = {n: getattr(Q, n).cpu().numpy() for n in ("ux", "pi", "lam", "t", "kk", "ret")}
    for q in drained:
        p = q % 1024
        one = qp.problem(p)
        got = dict(kk=int(g["kk"][q]), ret=int(g["ret"][q]), ux=[g["ux"][q, k] for k in range(101)],
                   pi=[g["pi"][q, k] for k in range(100)], lam=[g["lam"][q, k] for k in range(101)],
                   t=[g["t"][q, k] for k in range(101)])
        if p in GATES:
            c = GATES[p]
            got["stat"] = Q.stat[q].cpu().numpy()[: c.out["stat"].size]
            check_case(c, got)
            continue
        # the GATES rule: max(TOL_IPM, 4 x the oracle's own build spread on this problem) -- the drained problems are
        # the batch's slowest (alpha_min and k_max exits), whose last Newton systems lift last bits the most
        r = oracle.ipm(one.copy(), k_max=50)
        lam_max = max(float(np.max(np.abs(x))) for x in r["lam"])
        if r["ret"] == 1 and lam_max > 1e12:
            # a divergence that runs into k_max before its step length falls below alpha_min (lam ~1e20): as for
            # the ret-2 divergences (helpers.compare_ipm) only the exit is comparable -- same kk (k_max) and ret
            assert (got["kk"], got["ret"]) == (r["kk"], r["ret"]), (p, got["kk"], got["ret"], r["kk"], r["ret"])
            continue
        spread = compare_ipm(one, oracle_fma.ipm(one.copy(), k_max=50), r, tol=float("inf"), allow_divergent=True)
        compare_ipm(one, got, r, tol=max(TOL_IPM, 4 * spread), allow_divergent=True)


def test_gate_problems_every_path():
    """The headline batch's ill-conditioned problems (ipm_gate_* goldens: gate = 4 x the reference builds' spread)
    through the batched passes, the problem queue, the single-wave and the multi-wave solo kernels: identical kk /
    ret and the iterates within each problem's gate of the reference's answer."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.ocp import OCPQP

    cases = list(GATES.values())
    assert cases
    q0 = cases[0].qp
    qs = [c.qp for c in cases]
    qp = OCPQP(q0.N, q0.nx, q0.nu, q0.nb, q0.ng, q0.idxb, [np.stack([q.BAbt[k] for q in qs]) for k in range(q0.N)],
               [np.stack([q.RSQrq[k] for q in qs]) for k in range(q0.N + 1)],
               [np.stack([q.d[k] for q in qs]) for k in range(q0.N + 1)], [], len(qs))
    s = BatchSolver(qp, k_max=50)

    def check(src):
        g = {n: getattr(src, n).cpu().numpy() for n in ("ux", "pi", "lam", "t", "kk", "ret", "stat")}
        for p, c in enumerate(cases):
            got = dict(kk=int(g["kk"][p]), ret=int(g["ret"][p]), ux=[g["ux"][p, k] for k in range(q0.N + 1)],
                       pi=[g["pi"][p, k] for k in range(q0.N)], lam=[g["lam"][p, k] for k in range(q0.N + 1)],
                       t=[g["t"][p, k] for k in range(q0.N + 1)], stat=g["stat"][p][: c.out["stat"].size])
            check_case(c, got)

    s.ipm()
    torch.cuda.synchronize()
    check(s)
    Q = s.queue(3 * len(cases), 4)
    Q.run()
    torch.cuda.synchronize()
    _queue_equals_batch(s, Q, 3 * len(cases))
    old = os.environ.get("HPMPC_MI355X_SOLO")
    try:
        for mode in ("1", "0"):
            os.environ["HPMPC_MI355X_SOLO"] = mode
            for n in ("ux", "pi", "lam", "t"):
                getattr(s, n).zero_()
            s.ipm_solo()
            torch.cuda.synchronize()
            check(s)
    finally:
        if old is None:
            os.environ.pop("HPMPC_MI355X_SOLO", None)
        else:
            os.environ["HPMPC_MI355X_SOLO"] = old


def test_aliased_batch_layout(oracle):
    """The time-invariant / aliased batched mode (hpmpc_mi355x_layout BAbt_shared / RSQrq_shared): problems that
    differ only in x0 (stage 0's b row) read ONE copy of every other stage block, and every inner stage the same
    block (test_d_ip_hard.c:652-662).  Same data, same operations: the IPM (batch and queue) and the Riccati sv are
    bitwise those of the unaliased layout, and the oracle agrees problem by problem."""
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    qp = make_shard(40, 12, 4, 0, 1, 24, time_variant=False)
    full = BatchSolver(qp, k_max=50)
    al = BatchSolver(qp, k_max=50, aliased=True)
    assert al.BAbt.numel() < full.BAbt.numel() // 10 and al.RSQrq.numel() * 20 < full.RSQrq.numel()
    for s in (full, al):
        s.ipm()
    torch.cuda.synchronize()
    for n in ("ux", "pi", "lam", "t", "kk", "ret", "stat"):
        assert torch.equal(getattr(full, n), getattr(al, n)), n
    Q = al.queue(60, 16)
    Q.run()
    torch.cuda.synchronize()
    _queue_equals_batch(full, Q, 60)
    for p in (0, 7, 23):
        one = qp.problem(p)
        got = dict(kk=int(al.kk[p]), ret=int(al.ret[p]), ux=[al.ux[p, k].cpu().numpy() for k in range(41)],
                   pi=[al.pi[p, k].cpu().numpy() for k in range(40)], lam=[al.lam[p, k].cpu().numpy() for k in range(41)],
                   t=[al.t[p, k].cpu().numpy() for k in range(41)])
        compare_ipm(one, got, oracle.ipm(one.copy(), k_max=50), allow_divergent=True)
    qr = make_shard(40, 12, 4, 0, 1, 24, boxes=False, time_variant=False)
    f2, a2 = BatchSolver(qr, k_max=1), BatchSolver(qr, k_max=1, aliased=True)
    for s in (f2, a2):
        s.ric_sv(compute_pi=1, compute_Pb=1)
    torch.cuda.synchronize()
    for n in ("ux", "pi", "Pb"):
        assert torch.equal(getattr(f2, n), getattr(a2, n)), n


@pytest.mark.parametrize("N", [300, 301])
def test_solo_long_horizons(oracle, N):
    """The latency path at the multi-wave kernel's horizon limit (MW_NMAX = 300: the update's reduction rows fill its
    LDS buffer exactly) and one stage beyond it (N = 301: the single-wave solo kernel takes over).  Same kk / ret as the
    batched solve, bitwise equal to it beyond the limit, and both at the IPM gate of the oracle."""
    import torch

    from hpmpc_amd.batch import BatchSolver

    qp = mass_spring_qp(N, 8, 3, batch=2, time_variant=True, seed=N)
    s = BatchSolver(qp, k_max=50)
    s.ipm()
    torch.cuda.synchronize()
    ref = {n: getattr(s, n).clone() for n in ("ux", "pi", "lam", "t", "kk", "ret")}
    for n in ("ux", "pi", "lam", "t"):
        getattr(s, n).zero_()
    s.ipm_solo()
    torch.cuda.synchronize()
    assert torch.equal(s.kk, ref["kk"]) and torch.equal(s.ret, ref["ret"])
    if N > 300:
        for n, v in ref.items():
            assert torch.equal(getattr(s, n), v), n
    for p in range(2):
        one = qp.problem(p)
        r = oracle.ipm(one.copy(), k_max=50)
        got = dict(kk=int(s.kk[p]), ret=int(s.ret[p]), ux=[s.ux[p, k].cpu().numpy() for k in range(N + 1)],
                   pi=[s.pi[p, k].cpu().numpy() for k in range(N)], lam=[s.lam[p, k].cpu().numpy() for k in range(N + 1)],
                   t=[s.t[p, k].cpu().numpy() for k in range(N + 1)])
        compare_ipm(one, got, r, allow_divergent=True)


def test_multiwave_expired_wait_drains():
    """The multi-wave kernel's expired-wait path (hk_mw.h mw_wait_at): in the diagnostic build
    (libhpmpc_mi355x_stamps.so, -DHK_STAMPS) with HPMPC_MI355X_MW_FAULT=1 a helper drops one hand-over; the waits
    expire after ~2^22 polls, every later wait falls through, the launch drains and the problem reports
    ret = -20 (HPMPC_MI355X_EMW), and the drop-in entry point returns -20 with hpmpc_mi355x_last_error() set and its
    outputs untouched.  Run in a child process (the library path is chosen at import)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "hpmpc_amd", "lib", "libhpmpc_mi355x_stamps.so")
    assert os.path.exists(lib), "diagnostic build missing (hpmpc_amd/build.py build_stamps, run by build())"
    code = r"""
import numpy as np, torch
from hpmpc_amd.batch import BatchSolver, LIBPATH
from hpmpc_amd.cabi import HpmpcAPI, load
from hpmpc_amd.ocp import mass_spring_qp
qp = mass_spring_qp(30, 8, 3, batch=2, time_variant=True, seed=3)
s = BatchSolver(qp, k_max=50)
s.ipm_solo()
torch.cuda.synchronize()
assert s.ret.cpu().tolist() == [-20, -20], s.ret
api = HpmpcAPI(load(LIBPATH))
r = api.ipm(qp.problem(0), k_max=50)
assert r["ret"] == -20 and api.lib.hpmpc_mi355x_last_error() == -20, r["ret"]
assert all(not np.any(u) for u in r["ux"])
print("drained")
"""
    env = dict(os.environ, HPMPC_MI355X_LIB=lib, HPMPC_MI355X_MW_FAULT="1", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0 and "drained" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
