#!/usr/bin/env python3
"""Generate the golden vectors of tests/golden/*.npz from the REAL reference c99 build.

The reference (oracle/_ref/libhpmpc_ref.so, compiled from the sources under /root/reference by
oracle/Makefile, TARGET_C99_4X4, no BLASFEO) is called through its own C entry points on
deterministic inputs; inputs and outputs are stored as plain float64/int32 arrays (no pickles).
This script needs the dev container (the reference source tree); the committed .npz files are what
the tests read everywhere else.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from hpmpc_amd.cabi import HpmpcAPI, bq_from_qp, load  # noqa: E402
from hpmpc_amd.golden import save_case  # noqa: E402
from hpmpc_amd.ocp import (BS, OCPQP, lib4_size, mass_spring_qp, pack_lib4, rup,  # noqa: E402
                           unpack_lib4)

sys.path.insert(0, os.path.dirname(HERE))
from helpers import COND_FILL, parse_ric_driver, sub_block, xclamp_qp  # noqa: E402


def ref_api():
    path = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref.so")
    return HpmpcAPI(load(path))


def ref_avx_api():
    """The reference's default-target (X64_AVX) build of the alternate IPM (oracle/Makefile ref_avx): its
    d_kkt_solve_new_rhs_mpc_hard_tv binds the 9-parameter avx gradient helper.  Aligned marshalling."""
    path = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref_avx.so")
    return HpmpcAPI(load(path), aligned=True)


def rand_vecs(rng, sizes, pad=4, scale=1.0):
    return [np.concatenate([scale * rng.standard_normal(n), np.zeros(pad + (4 - n % 4) % 4)]) for n in sizes]


def clamp_qp(N=10, nx=8, nu=3):
    """Singular R and Q blocks: exercises the pivot clamp (kernel_dpotrf_c99_lib4.c:555-640)."""
    qp = mass_spring_qp(N, nx, nu, boxes=False)
    for k in range(N + 1):
        nux = qp.nux(k)
        M = unpack_lib4(qp.RSQrq[k], nux + 1, nux).copy()
        nuk = int(qp.nu[k])
        if nuk > 1:
            M[1, :] = 0.0
            M[:, 1] = 0.0
        if k == N:
            M[0, :] = 0.0
            M[:, 0] = 0.0
        qp.RSQrq[k] = pack_lib4(M)
    return qp


def x0_stage_qp(N=10, nx=8, nu=3):
    """nx[0] = nx (x0 kept as a variable): stage 0 is solved over the whole nux block."""
    base = mass_spring_qp(N, nx, nu, boxes=False)
    qp = base.copy()
    A = unpack_lib4(base.BAbt[1], nu + nx + 1, nx)
    qp.nx = base.nx.copy()
    qp.nx[0] = nx
    qp.BAbt[0] = base.BAbt[1].copy()
    qp.BAbt[0] = pack_lib4(A)
    qp.RSQrq[0] = base.RSQrq[1].copy()
    return qp


def ng_qp(N=30, nx=8, nu=3):
    """Terminal general constraints (ngN = nx, x_N in [-0.5, 0.5] via C = I), like the user guide's ngN example."""
    qp = mass_spring_qp(N, nx, nu, boxes=True)
    qp.ng = np.zeros(N + 1, dtype=np.int32)
    qp.ng[N] = nx
    qp.DCt = [np.zeros(8) for _ in range(N + 1)]
    qp.DCt[N] = pack_lib4(np.eye(nx))
    for k in range(N + 1):
        pnb, png = qp.pnb(k), qp.png(k)
        dk = np.zeros(2 * pnb + 2 * png)
        dk[: 2 * pnb] = qp.d[k][: 2 * pnb]
        if k == N:
            dk[2 * pnb: 2 * pnb + nx] = -0.5
            dk[2 * pnb + png: 2 * pnb + png + nx] = 0.5
        qp.d[k] = dk
    return qp


def main():
    ref = ref_api()
    rng = np.random.default_rng(20261015)
    out = []

    # ---------------- d_back_ric_rec_sv_tv_res ----------------
    for (N, nx, nu) in [(10, 8, 3), (30, 8, 3), (50, 8, 3), (100, 12, 4)]:
        qp = mass_spring_qp(N, nx, nu, boxes=False)
        ux, pi, Pb, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
        out.append(save_case(f"sv_ms_N{N}_nx{nx}_nu{nu}", "sv", qp, dict(compute_pi=1, compute_Pb=1),
                             dict(ux=ux, pi=pi, Pb=Pb)))
    qp = mass_spring_qp(20, 12, 4, boxes=False, batch=1, time_variant=True, seed=7).problem(0)
    ux, pi, Pb, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
    out.append(save_case("sv_tv_N20_nx12_nu4", "sv", qp, dict(compute_pi=1, compute_Pb=1), dict(ux=ux, pi=pi, Pb=Pb)))

    qp = clamp_qp()
    ux, pi, Pb, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
    out.append(save_case("sv_clamp_N10_nx8_nu3", "sv", qp, dict(compute_pi=1, compute_Pb=1), dict(ux=ux, pi=pi, Pb=Pb)))

    qp = x0_stage_qp()
    ux, pi, Pb, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
    out.append(save_case("sv_x0_N10_nx8_nu3", "sv", qp, dict(compute_pi=1, compute_Pb=1), dict(ux=ux, pi=pi, Pb=Pb)))

    # sv with update_b / update_q / box terms: also pins the in-place side effects on the caller's data
    qp = mass_spring_qp(10, 8, 3, boxes=True)
    N = qp.N
    b = rand_vecs(rng, [int(qp.nx[k + 1]) for k in range(N)])
    q = rand_vecs(rng, [qp.nux(k) for k in range(N + 1)])
    bd = [np.concatenate([1.0 + rng.random(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    Qx = [np.concatenate([0.5 + rng.random(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    qx = [np.concatenate([rng.standard_normal(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    q2 = qp.copy()
    ux, pi, Pb, _ = ref.ric_sv(q2, update_b=1, b=b, update_q=1, q=q, bd=bd, Qx=Qx, qx=qx, compute_pi=1,
                               compute_Pb=1)
    out.append(save_case("sv_update_box_N10_nx8_nu3", "sv", qp,
                         dict(compute_pi=1, compute_Pb=1, update_b=1, update_q=1),
                         dict(ux=ux, pi=pi, Pb=Pb, BAbt_after=q2.BAbt, RSQrq_after=q2.RSQrq),
                         extra=dict(b=b, q=q, bd=bd, Qx=Qx, qx=qx)))

    # ---------------- trf + trs ----------------
    qp = mass_spring_qp(30, 8, 3, boxes=True)
    N = qp.N
    b = rand_vecs(rng, [int(qp.nx[k + 1]) for k in range(N)])
    q = rand_vecs(rng, [qp.nux(k) for k in range(N + 1)])
    bd = [np.concatenate([1.0 + rng.random(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    Qx = [np.concatenate([0.5 + rng.random(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    qx = [np.concatenate([rng.standard_normal(int(qp.nb[k])), np.zeros(8)]) for k in range(N + 1)]
    q2 = qp.copy()
    mem = ref.ric_trf(q2, bd=bd, Qx=Qx)
    ux, pi, Pb = ref.ric_trs(q2, mem, b=b, q=q, qx=qx, compute_pi=1, compute_Pb=1)
    out.append(save_case("trf_trs_N30_nx8_nu3", "trf_trs", qp, dict(compute_pi=1, compute_Pb=1),
                         dict(ux=ux, pi=pi, Pb=Pb), extra=dict(b=b, q=q, bd=bd, Qx=Qx, qx=qx)))

    # ---------------- d_ip2_res_mpc_hard_tv ----------------
    for (N, nx, nu) in [(10, 8, 3), (30, 8, 3), (100, 12, 4)]:
        qp = mass_spring_qp(N, nx, nu, boxes=True)
        r = ref.ipm(qp.copy(), k_max=50)
        out.append(save_case(f"ipm_N{N}_nx{nx}_nu{nu}", "ipm", qp, dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                             dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                                  ret=r["ret"])))
    bq = mass_spring_qp(30, 12, 4, boxes=True, batch=4, time_variant=True, seed=11)
    for p in range(4):
        qp = bq.problem(p)
        r = ref.ipm(qp.copy(), k_max=50)
        out.append(save_case(f"ipm_tv_N30_nx12_nu4_p{p}", "ipm", qp,
                             dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                             dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                                  ret=r["ret"])))
    # warm start
    qp = mass_spring_qp(20, 8, 3, boxes=True)
    ux0 = rand_vecs(rng, [qp.nux(k) for k in range(qp.N + 1)], scale=0.1)
    r = ref.ipm(qp.copy(), k_max=50, warm_start=1, ux=ux0)
    out.append(save_case("ipm_warm_N20_nx8_nu3", "ipm", qp,
                         dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=1),
                         dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                              ret=r["ret"]), extra=dict(ux0=ux0)))
    # no constraints: mu_scal == 0 -> one sv (d_ip2_res_hard.c:428-450)
    qp = mass_spring_qp(20, 8, 3, boxes=False)
    r = ref.ipm(qp.copy(), k_max=50)
    out.append(save_case("ipm_noconstr_N20_nx8_nu3", "ipm", qp, dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                         dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                              ret=r["ret"])))
    # k_max reached (ret 1)
    qp = mass_spring_qp(30, 8, 3, boxes=True)
    r = ref.ipm(qp.copy(), k_max=4)
    out.append(save_case("ipm_kmax4_N30_nx8_nu3", "ipm", qp, dict(k_max=4, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                         dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                              ret=r["ret"])))
    # general constraints (oracle-only row: GPU path returns EUNSUPPORTED)
    qp = ng_qp()
    r = ref.ipm(qp.copy(), k_max=50)
    out.append(save_case("ipm_ng_N30_nx8_nu3", "ipm", qp, dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                         dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                              ret=r["ret"])))

    # ---------------- KKT re-solve + residuals + single Newton step ----------------
    qp = mass_spring_qp(30, 8, 3, boxes=True)
    r = ref.ipm(qp.copy(), k_max=50)
    b, q = bq_from_qp(qp)
    b2 = [x + 0.01 * rng.standard_normal(x.shape) for x in b]
    q2v = [x + 0.01 * rng.standard_normal(x.shape) for x in q]
    kk = ref.kkt_new_rhs(qp.copy(), r["work"], b2, q2v)
    out.append(save_case("kkt_N30_nx8_nu3", "kkt", qp, dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8),
                         dict(ux=kk["ux"], pi=kk["pi"], lam=kk["lam"], t=kk["t"]), extra=dict(b2=b2, q2=q2v)))
    uxp = [x + 0.01 * rng.standard_normal(x.shape) for x in r["ux"]]
    pip = [x + 0.01 * rng.standard_normal(x.shape) for x in r["pi"]]
    res = ref.residuals(qp.copy(), b, q, uxp, pip, r["lam"], r["t"])
    out.append(save_case("res_N30_nx8_nu3", "res", qp, {},
                         dict(rq=res["rq"], rb=res["rb"], rd=res["rd"], rm=res["rm"], mu=res["mu"]),
                         extra=dict(b=b, q=q, ux=uxp, pi=pip, lam=r["lam"], t=r["t"])))
    qp = mass_spring_qp(10, 8, 3, boxes=True)
    r = ref.ipm(qp.copy(), k_max=50)
    # interior starting point (t, lam away from 0) so the single Newton step is well conditioned
    lam0, t0 = [], []
    for k in range(qp.N + 1):
        nb = int(qp.nb[k])
        lam0.append(np.concatenate([1.0 + 0.1 * rng.random(2 * nb), np.zeros(4)]))
        t0.append(np.concatenate([0.5 + 0.1 * rng.random(2 * nb), np.zeros(4)]))
    ux0 = [0.9 * x for x in r["ux"]]
    pi0 = [0.9 * x for x in r["pi"]]
    sn = ref.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=1, mu0=0.1)
    out.append(save_case("newton_N10_nx8_nu3", "newton", qp, dict(k_max=1, mu0=0.1, mu_tol=1e-12, alpha_min=1e-8),
                         dict(ux=sn["ux"], pi=sn["pi"], lam=sn["lam"], t=sn["t"], stat=sn["stat"], kk=sn["kk"],
                              ret=sn["ret"]), extra=dict(ux0=ux0, pi0=pi0, lam0=lam0, t0=t0)))
    # ---------------- alternate IPM: d_ip2_mpc_hard_tv, d_kkt_solve_new_rhs_mpc_hard_tv, d_res_mpc_hard_tv ----
    alt(ref, ref_avx_api(), rng, out)
    pcond(ref, out)
    cond_parts(ref, out)
    xclamp(ref, out)
    gates(ref, out)
    xclamp_ipm(ref, out)
    soft_res(ref, out)
    iface(ref, out)
    iface_soft(ref, out)
    iface_mpc(ref, ref_avx_api(), out)
    wide(ref, ref_avx_api(), out)
    divergent(ref, out)
    driver(out)
    total = sum(os.path.getsize(p) for p in out)
    print(f"wrote {len(out)} cases, {total / 1e6:.2f} MB")


def alt(ref, refa, rng, out):
    """Cases of the alternate (phase-1 only) IPM of mpc_solvers/d_ip2_hard.c and its residuals."""
    def ipm_out(r):
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])

    cases = [("ms_N30_nx8_nu3", mass_spring_qp(30, 8, 3, boxes=True)), ("ng_N30_nx8_nu3", ng_qp())]
    for name, qp in cases:
        for tag, kw in (("tol1e-8", dict(mu_tol=1e-8)), ("kmax4", dict(k_max=4)), ("tol1e-12", dict(mu_tol=1e-12))):
            args = dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8)
            args.update(kw)
            r = ref.ipm(qp.copy(), res=False, **args)
            out.append(save_case(f"ipm2_{tag}_{name}", "ipm2", qp, args, ipm_out(r)))
    qp = mass_spring_qp(20, 8, 3, boxes=False)  # no constraints: sv into the workspace, outputs untouched
    args = dict(k_max=50, mu0=2.0, mu_tol=1e-8, alpha_min=1e-8)
    out.append(save_case("ipm2_noconstr_N20_nx8_nu3", "ipm2", qp, args, ipm_out(ref.ipm(qp.copy(), res=False, **args))))
    qp = mass_spring_qp(30, 12, 4, boxes=True, batch=1, time_variant=True, seed=5).problem(0)
    args = dict(k_max=50, mu0=2.0, mu_tol=1e-8, alpha_min=1e-8)
    out.append(save_case("ipm2_tv_N30_nx12_nu4", "ipm2", qp, args, ipm_out(ref.ipm(qp.copy(), res=False, **args))))

    for name, qp in cases + [("noconstr_N20_nx8_nu3", mass_spring_qp(20, 8, 3, boxes=False))]:
        args = dict(k_max=50, mu0=2.0, mu_tol=1e-8, alpha_min=1e-8)
        r = refa.ipm(qp.copy(), res=False, **args)
        b, q = bq_from_qp(qp)
        b2 = [x + 0.01 * rng.standard_normal(x.shape) for x in b]
        q2 = [x + 0.01 * rng.standard_normal(x.shape) for x in q]
        d2 = [x + 0.01 * rng.standard_normal(x.shape) for x in qp.d]
        k = refa.kkt_new_rhs_plain(qp.copy(), r["work"], b2, q2, d2, r["ux"])
        out.append(save_case(f"kkt2_{name}", "kkt2", qp, args, dict(ux=k["ux"], pi=k["pi"], lam=k["lam"], t=k["t"]),
                             extra=dict(b2=b2, q2=q2, d2=d2)))
        uxp = [x + 0.01 * rng.standard_normal(x.shape) for x in r["ux"]]
        pip = [x + 0.01 * rng.standard_normal(x.shape) for x in r["pi"]]
        res = ref.residuals_plain(qp.copy(), b, q, uxp, pip, r["lam"], r["t"])
        out.append(save_case(f"res2_{name}", "res2", qp, {}, dict(rq=res["rq"], rb=res["rb"], rd=res["rd"], mu=res["mu"]),
                             extra=dict(b=b, q=q, ux=uxp, pi=pip, lam=r["lam"], t=r["t"])))


def pcond(ref, out):
    """Partial condensing (lqcp_solvers/d_part_cond.c): d_part_cond outputs and d_part_expand_solution of random
    condensed-space vectors, on cases where the reference c99 build is right (nu <= 4: for nu > 4 its condensed
    Hessian is wrong past the 4th column of each inner u block); the C5 workload (nu = 6) is pinned
    by the reference's direct Riccati solution instead (kind pcond_sv: condense -> sv -> expand == direct sv)."""
    rng = np.random.default_rng(20261016)
    for (N, nx, nu, N2, boxes) in [(20, 8, 3, 4, False), (20, 8, 3, 4, True), (23, 6, 2, 5, True),
                                   (30, 24, 4, 3, True), (12, 4, 1, 12, True), (9, 8, 4, 2, True)]:
        qp = mass_spring_qp(N, nx, nu, boxes=boxes)
        c, _ = ref.part_cond(qp.copy(), N2)
        u2 = rand_vecs(rng, [c.nux(k) for k in range(N2 + 1)])
        p2 = rand_vecs(rng, [int(c.nx[k + 1]) for k in range(N2)])
        lam2 = [np.abs(x) for x in rand_vecs(rng, [c.nconstr(k) for k in range(N2 + 1)])]
        t2 = [np.abs(x) for x in rand_vecs(rng, [c.nconstr(k) for k in range(N2 + 1)])]
        e = ref.part_expand(qp, c, u2, p2, lam2, t2)
        outs = dict(BAbt2=c.BAbt, RSQrq2=c.RSQrq[:N2], DCt2=c.DCt[:N2] if c.DCt else [], d2=c.d[:N2],
                    idxb2=[i.astype(np.float64) for i in c.idxb[:N2]], nx2=c.nx, nu2=c.nu, nb2=c.nb, ng2=c.ng,
                    ux=e["ux"], pi=e["pi"], lam=e["lam"], t=e["t"])
        tag = "box" if boxes else "ms"
        out.append(save_case(f"pcond_{tag}_N{N}_nx{nx}_nu{nu}_N2_{N2}", "pcond", qp, dict(N2=N2), outs,
                             extra=dict(u2=u2, p2=p2, lam2=lam2, t2=t2)))
    for (N, nx, nu, N2) in [(200, 24, 6, 20), (40, 12, 6, 8)]:
        qp = mass_spring_qp(N, nx, nu, boxes=False)
        ux, pi, _, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=0)
        out.append(save_case(f"pcond_sv_N{N}_nx{nx}_nu{nu}_N2_{N2}", "pcond_sv", qp, dict(N2=N2), dict(ux=ux, pi=pi)))


def cond_parts(ref, out):
    """The building blocks of one condensing block alone (d_part_cond.c:214-689): d_cond_BAbt, then d_cond_RSQrq
    and d_cond_DCtd on the reference's own Gammas, outputs pre-filled with COND_FILL.  Blocks cut from
    time-variant boxed mass-spring problems, first block (nx_0 = 0) and inner ones, T = 1 .. 10, nu <= 4 (the c99
    build's RSQrq is wrong for nu > 4)."""
    for (N, nx, nu, s0, T) in [(12, 8, 3, 3, 5), (8, 12, 4, 0, 4), (6, 6, 2, 2, 1), (24, 24, 4, 10, 10),
                               (6, 4, 1, 1, 3), (9, 8, 3, 0, 9)]:
        qp = mass_spring_qp(N, nx, nu, boxes=True, batch=1, time_variant=True, seed=100 + N).problem(0)
        b = sub_block(qp, s0, T)
        G, B2 = ref.cond_BAbt(b.copy(), fill=COND_FILL)
        R2 = ref.cond_RSQrq(b.copy(), G, fill=COND_FILL)
        DCt2, d2, idxb2, (nbb, nbg) = ref.cond_DCtd(b.copy(), G, fill=COND_FILL)
        outs = dict(Gamma=G, BAbt2=B2, RSQrq2=R2, DCt2=DCt2, d2=d2, idxb2=idxb2.astype(np.float64), nbb=nbb, nbg=nbg)
        out.append(save_case(f"cond_parts_N{N}_s{s0}_T{T}_nx{nx}_nu{nu}", "cond_parts", b, dict(fill=COND_FILL),
                             outs))


def xclamp(ref, out):
    """The reference clamping an inner-stage x pivot (kernel_dpotrf_c99_lib4.c:555-640): helpers.xclamp_qp puts
    an exact pivot d <= 1e-15 with nonzero cross terms on state 0 of every stage k >= 1.  The clamp zeroes that
    column of Lxx, so the cost-to-go the reference carries loses the pivot's rank-one term (entries d and `off`:
    solution change ~off) and, through l_x, the gradient along it (change ~r).  The product's stages fail the clamp
    certificate there and are factorised as the reference does (kind sv_xclamp, DESIGN.md, pivot clamp)."""
    for name, kw in (("r0", dict(d=1e-16, off=1e-9, r=0.0)), ("r05", dict(d=1e-16, off=1e-9, r=0.5))):
        qp = xclamp_qp(**kw)
        ux, pi, Pb, _ = ref.ric_sv(qp.copy(), compute_pi=1, compute_Pb=1)
        out.append(save_case(f"sv_xclamp_{name}_N10_nx8_nu3", "sv_xclamp", qp, dict(compute_pi=1, compute_Pb=1, **kw),
                             dict(ux=ux, pi=pi, Pb=Pb)))


def xclamp_ipm(ref, out):
    """The clamp problems inside the IPM (tests/test_gpu_parity.py XCLAMP, N=20 with boxes): the c99 answer and the
    reference builds' spread (c99, c99 + FMA, X64_AVX, X64_AVX2), stored as a gated golden for every variant whose
    builds spread by more than TOL_IPM / 4 (the GATES rule of gates(): gate = max(1e-10, 4 x spread)).  ADVICE r4: the
    gate of the one non-converging variant was a hand-measured constant in the test."""
    from helpers import XCLAMP

    others = x64_apis()
    for d, off, r in XCLAMP:
        one = xclamp_qp(N=20, nx=8, nu=3, d=d, off=off, r=r, boxes=True)
        rs = {"c99": ref.ipm(one.copy(), k_max=50)}
        rs.update({n: api.ipm(one.copy(), k_max=50) for n, api in others.items()})
        sp, ds = build_spread(one, rs)
        print(f"  xclamp d={d:g} off={off:g} r={r:g}: kk {rs['c99']['kk']} ret {rs['c99']['ret']}, build spread "
              f"{sp:.2e} (stat {ds:.2e})")
        if not 4 * sp > 1e-10:
            continue
        c = rs["c99"]
        args = dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, xclamp_d=d, xclamp_off=off, xclamp_r=r, spread=sp,
                    gate=max(1e-10, 4 * sp), stat_gate=max(1e-9, 4 * ds))
        out.append(save_case(f"ipm_xclamp_d{d:g}_off{off:g}_r{r:g}_N20_nx8_nu3", "ipm", one, args,
                             dict(ux=c["ux"], pi=c["pi"], lam=c["lam"], t=c["t"], stat=c["stat"], kk=c["kk"],
                                  ret=c["ret"])))


def x64_apis():
    """The reference's x86 targets (oracle/Makefile ref_x64: X64_AVX, its default, and X64_AVX2) and the c99 sources
    rebuilt with -mfma -ffp-contract=fast (ref_fma): other builds of the same reference, other summation orders."""
    r = os.path.join(ROOT, "oracle", "_ref")
    return {"fma": HpmpcAPI(load(os.path.join(r, "libhpmpc_ref_fma.so"))),
            "avx": HpmpcAPI(load(os.path.join(r, "libhpmpc_ref_x64avx.so")), aligned=True),
            "avx2": HpmpcAPI(load(os.path.join(r, "libhpmpc_ref_x64avx2.so")), aligned=True)}


GATE_BATCH = 1024


def build_spread(one, rs):
    """Diameter of the reference builds' IPM answers on one problem: max over build pairs of the compare_ipm distance
    (ux, pi, lam, t relative to max(1, |.|)) and of the stat entries' relative distance (beyond the 1e-14 absolute
    allowance of the stat check); inf when two builds disagree on kk / ret."""
    from helpers import compare_ipm

    names, d, ds = list(rs), 0.0, 0.0
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            a, b = rs[names[i]], rs[names[j]]
            if a["kk"] != b["kk"] or a["ret"] != b["ret"]:
                return float("inf"), float("inf")
            d = max(d, compare_ipm(one, a, b, tol=1e300))
            sa, sb = np.asarray(a["stat"]), np.asarray(b["stat"])
            nz = np.abs(sb) > 0
            ds = max(ds, float(np.max((np.abs(sa - sb)[nz] - 1e-14) / np.abs(sb[nz]), initial=0.0)))
    return d, ds


def gates(ref, out):
    """Per-problem IPM gates for the ill-conditioned problems of the headline batch (make_shard(100, 12, 4, 0, 1,
    1024), global problem ids 0..1023): every converged problem whose reference builds (c99 = the goldens, c99 with
    FMA contraction, the X64_AVX and X64_AVX2 targets) spread by more than TOL_IPM / 4.  Such a problem ends in
    Newton systems at complementarity mu ~ 1e-12 that lift last-bit differences to ~1e-9 in the reference itself,
    so its gate is max(1e-10, 4 x that spread) (stat: max(1e-9, 4 x its spread)), stored in the golden with the c99
    answer; every other problem of the batch meets 1e-10 across the builds."""
    from hpmpc_amd.shard import make_shard

    others = x64_apis()
    qp = make_shard(100, 12, 4, 0, 1, GATE_BATCH)
    for p in range(GATE_BATCH):
        one = qp.problem(p)
        rs = {"c99": ref.ipm(one.copy(), k_max=50)}
        if rs["c99"]["ret"] != 0:
            continue
        rs.update({n: api.ipm(one.copy(), k_max=50) for n, api in others.items()})
        d, ds = build_spread(one, rs)
        if not 4 * d > 1e-10:
            continue
        r = rs["c99"]
        args = dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, problem=p, spread=d, gate=max(1e-10, 4 * d),
                    stat_gate=max(1e-9, 4 * ds))
        out.append(save_case(f"ipm_gate_p{p}_N100_nx12_nu4", "ipm", one, args,
                             dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                                  ret=r["ret"])))
        print(f"  p{p}: kk {r['kk']}, build spread {d:.2e} (stat {ds:.2e}) -> gate {max(1e-10, 4 * d):.2e}")


def soft_res(ref, out):
    """d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38) at random iterates (t, lam > 0) of soft problems: the
    driver's shape (nb = nu: the soft index idxb[nu + i] is the soft box), hard boxes at stage N (nu_N = 0: the
    soft index reads the hard entries, as the reference does), and general constraints on the inner stages."""
    from hpmpc_amd.soft import mass_spring_soft

    rng = np.random.default_rng(20261017)

    def with_general(sq, ng=2):
        sq.ng = np.array([0] + [ng] * (sq.N - 1) + [0], dtype=np.int32)
        sq.DCt = [np.zeros(8)] * (sq.N + 1)
        for k in range(1, sq.N):
            nb, ns, pnb, pns, png = int(sq.nb[k]), int(sq.ns[k]), rup(int(sq.nb[k]), 4), rup(int(sq.ns[k]), 4), rup(ng, 4)
            sq.DCt[k] = pack_lib4(rng.standard_normal((sq.nux(k), ng)))
            d = np.zeros(2 * pnb + 2 * png + 2 * pns + 4)
            d[:2 * pnb] = sq.d[k][:2 * pnb]
            d[2 * pnb:2 * pnb + ng] = -1.0
            d[2 * pnb + png:2 * pnb + png + ng] = 1.0
            d[2 * pnb + 2 * png:2 * pnb + 2 * png + 2 * pns] = sq.d[k][2 * pnb:2 * pnb + 2 * pns]
            sq.d[k] = d
        return sq

    cases = [("ms_N10_nx8_nu3", mass_spring_soft(10, 8, 3, Q_diag=1.0, Zq=0.5)),
             ("hardN_N12_nx8_nu2", mass_spring_soft(12, 8, 2, hard_last=2, time_variant=True, seed=3)),
             ("ng_N8_nx6_nu2", with_general(mass_spring_soft(8, 6, 2, Q_diag=0.5)))]
    for name, sq in cases:
        N = sq.N
        ux, pi, lam, t = sq.alloc_solution()
        for k in range(N + 1):
            ux[k][:sq.nux(k)] = rng.standard_normal(sq.nux(k))
            lam[k][:sq.ncv(k)] = 0.1 + rng.random(sq.ncv(k))
            t[k][:sq.ncv(k)] = 0.1 + rng.random(sq.ncv(k))
            if k < N:
                pi[k][:int(sq.nx[k + 1])] = rng.standard_normal(int(sq.nx[k + 1]))
        q = [np.concatenate([rng.standard_normal(sq.nux(k)), np.zeros(8)]) for k in range(N + 1)]
        r = ref.residuals_soft(sq.copy(), q, ux, pi, lam, t)
        out.append(save_case(f"softres_{name}", "soft_res", sq, {}, dict(rq=r["rq"], rb=r["rb"], rd=r["rd"],
                             rz=r["rz"], mu=r["mu"]), extra=dict(ns=[sq.ns.astype(np.float64)], Z=sq.Z, z=sq.z, q=q,
                                                                  ux=ux, pi=pi, lam=lam, t=t)))


def iface(ref, out):
    """High-level wrappers of include/c_interface.h, restated by oracle/iface_oracle.py over the reference's own
    low-level entry points (the reference wrapper sources need the generated include/target.h and are
    unbuildable here): full space, partially condensed, stage-0 state as a variable with general constraints at
    N, the cost-based mu0, and the KKT re-solve with new right-hand sides."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import iface_oracle as IO

    cases = [("full_N10_nx4_nu2", (10, [0] + [4] * 10, [2] * 10, 2, 2, None, 0), 10, 2.0),
             ("cond_N12_nx4_nu1_N2_4", (12, [0] + [4] * 12, [1] * 12, 1, 2, None, 1), 4, 2.0),
             ("x0var_ngN_N8_nx3_nu2", (8, [3] * 9, [2] * 8, 1, 1, [0] * 8 + [2], 2), 8, 2.0),
             ("automu0_N15_nx6_nu3", (15, [0] + [6] * 15, [3] * 15, 3, 3, None, 3), 15, -1.0)]
    for name, (N, nx, nu, bu, bx, ng, seed), N2, mu0 in cases:
        P = IO.random_iface_problem(N, nx, nu, bu, bx, ng, seed=seed)
        r = IO.ip_ocp(ref, P, N2, k_max=50, mu0=mu0, mu_tol=1e-10)
        qp = IO.to_qp(P)
        outs = dict(u=r["u"], x=r["x"], pi=r["pi"], lam=r["lam"], inf_norm_res=r["inf_norm_res"], kk=r["kk"],
                    ret=r["status"], stat=r["stat"])
        out.append(save_case(f"iface_{name}", "iface", qp, dict(N2=N2, mu0=mu0, mu_tol=1e-10, k_max=50), outs,
                             extra=IO.to_flat(P)))
    # fortran_order_d_ip_ocp_hard_tv_single_newton_step: two Newton steps from an interior point near the solution
    # (ux0, pi0 at 0.9 x the IPM's, lam0 / t0 as [lower(nb) | upper(nb)] away from 0)
    P = IO.random_iface_problem(10, [0] + [4] * 10, [2] * 10, 2, 2, None, seed=7)
    qp = IO.to_qp(P)
    r = ref.ipm(qp.copy(), k_max=50, mu0=2.0, mu_tol=1e-10)
    nrng = np.random.default_rng(8)
    ux0 = [0.9 * x for x in r["ux"]]
    pi0 = [0.9 * x for x in r["pi"]]
    lam0 = [np.r_[1.0 + 0.1 * nrng.random(2 * P["nb"][k]), np.zeros(4)] for k in range(P["N"] + 1)]
    t0 = [np.r_[0.5 + 0.1 * nrng.random(2 * P["nb"][k]), np.zeros(4)] for k in range(P["N"] + 1)]
    n = IO.newton_ocp(ref, P, ux0, pi0, lam0, t0, k_max=2, mu0=0.1, mu_tol=1e-12)
    extra = IO.to_flat(P)
    extra.update(ux0=ux0, pi0=pi0, lam0=lam0, t0=t0)
    out.append(save_case("iface_newton_N10_nx4_nu2", "iface_newton", qp, dict(mu0=0.1, mu_tol=1e-12, k_max=2),
                         dict(u=n["u"], x=n["x"], pi=n["pi"], lam=n["lam"], t=n["t"], inf_norm_res=n["inf_norm_res"],
                              kk=n["kk"], ret=n["status"], stat=n["stat"]), extra=extra))
    P = IO.random_iface_problem(10, [0] + [4] * 10, [2] * 10, 2, 2, None, seed=5)
    P2 = IO.new_rhs(P, seed=6)
    k = IO.kkt_ocp(ref, P, P2, mu_tol=1e-10)
    extra = IO.to_flat(P)
    extra.update({"N" + key: v for key, v in IO.to_flat(P2).items()})
    out.append(save_case("iface_kkt_N10_nx4_nu2", "iface_kkt", IO.to_qp(P), dict(mu0=2.0, mu_tol=1e-10, k_max=50),
                         dict(u=k["u"], x=k["x"], pi=k["pi"], lam=k["lam"], inf_norm_res=k["inf_norm_res"]),
                         extra=extra))


MPC_CASES = [  # name, (N, nx, nu, nb, ng, ngN, ti, seed, eq), mu0, warm
    ("tv_N10_nx4_nu2", (10, 4, 2, 6, 0, 0, 0, 21, ()), 2.0, False),
    ("ti_ng_N12_nx3_nu2", (12, 3, 2, 4, 2, 1, 1, 22, ()), 2.0, False),
    ("tv_ng_automu0_N8_nx5_nu2", (8, 5, 2, 5, 2, 2, 0, 23, ()), -1.0, False),
    ("ti_automu0_N9_nx4_nu3", (9, 4, 3, 5, 0, 0, 1, 25, ()), -1.0, False),
    ("tv_nbltnu_N6_nx3_nu3", (6, 3, 3, 2, 0, 0, 0, 25, ()), 2.0, False),
    ("tv_N1_nx3_nu2", (1, 3, 2, 5, 0, 1, 0, 26, ()), 2.0, False),
    ("tv_warm_N10_nx4_nu2", (10, 4, 2, 6, 0, 0, 0, 28, ()), 2.0, True),
]


def iface_mpc(ref, refa, out):
    """The legacy uniform-size wrappers fortran_order_d_ip_mpc_hard_tv / c_order_ twin and their KKT re-solves
    (include/c_interface.h:45-53), restated by oracle/iface_oracle.py ip_mpc / kkt_mpc over the reference's own
    d_ip2_mpc_hard_tv, d_kkt_solve_new_rhs_mpc_hard_tv and d_res_mpc_hard_tv (the wrapper sources need the
    generated include/target.h): time-variant and time-invariant data, general constraints (time-invariant: the
    shared-bounds quirk), the cost-based mu0, fewer boxes than inputs, N = 1, a warm start, and the KKT re-solve."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import iface_oracle as IO

    for name, (N, nx, nu, nb, ng, ngN, ti, seed, eq), mu0, warm in MPC_CASES:
        M = IO.random_mpc_problem(N, nx, nu, nb, ng, ngN, ti, seed=seed, eq=eq)
        w = None
        if warm:
            r0 = IO.ip_mpc(ref, M, k_max=50, mu0=mu0, mu_tol=1e-8)
            w = dict(u=0.9 * r0["u"], x=0.9 * r0["x"])
        # mu_tol 1e-8: below it these small random problems reach the end game where the reference's own c99 and avx
        # builds already differ in the step length of the last iteration (~1e-6 relative)
        r = IO.ip_mpc(ref, M, k_max=50, mu0=mu0, mu_tol=1e-8, warm=w)
        args = dict(N=N, nx=nx, nu=nu, nb=nb, ng=ng, ngN=ngN, ti=ti, mu0=mu0, mu_tol=1e-8, k_max=50,
                    warm=int(warm))
        extra = IO.mpc_to_flat(M)
        if warm:
            extra.update(warm_u=[w["u"]], warm_x=[w["x"]])
        outs = dict(u=[r["u"]], x=[r["x"]], pi=[r["pi"]], lam=[r["lam"]], t=[r["t"]], inf_norm_res=r["inf_norm_res"],
                    kk=r["kk"], ret=r["status"], stat=r["stat"])
        out.append(save_case(f"iface_mpc_{name}", "iface_mpc", r["qp"], args, outs, extra=extra))
    for name, (N, nx, nu, nb, ng, ngN, ti, seed), order in (("tv_N10_nx4_nu2", (10, 4, 2, 6, 0, 0, 0, 31), "F"),
                                                            ("ti_ng_N12_nx3_nu2", (12, 3, 2, 4, 2, 1, 1, 32), "F"),
                                                            ("ti_ng_N12_nx3_nu2_c", (12, 3, 2, 4, 2, 1, 1, 32), "C")):
        M = IO.random_mpc_problem(N, nx, nu, nb, ng, ngN, ti, seed=seed)
        M2 = IO.mpc_new_rhs(M, seed=seed + 100)  # same matrices, perturbed right-hand sides
        # the KKT re-solve's goldens come from the reference's default-target (avx) build of the alternate IPM, whose
        # d_kkt_solve_new_rhs_mpc_hard_tv binds its gradient helper with the right arity (oracle/Makefile ref_avx)
        k = IO.kkt_mpc(refa, M, M2, k_max=50, mu0=2.0, mu_tol=1e-8, order=order)
        args = dict(N=N, nx=nx, nu=nu, nb=nb, ng=ng, ngN=ngN, ti=ti, mu0=2.0, mu_tol=1e-8, k_max=50,
                    order=0 if order == "F" else 1)
        extra = IO.mpc_to_flat(M)
        extra.update({"N" + key: v for key, v in IO.mpc_to_flat(M2).items()})
        qp, _, _ = IO.mpc_pack(M)
        out.append(save_case(f"iface_mpc_kkt_{name}", "iface_mpc_kkt", qp, args,
                             dict(u=[k["u"]], x=[k["x"]], pi=[k["pi"]], lam=[k["lam"]], t=[k["t"]],
                                  inf_norm_res=k["inf_norm_res"]), extra=extra))


def iface_soft(ref, out):
    """fortran_order_d_ip_ocp_soft_tv (interfaces/c/fortran_order_interface.c:1442) restated by
    oracle/iface_oracle.py ip_ocp_soft over the reference's d_ip2_mpc_soft_tv and d_res_mpc_soft_tv: the driver's
    shape (hard input boxes, soft state boxes), a fixed and the cost-based mu0, stopped at mu_tol 1e-6 (the soft end
    game is rounding-sensitive)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import iface_oracle as IO

    for name, (N, nx, nu, seed), mu0 in (("N12_nx8_nu3", (12, 8, 3, 12), 100.0), ("automu0_N10_nx4_nu1", (10, 4, 1, 10), -1.0),
                                         ("N8_nx12_nu4", (8, 12, 4, 8), 50.0)):
        P = IO.random_soft_iface_problem(N, nx, nu, seed=seed)
        r = IO.ip_ocp_soft(ref, P, k_max=50, mu0=mu0, mu_tol=1e-6)
        outs = dict(u=r["u"], x=r["x"], pi=r["pi"], lam=r["lam"], inf_norm_res=r["inf_norm_res"], kk=r["kk"],
                    ret=r["status"], stat=r["stat"])
        out.append(save_case(f"iface_soft_{name}", "iface_soft", IO.to_soft_qp(P), dict(mu0=mu0, mu_tol=1e-6, k_max=50),
                             outs, extra=IO.to_flat(P)))


def wide(ref, refa, out):
    """Problems beyond the 16-wide register tile of the product's narrow kernels (they run on its wide-stage IPM,
    hk_wide_ipm.hip): configs[4]'s stage shape nx=24 nu=6 (mass-spring, time-variant, warm start, k_max, no
    constraints), random problems with more than 16 constraint slots per stage (dense general constraints, also
    on narrow stages), the KKT re-solve, the residuals, a single Newton step, the alternate IPM with its KKT
    re-solve and residuals, and the c_interface wrappers with a partially condensed horizon whose condensed
    stages (nu2 = 40) exceed the tile, with the inner state boxes turned into general constraints."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from helpers import random_qp
    import iface_oracle as IO

    rng = np.random.default_rng(20261017)
    args = dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8)

    def ipm_out(r):
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])

    ms = mass_spring_qp(20, 24, 6, boxes=True)
    tv = mass_spring_qp(15, 24, 6, boxes=True, batch=1, time_variant=True, seed=7).problem(0)
    gen = random_qp(12, [0] + [20] * 12, [4] * 12 + [0], [4] + [8] * 11 + [6], seed=41,
                    ng=[6] + [20] * 11 + [24])
    slots = random_qp(20, [0] + [8] * 20, [3] * 20 + [0], [3] + [11] * 19 + [8], seed=46,
                      ng=[2] + [8] * 19 + [9])
    for name, qp, a in (("N20_nx24_nu6", ms, args), ("tv_N15_nx24_nu6", tv, args),
                        ("ng_N12_nx20_nu4", gen, dict(args, k_max=60)), ("slots_N20_nx8_nu3", slots, args),
                        ("kmax4_N20_nx24_nu6", ms, dict(args, k_max=4))):
        out.append(save_case(f"ipmw_{name}", "ipm", qp, a, ipm_out(ref.ipm(qp.copy(), **a))))
    ux0 = rand_vecs(rng, [ms.nux(k) for k in range(ms.N + 1)], scale=0.1)
    r = ref.ipm(ms.copy(), warm_start=1, ux=ux0, **args)
    out.append(save_case("ipmw_warm_N20_nx24_nu6", "ipm", ms, dict(args, warm_start=1), ipm_out(r),
                         extra=dict(ux0=ux0)))
    qp = mass_spring_qp(15, 24, 6, boxes=False)
    out.append(save_case("ipmw_noconstr_N15_nx24_nu6", "ipm", qp, args, ipm_out(ref.ipm(qp.copy(), **args))))
    for name, qp in (("N20_nx24_nu6", ms), ("ng_N12_nx20_nu4", gen)):
        r = ref.ipm(qp.copy(), **dict(args, k_max=60))
        b, q = bq_from_qp(qp)
        b2 = [x + 0.01 * rng.standard_normal(x.shape) for x in b]
        q2 = [x + 0.01 * rng.standard_normal(x.shape) for x in q]
        k = ref.kkt_new_rhs(qp.copy(), r["work"], b2, q2)
        out.append(save_case(f"kktw_{name}", "kkt", qp, dict(args, k_max=60),
                             dict(ux=k["ux"], pi=k["pi"], lam=k["lam"], t=k["t"]), extra=dict(b2=b2, q2=q2)))
        uxp = [x + 0.01 * rng.standard_normal(x.shape) for x in r["ux"]]
        pip = [x + 0.01 * rng.standard_normal(x.shape) for x in r["pi"]]
        res = ref.residuals(qp.copy(), b, q, uxp, pip, r["lam"], r["t"])
        out.append(save_case(f"resw_{name}", "res", qp, {},
                             dict(rq=res["rq"], rb=res["rb"], rd=res["rd"], rm=res["rm"], mu=res["mu"]),
                             extra=dict(b=b, q=q, ux=uxp, pi=pip, lam=r["lam"], t=r["t"])))
        res = ref.residuals_plain(qp.copy(), b, q, uxp, pip, r["lam"], r["t"])
        out.append(save_case(f"res2w_{name}", "res2", qp, {},
                             dict(rq=res["rq"], rb=res["rb"], rd=res["rd"], mu=res["mu"]),
                             extra=dict(b=b, q=q, ux=uxp, pi=pip, lam=r["lam"], t=r["t"])))
        a2 = dict(args, mu_tol=1e-8)
        out.append(save_case(f"ipm2w_{name}", "ipm2", qp, a2, ipm_out(ref.ipm(qp.copy(), res=False, **a2))))
        r2 = refa.ipm(qp.copy(), res=False, **a2)
        d2 = [x + 0.01 * rng.standard_normal(x.shape) for x in qp.d]
        k2 = refa.kkt_new_rhs_plain(qp.copy(), r2["work"], b2, q2, d2, r2["ux"])
        out.append(save_case(f"kkt2w_{name}", "kkt2", qp, a2, dict(ux=k2["ux"], pi=k2["pi"], lam=k2["lam"], t=k2["t"]),
                             extra=dict(b2=b2, q2=q2, d2=d2)))
    qp = mass_spring_qp(10, 24, 6, boxes=True)
    r = ref.ipm(qp.copy(), **args)
    lam0, t0 = [], []
    for k in range(qp.N + 1):
        nb = int(qp.nb[k])
        lam0.append(np.concatenate([1.0 + 0.1 * rng.random(2 * nb), np.zeros(4)]))
        t0.append(np.concatenate([0.5 + 0.1 * rng.random(2 * nb), np.zeros(4)]))
    ux0 = [0.9 * x for x in r["ux"]]
    pi0 = [0.9 * x for x in r["pi"]]
    sn = ref.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=1, mu0=0.1)
    out.append(save_case("newtonw_N10_nx24_nu6", "newton", qp, dict(k_max=1, mu0=0.1, mu_tol=1e-12, alpha_min=1e-8),
                         ipm_out(sn), extra=dict(ux0=ux0, pi0=pi0, lam0=lam0, t0=t0)))
    # c_interface wrappers, condensed N2 < N with condensed stages beyond the tile (nu <= 4: the reference's
    # c99 condensing is right there), and a full-space wide problem
    for name, (N, nx, nu, bu, bx, ng, seed), N2 in (
            ("condw_N40_nx12_nu4_N2_4", (40, [0] + [12] * 40, [4] * 40, 4, 6, None, 11), 4),
            ("fullw_N10_nx20_nu4", (10, [0] + [20] * 10, [4] * 10, 4, 8, None, 12), 10)):
        P = IO.random_iface_problem(N, nx, nu, bu, bx, ng, seed=seed)
        r = IO.ip_ocp(ref, P, N2, k_max=50, mu0=2.0, mu_tol=1e-10)
        outs = dict(u=r["u"], x=r["x"], pi=r["pi"], lam=r["lam"], inf_norm_res=r["inf_norm_res"], kk=r["kk"],
                    ret=r["status"], stat=r["stat"])
        out.append(save_case(f"iface_{name}", "iface", IO.to_qp(P), dict(N2=N2, mu0=2.0, mu_tol=1e-10, k_max=50),
                             outs, extra=IO.to_flat(P)))


def driver(out):
    """The reference's own driver test_problems/test_d_ric_mpc.c, compiled unchanged and linked against the full
    reference (tools/relink/Makefile), run on the host: its printed ux / pi (N=10 nx=8 nu=3, after 1000 sv, trf and
    trs calls) pin tests/test_gpu_ref_driver.py, which runs the same driver relinked against libhpmpc_mi355x.so."""
    import subprocess
    import tempfile

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "relink"), "drivers"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "relink", "test_d_ric_mpc_ref")
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "test_problems", "results"))
        text = subprocess.run([exe], cwd=d, check=True, capture_output=True, text=True, timeout=300).stdout
    b = parse_ric_driver(text)
    path = os.path.join(HERE, "drivers", "test_d_ric_mpc.npz")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    ux = np.concatenate([np.asarray(r) for r in b["ux"]])
    uxn = np.array([len(r) for r in b["ux"]], dtype=np.int32)
    np.savez_compressed(path, ux=ux, ux_len=uxn, pi=np.asarray(b["pi"]))
    out.append(path)
    # tools/relink/relink_driver.c (the low-level call sequence of test_d_ip_hard.c / test_d_ric_mpc.c) linked against
    # the whole reference: every number it prints, at full precision
    exe = os.path.join(ROOT, "oracle", "_ref", "relink", "relink_driver_ref")
    text = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=300).stdout
    path = os.path.join(HERE, "drivers", "relink_driver.txt")
    with open(path, "w") as f:
        f.write(text)
    out.append(path)
    # Its alternate-IPM KKT re-solve (kkt2) and that re-solve's residuals (res2) from the reference's default-target
    # build instead: the c99 build's
    # d_kkt_solve_new_rhs_mpc_hard_tv passes 9 arguments to the 8-parameter c99 gradient helper (oracle/Makefile
    # ref_avx), and on this driver's problem its kkt2 ends 8.3e-8 (ux) / 3.4e-7 (pi) from the X64_AVX / X64_AVX2
    # builds and the oracle, which agree with each other to 1e-15.  Same problem and call sequence as the driver
    # (relink_qp; its c99 run reproduces the printed kkt2 lines bitwise).
    qp, b, q = relink_qp()
    avx = ref_avx_api()
    r = avx.ipm(qp.copy(), k_max=50, mu0=2.0, mu_tol=1e-8, alpha_min=1e-8, res=False)
    kk = avx.kkt_new_rhs_plain(qp.copy(), r["work"], b, q, qp.d, r["ux"])
    path = os.path.join(HERE, "drivers", "relink_kkt2_avx.npz")
    arrs = {f"ux_{k}": kk["ux"][k][: qp.nux(k)] for k in range(qp.N + 1)}
    arrs.update({f"pi_{k}": kk["pi"][k][: int(qp.nx[k + 1])] for k in range(qp.N)})
    # and the residuals of that re-solve (d_res_mpc_hard_tv on its ux, pi, lam, t: the driver prints res2.mu)
    arrs["mu_0"] = np.array([avx.residuals_plain(qp, b, q, kk["ux"], kk["pi"], kk["lam"], kk["t"])["mu"]])
    np.savez_compressed(path, **arrs)
    out.append(path)


def relink_qp():
    """The problem of tools/relink/relink_driver.c:53-100 (N=10, nx = 0 at stage 0 then 8, nu=3, boxes on the first
    nu + nx/2 variables) and the new right-hand sides b, q of its re-solves (:120-125)."""
    N, NX, NU = 10, 8, 3
    nx = np.array([0 if k == 0 else NX for k in range(N + 1)])
    nu = np.array([NU if k < N else 0 for k in range(N + 1)])
    nb = nu + nx // 2
    idxb = [np.arange(nb[k], dtype=np.int32) for k in range(N + 1)]
    R, Bl, D = [], [], []
    for k in range(N + 1):
        nux = int(nu[k] + nx[k])
        nx1 = int(nx[k + 1]) if k < N else 0
        M = np.zeros((nux + 1, nux))
        M[np.arange(nux), np.arange(nux)] = 2.0
        M[nux, :] = 0.1
        R.append(pack_lib4(M))
        if k < N:
            B = np.zeros((nux + 1, nx1))
            for i in range(nx1):
                B[nu[k] + i % (nx[k] if nx[k] > 0 else 1), i] = 1.0
            for i in range(nx1):
                B[i % (nu[k] if nu[k] > 0 else 1), i] += 0.1
            B[nux, :] = 0.05
            Bl.append(pack_lib4(B))
        pnb = rup(int(nb[k]), BS)
        d = np.zeros(2 * pnb + 4)
        d[: nb[k]] = -1.0
        d[pnb: pnb + nb[k]] = 1.0
        D.append(d)
    qp = OCPQP(N, nx, nu, nb, np.zeros(N + 1, dtype=nx.dtype), idxb, Bl, R, D, [], None)
    b = [np.array([0.03 * ((i + k) % 3) for i in range(int(nx[k + 1]))] + [0.0] * 4) for k in range(N)]
    q = [np.array([0.01 * (i + 1) - 0.02 * k for i in range(qp.nux(k))] + [0.0] * 4) for k in range(N + 1)]
    return qp, b, q


def divergent(ref, out):
    """Infeasible draws of the benchmark workload (hpmpc_amd.shard.make_shard(100, 12, 4, 0, 1, 1024), global
    problems 841 and 920): the primal-dual iterates diverge (lam -> 1e17..1e19) until the step length falls below
    alpha_min (ret 2).  The exit iteration is set by amplified last bits: the oracle (a second c99 build of the
    same algorithm) exits 2 iterations earlier than the reference on both (28 vs 30, 38 vs 40; over the whole
    1024-problem batch the two builds differ by 1-2 iterations on 30 of its 91 divergent problems).  These pin
    the divergence gate of tests/helpers.py compare_ipm (same ret, kk within 2)."""
    from hpmpc_amd.shard import make_shard

    qp = make_shard(100, 12, 4, 0, 1, 1024)
    args = dict(k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8)
    for p in (841, 920):
        one = qp.problem(p)
        r = ref.ipm(one.copy(), **args)
        out.append(save_case(f"ipm_div_p{p}_N100_nx12_nu4", "ipm_div", one, args,
                             dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"],
                                  ret=r["ret"])))


def soft(ref, out):
    """Soft-constraint IPM d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:83): the reference driver's problem
    (test_d_ip_soft.c: Q = 0, Z = 0, z = 100, mu0 = 100) at three sizes, stopped at mu_tol = 1e-5 -- below that its
    end game is rounding-chaotic (the reference's own -mfma -ffp-contract=fast build stops at a different iterate,
    DESIGN.md) -- plus an iteration cap, hard boxes at stage N (alpha collapses at iteration 3, through the
    soft-gradient write the reference makes past qx_N into Zl / zl), a time-variant Q = I, Z = 1 case, only hard
    boxes, and no constraints at all."""
    from hpmpc_amd.soft import mass_spring_soft

    cases = [("ms_N10_nx4_nu1", mass_spring_soft(10, 4, 1), dict(mu_tol=1e-5)),
             ("ms_N10_nx8_nu3", mass_spring_soft(10, 8, 3), dict(mu_tol=1e-5)),
             ("ms_N15_nx12_nu4", mass_spring_soft(15, 12, 4), dict(mu_tol=1e-5)),
             ("kmax4_N15_nx12_nu4", mass_spring_soft(15, 12, 4), dict(k_max=4, mu_tol=1e-5)),
             ("hardN_N12_nx8_nu2", mass_spring_soft(12, 8, 2, hard_last=2), dict(mu_tol=1e-5)),
             ("hardN_N10_nx4_nu2", mass_spring_soft(10, 4, 2, hard_last=4), dict(mu_tol=1e-5)),
             ("tv_N8_nx12_nu4", mass_spring_soft(8, 12, 4, time_variant=True, Zq=1.0, zl=10.0, Q_diag=1.0),
              dict(mu_tol=1e-6)),
             ("q1_N20_nx8_nu2", mass_spring_soft(20, 8, 2, Q_diag=1.0, Zq=0.5, zl=20.0), dict(mu_tol=1e-6)),
             ("hardonly_N10_nx8_nu3", mass_spring_soft(10, 8, 3, soft=False, Q_diag=1.0), dict(mu_tol=1e-6)),
             ("noconstr_N10_nx8_nu3", mass_spring_soft(10, 8, 3, soft=False, hard=False, Q_diag=1.0),
              dict(mu_tol=1e-6))]
    for name, sq, kw in cases:
        args = dict(k_max=50, mu0=100.0, mu_tol=1e-8, alpha_min=1e-8)
        args.update(kw)
        r = ref.ipm_soft(sq.copy(), work_extra=1 << 16, **args)
        outs = dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
        out.append(save_case(f"soft_{name}", "soft", sq, args, outs,
                             extra=dict(ns=[sq.ns.astype(np.float64)], Z=sq.Z, z=sq.z)))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "soft":
        o = []
        soft(ref_api(), o)
        print(f"wrote {len(o)} soft cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "iface":
        o = []
        iface(ref_api(), o)
        print(f"wrote {len(o)} iface cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "wide":
        o = []
        wide(ref_api(), ref_avx_api(), o)
        print(f"wrote {len(o)} wide cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "driver":
        o = []
        driver(o)
        print(f"wrote {o}")
    elif len(sys.argv) > 1 and sys.argv[1] == "divergent":
        o = []
        divergent(ref_api(), o)
        print(f"wrote {len(o)} divergent cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "iface_mpc":
        o = []
        iface_mpc(ref_api(), ref_avx_api(), o)
        print(f"wrote {len(o)} iface_mpc cases")
    elif len(sys.argv) > 1 and sys.argv[1] == "iface_soft":
        o = []
        iface_soft(ref_api(), o)
        print(f"wrote {len(o)} iface_soft cases")
    elif len(sys.argv) > 1 and sys.argv[1] == "soft_res":
        o = []
        soft_res(ref_api(), o)
        print(f"wrote {len(o)} soft_res cases")
    elif len(sys.argv) > 1 and sys.argv[1] == "gates":
        o = []
        gates(ref_api(), o)
        print(f"wrote {len(o)} gate cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "xclamp":
        o = []
        xclamp(ref_api(), o)
        print(f"wrote {len(o)} xclamp cases")
    elif len(sys.argv) > 1 and sys.argv[1] == "xclamp_ipm":
        o = []
        xclamp_ipm(ref_api(), o)
        print(f"wrote {len(o)} xclamp IPM gate cases")
    elif len(sys.argv) > 1 and sys.argv[1] == "cond_parts":
        o = []
        cond_parts(ref_api(), o)
        print(f"wrote {len(o)} cond_parts cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    elif len(sys.argv) > 1 and sys.argv[1] == "pcond":
        o = []
        pcond(ref_api(), o)
        print(f"wrote {len(o)} pcond cases, {sum(os.path.getsize(p) for p in o) / 1e6:.2f} MB")
    else:
        main()
