"""Run a golden case through any library exporting the reference prototypes and compare outputs."""
import numpy as np

from hpmpc_amd.cabi import bq_from_qp

TOL_RIC = 1e-12   # Riccati sv/trf/trs: |a-b| <= TOL * max(1, |ref|)   
TOL_IPM = 1e-10   # IPM ux/pi/lam/t with identical iteration count
TOL_STAT = 1e-9
# The alternate IPM (d_ip2_mpc_hard_tv) has no residual correction: its last Newton systems carry the
# Hessian terms lam/t of the current iterate (~1/mu), so lam (and the step lengths in stat) are determined
# only to ~eps*lam/t; ux/pi/t stay well conditioned.  Measured oracle-vs-reference: lam 3e-6 (stopped at
# mu_tol 1e-8), 5e-3 (run to 1e-12, lam/t ~ 1e16 in the last iteration); ux/pi/t 2e-15 / 6e-10.
TOL_IPM2 = dict(ux=1e-10, pi=1e-10, t=1e-10, lam=1e-4, stat=1e-9)
TOL_IPM2_TIGHT = dict(ux=1e-8, pi=1e-8, t=1e-8, lam=5e-2, stat=5e-2)  # mu_tol < 1e-8
TOL_KKT2 = dict(ux=1e-8, pi=1e-8, t=1e-8, lam=1e-4)  # re-solve on the factor of that last iteration


def run_case(api, case):
    """Execute `case` with `api`; returns dict of outputs keyed like case.out."""
    qp = case.fresh_qp()
    a = case.args
    inp = case.inp
    if case.kind in ("sv", "sv_xclamp"):
        kw = {}
        if a.get("update_b"):
            kw.update(update_b=1, b=inp["b"], update_q=1, q=inp["q"], bd=inp["bd"], Qx=inp["Qx"], qx=inp["qx"])
        ux, pi, Pb, _ = api.ric_sv(qp, compute_pi=int(a["compute_pi"]), compute_Pb=int(a["compute_Pb"]), **kw)
        out = dict(ux=ux, pi=pi, Pb=Pb)
        if a.get("update_b"):
            out.update(BAbt_after=qp.BAbt, RSQrq_after=qp.RSQrq)
        return out
    if case.kind == "trf_trs":
        mem = api.ric_trf(qp, bd=inp["bd"], Qx=inp["Qx"])
        ux, pi, Pb = api.ric_trs(qp, mem, b=inp["b"], q=inp["q"], qx=inp["qx"], compute_pi=1, compute_Pb=1)
        return dict(ux=ux, pi=pi, Pb=Pb)
    if case.kind in ("ipm", "ipm_div"):
        kw = dict(k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"])
        if a.get("warm_start"):
            kw.update(warm_start=1, ux=inp["ux0"])
        r = api.ipm(qp, **kw)
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    if case.kind == "kkt":
        r = api.ipm(qp, k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"])
        k = api.kkt_new_rhs(qp, r["work"], inp["b2"], inp["q2"])
        return dict(ux=k["ux"], pi=k["pi"], lam=k["lam"], t=k["t"])
    if case.kind == "ipm2":
        r = api.ipm(qp, k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"], res=False)
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    if case.kind == "kkt2":
        r = api.ipm(qp, k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"], res=False)
        k = api.kkt_new_rhs_plain(qp, r["work"], inp["b2"], inp["q2"], inp["d2"], r["ux"])
        return dict(ux=k["ux"], pi=k["pi"], lam=k["lam"], t=k["t"])
    if case.kind == "res2":
        r = api.residuals_plain(qp, inp["b"], inp["q"], inp["ux"], inp["pi"], inp["lam"], inp["t"])
        return dict(rq=r["rq"], rb=r["rb"], rd=r["rd"], mu=r["mu"])
    if case.kind == "res":
        r = api.residuals(qp, inp["b"], inp["q"], inp["ux"], inp["pi"], inp["lam"], inp["t"])
        return dict(rq=r["rq"], rb=r["rb"], rd=r["rd"], rm=r["rm"], mu=r["mu"])
    if case.kind == "newton":
        r = api.single_newton(qp, inp["ux0"], inp["pi0"], inp["lam0"], inp["t0"], k_max=int(a["k_max"]),
                              mu0=a["mu0"])
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    if case.kind == "pcond":
        c, _ = api.part_cond(qp, int(a["N2"]))
        e = api.part_expand(qp, c, inp["u2"], inp["p2"], inp["lam2"], inp["t2"])
        return dict(cqp=c, ux=e["ux"], pi=e["pi"], lam=e["lam"], t=e["t"])
    if case.kind == "pcond_sv":
        return pcond_sv(api, qp, int(a["N2"]))
    if case.kind == "soft_res":
        from hpmpc_amd.soft import SoftQP

        return api.residuals_soft(SoftQP.from_case(case), inp["q"], inp["ux"], inp["pi"], inp["lam"], inp["t"])
    if case.kind == "cond_parts":
        # each building block alone; RSQrq and DCtd on the reference's own Gammas
        f = a["fill"]
        G, B2 = api.cond_BAbt(qp.copy(), fill=f)
        R2 = api.cond_RSQrq(qp.copy(), case.out["Gamma"], fill=f)
        DCt2, d2, idxb2, _ = api.cond_DCtd(qp.copy(), case.out["Gamma"], fill=f)
        return dict(Gamma=G, BAbt2=B2, RSQrq2=R2, DCt2=DCt2, d2=d2, idxb2=idxb2)
    if case.kind in ("iface", "iface_kkt", "iface_newton", "iface_soft"):
        return run_iface(api, case)
    if case.kind in ("iface_mpc", "iface_mpc_kkt"):
        return run_iface_mpc(api, case)
    if case.kind == "soft":
        from hpmpc_amd.soft import SoftQP

        r = api.ipm_soft(SoftQP.from_case(case), k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"],
                         alpha_min=a["alpha_min"])
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    raise ValueError(case.kind)


def _iface_oracle():
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import iface_oracle

    return iface_oracle


def run_iface(api, case, order="F"):
    """The c_interface.h wrappers: through the library's own wrapper symbols when it has them (the product),
    else the restatement oracle/iface_oracle.py over the library's low-level entry points (the oracle)."""
    IO = _iface_oracle()
    qp, a = case.qp, case.args
    P = IO.from_flat(qp.N, qp.nx, qp.nu, qp.nb, qp.ng, case.inp)
    kw = dict(k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"])
    if case.kind == "iface_soft":
        r = api.ip_ocp_soft(P, **kw) if hasattr(api.lib, api.p + "fortran_order_d_ip_ocp_soft_tv") else \
            IO.ip_ocp_soft(api, P, **kw)
        out = {k: r[k] for k in ("u", "x", "pi", "lam", "inf_norm_res", "kk", "stat")}
        out["ret"] = r["status"]
        return out
    has = hasattr(api.lib, api.p + "fortran_order_d_ip_ocp_hard_tv")
    if case.kind == "iface":
        r = api.ip_ocp(P, int(a["N2"]), order=order, **kw) if has else IO.ip_ocp(api, P, int(a["N2"]), **kw)
        out = {k: r[k] for k in ("u", "x", "pi", "lam", "inf_norm_res", "kk", "stat")}
        out["ret"] = r["status"]
        return out
    if case.kind == "iface_newton":
        kw = dict(k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"])
        st = [case.inp[k] for k in ("ux0", "pi0", "lam0", "t0")]
        if hasattr(api.lib, api.p + "fortran_order_d_ip_ocp_hard_tv_single_newton_step"):
            r = api.newton_ocp(P, *st, **kw)
        else:
            r = IO.newton_ocp(api, P, *st, **kw)
        out = {k: r[k] for k in ("u", "x", "pi", "lam", "t", "inf_norm_res", "kk", "stat")}
        out["ret"] = r["status"]
        return out
    P2 = IO.from_flat(qp.N, qp.nx, qp.nu, qp.nb, qp.ng, {k[1:]: v for k, v in case.inp.items() if k.startswith("NP_")})
    if has:
        r = api.ip_ocp(P, qp.N, order=order, **kw)
        k = api.kkt_ocp(P2, r["work0"], order=order)
    else:
        k = IO.kkt_ocp(api, P, P2, **kw)
    return {key: k[key] for key in ("u", "x", "pi", "lam", "inf_norm_res")}


def run_iface_mpc(api, case, order=None):
    """The legacy uniform-size wrappers (include/c_interface.h:45-53): through the library's own symbols when it has
    them (the product), else oracle/iface_oracle.py ip_mpc / kkt_mpc over its low-level entry points."""
    IO = _iface_oracle()
    a = case.args
    M = IO.mpc_from_flat(a, case.inp)
    kw = dict(k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"])
    has = hasattr(api.lib, api.p + "fortran_order_d_ip_mpc_hard_tv")
    keys = ("u", "x", "pi", "lam", "t", "inf_norm_res")
    if case.kind == "iface_mpc":
        order = order or "F"
        w = dict(u=case.inp["warm_u"][0], x=case.inp["warm_x"][0]) if int(a.get("warm", 0)) else None
        r = api.ip_mpc(M, order=order, warm=w, **kw) if has else IO.ip_mpc(api, M, warm=w, **kw)
        out = {k: [r[k]] for k in keys[:-1]}
        out.update(inf_norm_res=r["inf_norm_res"], kk=r["kk"], ret=r["status"], stat=r["stat"])
        return out
    order = "C" if int(a["order"]) else "F"
    M2 = IO.mpc_from_flat(a, {k[1:]: v for k, v in case.inp.items() if k.startswith("N")})
    if has:
        r = api.ip_mpc(M, order=order, **kw)
        k = api.kkt_mpc(M2, r["work0"], order=order)
    else:
        k = IO.kkt_mpc(api, M, M2, order=order, **kw)
    out = {key: [k[key]] for key in keys[:-1]}
    out["inf_norm_res"] = k["inf_norm_res"]
    return out


def check_iface(case, got):
    out = case.out
    if case.kind == "iface_soft":  # the soft IPM's gates (TOL_SOFT); residual norms at its mu_tol 1e-6
        assert int(got["kk"]) == int(out["kk"]) and int(got["ret"]) == int(out["ret"]), (case.name, got["kk"], out["kk"])
        np.testing.assert_allclose(got["stat"], out["stat"], rtol=TOL_SOFT["stat"], atol=1e-14, err_msg=case.name)
        for key, tol in (("u", TOL_SOFT["ux"]), ("x", TOL_SOFT["ux"]), ("pi", TOL_SOFT["pi"]), ("lam", TOL_SOFT["lam"])):
            for k, (g, r) in enumerate(zip(got[key], out[key])):
                g, r = np.asarray(g), np.asarray(r)
                if r.size:
                    e = float(np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r))))
                    assert e <= tol, f"{case.name}: {key}[{k}] err {e:.3e}"
        np.testing.assert_allclose(got["inf_norm_res"], out["inf_norm_res"], rtol=0, atol=1e-7, err_msg=case.name)
        return
    if "kk" in out:
        assert int(got["kk"]) == int(out["kk"]) and int(got["ret"]) == int(out["ret"]), (case.name, got["kk"], out["kk"])
        np.testing.assert_allclose(got["stat"], out["stat"], rtol=TOL_STAT, atol=1e-14, err_msg=case.name)
    for key in ("u", "x", "pi", "lam", "t"):
        if key not in out:
            continue
        for k, (g, r) in enumerate(zip(got[key], out[key])):
            g, r = np.asarray(g), np.asarray(r)
            if r.size:
                e = float(np.max(np.abs(g - r) / np.maximum(1.0, np.abs(r))))
                assert e <= TOL_IPM, f"{case.name}: {key}[{k}] err {e:.3e}"
    # residual infinity norms of a converged solve are rounding-level (~1e-12): absolute comparison
    np.testing.assert_allclose(got["inf_norm_res"], out["inf_norm_res"], rtol=0, atol=1e-9, err_msg=case.name)


def pcond_sv(api, qp, N2):
    """condense (d_part_cond) -> Riccati sv on the condensed problem -> expand (d_part_expand_solution)."""
    c, _ = api.part_cond(qp, N2)
    u2, p2, _, _ = api.ric_sv(c.copy(), compute_pi=1, compute_Pb=0)
    z = [np.zeros(max(c.nconstr(k), 1)) for k in range(N2 + 1)]
    e = api.part_expand(qp, c, u2, p2, z, z)
    return dict(ux=e["ux"], pi=e["pi"])


TOL_PCOND_SV = 1e-11  # condensed pipeline vs the reference's direct Riccati (oracle measured 4e-14 absolute)


def check_pcond(case, got):
    """Condensed data of d_part_cond (lower triangle of RSQrq2: the only part any consumer reads) and the
    expanded solution."""
    from hpmpc_amd.ocp import unpack_lib4

    out, c = case.out, got["cqp"]
    for f in ("nx2", "nu2", "nb2", "ng2"):
        np.testing.assert_array_equal(getattr(c, f[:2]), out[f], err_msg=case.name + f)
    N2 = c.N
    for k in range(N2):
        nux = c.nux(k)
        A = unpack_lib4(c.BAbt[k], nux + 1, int(c.nx[k + 1]))
        B = unpack_lib4(out["BAbt2"][k], nux + 1, int(c.nx[k + 1]))
        np.testing.assert_allclose(A, B, rtol=TOL_RIC, atol=TOL_RIC, err_msg=f"{case.name} BAbt2[{k}]")
        A = np.tril(unpack_lib4(c.RSQrq[k], nux + 1, nux))
        B = np.tril(unpack_lib4(out["RSQrq2"][k], nux + 1, nux))
        np.testing.assert_allclose(A, B, rtol=TOL_RIC, atol=TOL_RIC, err_msg=f"{case.name} RSQrq2[{k}]")
        if c.ng[k]:
            A = unpack_lib4(c.DCt[k], nux, int(c.ng[k]))
            B = unpack_lib4(out["DCt2"][k], nux, int(c.ng[k]))
            np.testing.assert_allclose(A, B, rtol=TOL_RIC, atol=TOL_RIC, err_msg=f"{case.name} DCt2[{k}]")
        nb, pnb, ng, png = int(c.nb[k]), c.pnb(k), int(c.ng[k]), c.png(k)
        idx = np.r_[0:nb, pnb:pnb + nb, 2 * pnb:2 * pnb + ng, 2 * pnb + png:2 * pnb + png + ng].astype(int)
        np.testing.assert_allclose(c.d[k][idx], out["d2"][k][idx], rtol=TOL_RIC, atol=TOL_RIC,
                                   err_msg=f"{case.name} d2[{k}]")
        np.testing.assert_array_equal(c.idxb[k], out["idxb2"][k].astype(np.int32), err_msg=f"{case.name} idxb2")
    for key in ("ux", "pi", "lam", "t"):
        e = max_err(case, key, got[key], out[key])
        assert e <= TOL_RIC, f"{case.name}: {key} err {e:.3e}"


def _valid_len(case, key, k):
    qp = case.qp
    if key in ("ux", "rq"):
        return qp.nux(k)
    if key in ("pi", "Pb", "rb"):
        return int(qp.nx[k + 1])
    if key in ("lam", "t", "rd", "rm"):
        return qp.nconstr(k)
    return None


def max_err(case, key, got, ref):
    """max_k,i |got-ref| / max(1,|ref|) over the valid part of each stage vector."""
    if isinstance(ref, list):
        e = 0.0
        for k, r in enumerate(ref):
            n = _valid_len(case, key, k)
            n = len(r) if n is None else n
            if key in ("lam", "t", "rd", "rm"):
                pnb, png, nb, ng = case.qp.pnb(k), case.qp.png(k), int(case.qp.nb[k]), int(case.qp.ng[k])
                idx = np.r_[0:nb, pnb:pnb + nb, 2 * pnb:2 * pnb + ng, 2 * pnb + png:2 * pnb + png + ng].astype(int)
            else:
                idx = np.arange(n)
            if idx.size == 0:
                continue
            g = np.asarray(got[k])[idx]
            rr = np.asarray(r)[idx]
            e = max(e, float(np.max(np.abs(g - rr) / np.maximum(1.0, np.abs(rr)))))
        return e
    ref = np.asarray(ref, dtype=np.float64)
    got = np.asarray(got, dtype=np.float64)
    if ref.size == 0:
        return 0.0
    return float(np.max(np.abs(got.reshape(ref.shape) - ref) / np.maximum(1.0, np.abs(ref))))


# d_ip2_mpc_soft_tv, identical kk / ret: the reference's own -mfma -ffp-contract=fast build differs from its
# default build by up to ux 4e-9, pi 1.5e-7, lam 4e-8, stat 1e-9 on the golden cases and stat 1.3e-7 at mu_tol 1e-8
# (soft constraints)
TOL_SOFT = dict(ux=5e-8, t=5e-8, pi=1e-6, lam=1e-6, stat=1e-7)


def check_soft(case, got):
    from hpmpc_amd.soft import SoftQP

    sq = SoftQP.from_case(case)
    out = case.out
    assert int(got["kk"]) == int(out["kk"]), (case.name, got["kk"], out["kk"])
    assert int(got["ret"]) == int(out["ret"]), (case.name, got["ret"], out["ret"])
    if int(out["kk"]) > 0:
        st = np.asarray(out["stat"])
        e = float(np.max(np.abs(np.asarray(got["stat"])[: st.size] - st) / np.maximum(1.0, np.abs(st))))
        assert e <= TOL_SOFT["stat"], f"{case.name}: stat err {e:.3e}"
    for key in ("ux", "pi", "lam", "t"):
        e = 0.0
        for k, r in enumerate(out[key]):
            if key == "ux":
                idx = np.arange(sq.nux(k))
            elif key == "pi":
                idx = np.arange(int(sq.nx[k + 1]))
            else:
                nb, ns = int(sq.nb[k]), int(sq.ns[k])
                pnb, pns = (nb + 3) // 4 * 4, (ns + 3) // 4 * 4
                idx = np.concatenate([np.arange(nb), np.arange(pnb, pnb + nb)] +
                                     [np.arange(2 * pnb + s * pns, 2 * pnb + s * pns + ns) for s in range(4)])
            if idx.size == 0:
                continue
            g, rr = np.asarray(got[key][k])[idx], np.asarray(r)[idx]
            e = max(e, float(np.max(np.abs(g - rr) / np.maximum(1.0, np.abs(rr)))))
        assert e <= TOL_SOFT[key], f"{case.name}: {key} err {e:.3e} > {TOL_SOFT[key]:.0e}"


def sub_block(qp, s0: int, T: int):
    """Stages s0 .. s0+T of qp as a horizon-T problem: one condensing block (its stage T only sizes nx_T)."""
    from hpmpc_amd.ocp import OCPQP

    sl = slice(s0, s0 + T + 1)
    return OCPQP(T, qp.nx[sl].copy(), qp.nu[sl].copy(), qp.nb[sl].copy(), np.zeros(T + 1, np.int32),
                 [i.copy() for i in qp.idxb[sl]], [b.copy() for b in qp.BAbt[s0:s0 + T]],
                 [r.copy() for r in qp.RSQrq[sl]], [d.copy() for d in qp.d[sl]], [], None)


COND_FILL = 7.25  # sentinel pre-filled into every output: what the reference leaves alone stays 7.25


def dense_kkt(qp):
    """The exact solution of an OCP QP without inequality constraints from its dense KKT system (numpy LU):
    ux_k and pi_k with the reference's sign (pi_k = the gradient of the cost-to-go at x_{k+1})."""
    from hpmpc_amd.ocp import unpack_lib4

    N = qp.N
    sizes = [qp.nux(k) for k in range(N + 1)]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    n = int(off[-1])
    H, g = np.zeros((n, n)), np.zeros(n)
    for k in range(N + 1):
        m = sizes[k]
        M = unpack_lib4(qp.RSQrq[k], m + 1, m)
        L = np.tril(M[:m])
        H[off[k]:off[k + 1], off[k]:off[k + 1]] = L + np.tril(L, -1).T
        g[off[k]:off[k + 1]] = M[m]
    ncon = sum(int(qp.nx[k + 1]) for k in range(N))
    Cm, c, r0 = np.zeros((ncon, n)), np.zeros(ncon), 0
    for k in range(N):
        m, nx1, nu1 = sizes[k], int(qp.nx[k + 1]), int(qp.nu[k + 1])
        Bt = unpack_lib4(qp.BAbt[k], m + 1, nx1)
        Cm[r0:r0 + nx1, off[k]:off[k + 1]] = -Bt[:m].T
        Cm[r0:r0 + nx1, off[k + 1] + nu1:off[k + 1] + nu1 + nx1] = np.eye(nx1)
        c[r0:r0 + nx1] = Bt[m]
        r0 += nx1
    K = np.block([[H, Cm.T], [Cm, np.zeros((ncon, ncon))]])
    sol = np.linalg.solve(K, np.concatenate([-g, c]))
    z, lam = sol[:n], sol[n:]
    ux = [z[off[k]:off[k + 1]] for k in range(N + 1)]
    pi, r0 = [], 0
    for k in range(N):
        nx1 = int(qp.nx[k + 1])
        pi.append(-lam[r0:r0 + nx1])
        r0 += nx1
    return ux, pi


# The clamp variants (d, off, r) of xclamp_qp that tests/test_gpu_parity.py runs through every kernel family: exact
# clamps, a clamp with a gradient term, a zero pivot, a near-clamp pivot, and two that fail the certificate without a
# clamp (d = 2e-15 is left out: there the reference's own builds spread by 1e-11).
XCLAMP = [(1e-16, 1e-9, 0.0), (1e-16, 1e-9, 0.5), (0.0, 0.0, 0.3), (5e-16, 1e-8, 0.2), (1e-8, 1e-9, 0.1),
          (1e-4, 1e-3, 0.2)]


def xclamp_qp(N=10, nx=8, nu=3, d=1e-16, off=1e-9, r=0.0, boxes=False):
    """State 0 of every stage k >= 1 has Hessian diagonal d <= 1e-15, cross terms `off` with the other states,
    gradient r and no effect on the next state (its A' row is zero), so the first x pivot of the reference's
    stage Cholesky is exactly d and is clamped (kernel_dpotrf_c99_lib4.c:555-640) while the stage Hessian stays
    positive semidefinite (off^2 <= d Q_ll).  boxes: the mass-spring boxes, except on that state (a box term
    there would lift the pivot above the clamp)."""
    from hpmpc_amd.ocp import OCPQP, mass_spring_qp, pack_lib4, rup, unpack_lib4

    qp = mass_spring_qp(N, nx, nu, boxes=boxes)
    if boxes:
        idxb, dd, nb = [], [], qp.nb.copy()
        for k in range(N + 1):
            keep = qp.idxb[k] != (int(qp.nu[k]) if k >= 1 else -1)
            ib = qp.idxb[k][keep]
            p0, p1 = qp.pnb(k), rup(int(ib.size), 4)
            lb, ub = qp.d[k][:p0][: qp.idxb[k].size][keep], qp.d[k][p0:2 * p0][: qp.idxb[k].size][keep]
            dk = np.zeros(max(2 * p1, 1))
            dk[: ib.size], dk[p1:p1 + ib.size] = lb, ub
            idxb.append(ib.astype(np.int32))
            dd.append(dk)
            nb[k] = ib.size
        qp = OCPQP(N, qp.nx, qp.nu, nb, qp.ng, idxb, qp.BAbt, qp.RSQrq, dd, [], None)
    for k in range(1, N + 1):
        nuk, nux = int(qp.nu[k]), qp.nux(k)
        M = unpack_lib4(qp.RSQrq[k], nux + 1, nux).copy()
        j = nuk
        M[j, :] = 0.0
        M[:, j] = 0.0
        M[j, j] = d
        M[j + 1:nux, j] = off
        M[nux, j] = r
        qp.RSQrq[k] = pack_lib4(M)
        if k < N:
            Bt = unpack_lib4(qp.BAbt[k], nux + 1, int(qp.nx[k + 1])).copy()
            Bt[j, :] = 0.0
            qp.BAbt[k] = pack_lib4(Bt)
    return qp


def _check_written(name, got, ref, fill, tol):
    """Same elements written (the rest still holds the pre-filled sentinel), written values within tol."""
    got, ref = np.asarray(got)[: len(ref)], np.asarray(ref)
    w = ref != fill
    np.testing.assert_array_equal(got == fill, ~w, err_msg=name + " (written elements)")
    if w.any():
        e = float(np.max(np.abs(got[w] - ref[w]) / np.maximum(1.0, np.abs(ref[w]))))
        assert e <= tol, f"{name}: err {e:.3e}"


def check_cond_parts(case, got):
    """d_cond_BAbt / d_cond_RSQrq / d_cond_DCtd: every element the reference writes and nothing else, except the
    strict upper triangle of pRSQrq2, which the reference fills for the u_s x u_s blocks and the first stage's
    square from its work matrix and no consumer reads: there only the lower triangle is compared (and an element
    the reference leaves alone must stay untouched)."""
    from hpmpc_amd.ocp import rup, unpack_lib4

    out, f, qp = case.out, case.args["fill"], case.qp
    for j, (g, r) in enumerate(zip(got["Gamma"], out["Gamma"])):
        _check_written(f"{case.name} Gamma[{j}]", g, r, f, TOL_RIC)
    for key in ("BAbt2", "DCt2", "d2"):
        _check_written(f"{case.name} {key}", got[key], out[key], f, TOL_RIC)
    np.testing.assert_array_equal(np.asarray(got["idxb2"]), out["idxb2"].astype(np.int32), err_msg=case.name)
    nv = int(np.sum(qp.nu[: qp.N])) + int(qp.nx[0])
    n = rup(nv + 1, 4) * rup(nv, 2)
    A, B = unpack_lib4(np.asarray(got["RSQrq2"])[:n], nv + 1, nv), unpack_lib4(out["RSQrq2"][:n], nv + 1, nv)
    lo = np.tril(np.ones((nv + 1, nv), dtype=bool))
    assert np.all(A[lo] != f) and np.all(B[lo] != f), case.name
    e = float(np.max(np.abs(A[lo] - B[lo]) / np.maximum(1.0, np.abs(B[lo]))))
    assert e <= TOL_RIC, f"{case.name}: RSQrq2 lower err {e:.3e}"
    assert np.all(A[B == f] == f), case.name + " RSQrq2 wrote where the reference does not"
    flat_g, flat_r = np.asarray(got["RSQrq2"]), out["RSQrq2"]
    pad = np.ones(flat_r.size, dtype=bool)  # lib4 padding rows / columns outside the matrix
    pad[:n] = False
    assert np.all(flat_g[: flat_r.size][pad & (flat_r == f)] == f), case.name


def check_soft_res(case, got):
    """d_res_mpc_soft_tv: r_q / r_b on the stage sizes, r_d on its hard, general and first two soft blocks,
    r_z on its two soft blocks, mu; 1e-12 relative to max(1, |ref|) (residuals)."""
    from hpmpc_amd.soft import SoftQP

    sq, out = SoftQP.from_case(case), case.out
    rel = lambda g, r: float(np.max(np.abs(np.asarray(g) - r) / np.maximum(1.0, np.abs(r)), initial=0.0))
    for k in range(sq.N + 1):
        n = sq.nux(k)
        assert rel(got["rq"][k][:n], out["rq"][k][:n]) <= TOL_RIC, (case.name, "rq", k)
        if k < sq.N:
            m = int(sq.nx[k + 1])
            assert rel(got["rb"][k][:m], out["rb"][k][:m]) <= TOL_RIC, (case.name, "rb", k)
        nb, ng, ns = int(sq.nb[k]), int(sq.ng[k]), int(sq.ns[k])
        pnb, png, pns = (nb + 3) // 4 * 4, (ng + 3) // 4 * 4, (ns + 3) // 4 * 4
        os_ = 2 * pnb + 2 * png
        idx = np.r_[0:nb, pnb:pnb + nb, 2 * pnb:2 * pnb + ng, 2 * pnb + png:2 * pnb + png + ng, os_:os_ + ns,
                    os_ + pns:os_ + pns + ns].astype(int)
        assert rel(np.asarray(got["rd"][k])[idx], out["rd"][k][idx]) <= TOL_RIC, (case.name, "rd", k)
        iz = np.r_[0:ns, pns:pns + ns].astype(int)
        assert rel(np.asarray(got["rz"][k])[iz], out["rz"][k][iz]) <= TOL_RIC, (case.name, "rz", k)
    assert abs(got["mu"] - float(out["mu"])) <= TOL_RIC * max(1.0, abs(float(out["mu"]))), case.name


def check_case(case, got):
    """Assert parity of `got` against the golden outputs of `case`."""
    if case.kind == "soft_res":
        return check_soft_res(case, got)
    if case.kind == "cond_parts":
        return check_cond_parts(case, got)
    if case.kind == "soft":
        return check_soft(case, got)
    if case.kind == "pcond":
        return check_pcond(case, got)
    if case.kind in ("iface", "iface_kkt", "iface_newton", "iface_soft", "iface_mpc", "iface_mpc_kkt"):
        return check_iface(case, got)
    if case.kind == "ipm_div":
        # a diverging infeasible problem: only ret and kk to +-2 are comparable (the reference and a second c99
        # build of it differ by 2 iterations on these very cases, make_golden.py divergent())
        out = case.out
        assert int(got["ret"]) == int(out["ret"]) == 2, (case.name, got["ret"], out["ret"])
        assert abs(int(got["kk"]) - int(out["kk"])) <= 2, (case.name, got["kk"], out["kk"])
        return
    if case.kind == "pcond_sv":
        for key in ("ux", "pi"):
            e = max_err(case, key, got[key], case.out[key])
            assert e <= TOL_PCOND_SV, f"{case.name}: {key} err {e:.3e}"
        return
    out = case.out
    if "kk" in out:
        assert int(got["kk"]) == int(out["kk"]), (case.name, got["kk"], out["kk"])
        assert int(got["ret"]) == int(out["ret"]), (case.name, got["ret"], out["ret"])
    tol = TOL_RIC if case.kind in ("sv", "sv_xclamp", "trf_trs", "res", "res2") else TOL_IPM
    # an ill-conditioned headline problem carries its own gate: 4 x the spread of the reference's builds (ipm_gate_*,
    # make_golden.py gates())
    tol = case.args.get("gate", tol)
    per_key = {"stat": case.args["stat_gate"]} if "stat_gate" in case.args else {}
    if case.kind == "ipm2":
        per_key = TOL_IPM2_TIGHT if case.args["mu_tol"] < 1e-8 and int(out["kk"]) < case.args["k_max"] else TOL_IPM2
    elif case.kind == "kkt2":
        per_key = TOL_KKT2
    for key, ref in out.items():
        if key in ("kk", "ret"):
            continue
        t = per_key.get(key, TOL_STAT if key == "stat" else tol)
        if key in ("BAbt_after", "RSQrq_after"):
            for a, b in zip(got[key], ref):
                np.testing.assert_allclose(np.asarray(a)[: len(b)], b, rtol=0, atol=1e-14, err_msg=case.name + key)
            continue
        e = max_err(case, key, got[key], ref)
        assert e <= t, f"{case.name}: {key} err {e:.3e} > {t:.0e}"


def random_qp(N, nx, nu, nb=None, seed=0, box=1.0, ng=None, coupling=1.0):
    """Random well-posed OCP QP with per-stage sizes (lists of length N+1; nu[N] is forced to 0),
    random box subsets idxb (any variable order), SPD stage Hessians.  Exercises size patterns the
    mass-spring workload does not (odd sizes, nu > nx, varying stage sizes, x-only boxes).
    ng: general constraints per stage, lg <= D ux <= ug with a random dense D (0 strictly feasible).
    coupling: scale of the off-identity part of the stage Hessians (small values: diagonally dominant data, on which
    the clamp certificates hold)."""
    from hpmpc_amd.ocp import OCPQP, pack_lib4, rup

    rng = np.random.default_rng(seed)
    nx = np.asarray(nx, dtype=np.int32)
    nu = np.asarray(nu, dtype=np.int32).copy()
    nu[N] = 0
    nx[0] = 0 if nx[0] == 0 else nx[0]
    nb = np.zeros(N + 1, dtype=np.int32) if nb is None else np.asarray(nb, dtype=np.int32)
    ngv = np.zeros(N + 1, dtype=np.int32) if ng is None else np.asarray(ng, dtype=np.int32)
    BAbt, RSQrq, d, idxb, DCt = [], [], [], [], []
    for k in range(N + 1):
        nuk, nxk = int(nu[k]), int(nx[k])
        nux = nuk + nxk
        if k < N:
            nx1 = int(nx[k + 1])
            M = np.zeros((nux + 1, nx1))
            M[:nux] = 0.5 * rng.standard_normal((nux, nx1)) / np.sqrt(max(nux, 1))
            M[nux] = 0.3 * rng.standard_normal(nx1)
            BAbt.append(pack_lib4(M))
        G = rng.standard_normal((nux, nux))
        H = coupling * (G @ G.T) / max(nux, 1) + np.eye(nux)
        M = np.zeros((nux + 1, nux))
        M[:nux] = H
        M[nux] = 0.5 * rng.standard_normal(nux)
        RSQrq.append(pack_lib4(M))
        nbk = int(nb[k])
        ib = np.sort(rng.choice(nux, size=nbk, replace=False)).astype(np.int32) if nbk else np.zeros(0, np.int32)
        idxb.append(ib)
        pnb = rup(nbk, 4)
        ngk = int(ngv[k])
        png = rup(ngk, 4)
        dk = np.zeros(max(2 * pnb + 2 * png, 1))
        dk[:nbk] = -box * (0.5 + rng.random(nbk))
        dk[pnb:pnb + nbk] = box * (0.5 + rng.random(nbk))
        if ngk:
            D = rng.standard_normal((ngk, nux)) / np.sqrt(max(nux, 1))
            DCt.append(pack_lib4(D.T.copy()))
            dk[2 * pnb:2 * pnb + ngk] = -box * (0.5 + rng.random(ngk))
            dk[2 * pnb + png:2 * pnb + png + ngk] = box * (0.5 + rng.random(ngk))
        else:
            DCt.append(np.zeros(8))
        d.append(dk)
    if not ngv.any():
        DCt = []
    return OCPQP(N, nx, nu, nb, ngv, idxb, BAbt, RSQrq, d, DCt, None)


# Every comparison that took compare_ipm's divergence escape, as (kk, max |lam|): tests that allow the escape
# bound how many of their cases may take it.
DIVERGENT_SKIPS = []


def compare_ipm(case_like_qp, a, b, tol=TOL_IPM, allow_divergent=False):
    """max error of two ipm() results over valid parts.

    A primal-dual divergence (the oracle stops on alpha_min, ret 2, with |lam| > 1e12: an infeasible QP whose
    lam runs to 1e33) amplifies last-bit differences without bound -- the oracle and the reference build itself
    differ by O(1) there -- so only ret (and kk to +-2) are comparable.  That escape is taken only where the caller
    allows it (allow_divergent, for deliberately sampled non-converged problems), and every use is recorded in
    DIVERGENT_SKIPS; a converged problem (ret 0) can never take it."""
    qp = case_like_qp
    assert a["ret"] == b["ret"], (a["kk"], b["kk"], a["ret"], b["ret"])
    if b["ret"] == 2:
        lam_max = max(float(np.max(np.abs(x))) for x in b["lam"])
        if lam_max > 1e12:
            assert allow_divergent, f"oracle diverged (ret 2, |lam| = {lam_max:.1e}) on a case that must compare"
            # the iteration at which the step length of a divergence (lam growing ~10x per iteration) falls
            # below alpha_min is itself set by amplified last bits: +-2 iterations, same exit code -- the
            # reference build and the oracle differ by exactly that on the ipm_div goldens (make_golden.py)
            assert abs(a["kk"] - b["kk"]) <= 2, (a["kk"], b["kk"])
            DIVERGENT_SKIPS.append((int(b["kk"]), lam_max))
            return 0.0
    assert a["kk"] == b["kk"], (a["kk"], b["kk"], a["ret"], b["ret"])
    e = 0.0
    for k in range(qp.N + 1):
        n = qp.nux(k)
        e = max(e, float(np.max(np.abs(a["ux"][k][:n] - b["ux"][k][:n]) / np.maximum(1, np.abs(b["ux"][k][:n])),
                                initial=0)))
        if k < qp.N:
            m = int(qp.nx[k + 1])
            e = max(e, float(np.max(np.abs(a["pi"][k][:m] - b["pi"][k][:m]) / np.maximum(1, np.abs(b["pi"][k][:m])),
                                    initial=0)))
        nbk, pnb, ngk, png = int(qp.nb[k]), qp.pnb(k), int(qp.ng[k]), qp.png(k)
        idx = np.r_[0:nbk, pnb:pnb + nbk, 2 * pnb:2 * pnb + ngk, 2 * pnb + png:2 * pnb + png + ngk].astype(int)
        for key in ("lam", "t"):
            g, r = a[key][k][idx], b[key][k][idx]
            e = max(e, float(np.max(np.abs(g - r) / np.maximum(1, np.abs(r)), initial=0)))
    assert e <= tol, e
    return e


def parse_ric_driver(text):
    """ux / pi rows printed by test_problems/test_d_ric_mpc.c (d_print_mat, "%9.5f")."""
    blocks = {"ux": [], "pi": []}
    cur = None
    for line in text.splitlines():
        w = line.split()
        if w in (["ux"], ["pi"]):
            cur = w[0]
            continue
        if cur and w:
            try:
                blocks[cur].append([float(x) for x in w])
            except ValueError:
                cur = None
    return blocks


def stack_qps(qps):
    """A batch of single problems that share stage sizes and idxb."""
    from hpmpc_amd.ocp import OCPQP

    q0 = qps[0]
    return OCPQP(q0.N, q0.nx.copy(), q0.nu.copy(), q0.nb.copy(), q0.ng.copy(), [i.copy() for i in q0.idxb],
                 [np.stack([q.BAbt[k] for q in qps]) for k in range(q0.N)],
                 [np.stack([q.RSQrq[k] for q in qps]) for k in range(q0.N + 1)],
                 [np.stack([q.d[k] for q in qps]) for k in range(q0.N + 1)], [], len(qps))
