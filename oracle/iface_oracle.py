"""TEST INFRASTRUCTURE ONLY -- restatement of the high-level wrappers of include/c_interface.h.

fortran_order_d_ip_ocp_hard_tv (interfaces/c/fortran_order_interface.c:53-688) and its c_order twin
(interfaces/c/c_order_interface.c:53-691) are packing code around the hot path: dense problem data -> lib4
stage blocks (:257-380), the cost-based mu0 when mu0 <= 0 (:311-329), partial condensing when N2 < N and no
general constraints before stage N (:86-101, :388-545), the residual IPM d_ip2_res_mpc_hard_tv, the
expansion, the plain residuals d_res_mpc_hard_tv and their infinity norms (:590-686).  This module restates
that composition in numpy over ANY library exporting the low-level reference prototypes (hpmpc_amd.cabi.HpmpcAPI):
over oracle/liboracle.so it is the checker of the product's wrappers, over the reference c99 build
(oracle/_ref) it produces the goldens.  The reference wrapper sources themselves need the reference build
system's generated include/target.h and are unbuildable here, so the wrappers are pinned by this
composition over the reference's own low-level entry points.

Problems are given in "interface form": lists of dense numpy matrices A[k] (nx[k+1] x nx[k]), B[k]
(nx[k+1] x nu[k]), b[k], Q[k], S[k] (nu x nx), R[k], q[k], r[k], lb/ub[k] (nb[k]) with hidxb[k], C[k] (ng x nx),
D[k] (ng x nu), lg/ug[k].
"""
from __future__ import annotations

import numpy as np

from hpmpc_amd.cabi import bq_from_qp
from hpmpc_amd.ocp import OCPQP, pack_lib4, rup


def random_iface_problem(N, nx, nu, nb_u, nb_x, ng=None, seed=0):
    """Random well-posed OCP in interface form; stage 0 keeps x0 as a variable unless nx[0] == 0.
    nb_u / nb_x: boxed inputs / states per stage (the first ones)."""
    rng = np.random.default_rng(seed)
    nx = list(nx)
    nu = list(nu) + [0] if len(nu) == N else list(nu)
    nu[N] = 0
    ng = [0] * (N + 1) if ng is None else list(ng)
    P = dict(N=N, nx=nx, nu=nu, ng=ng, A=[], B=[], b=[], Q=[], S=[], R=[], q=[], r=[], lb=[], ub=[], hidxb=[],
             nb=[], C=[], D=[], lg=[], ug=[])
    for k in range(N + 1):
        nxk, nuk = nx[k], nu[k]
        if k < N:
            nx1 = nx[k + 1]
            P["A"].append(np.eye(nx1, nxk) + 0.2 * rng.standard_normal((nx1, nxk)) / np.sqrt(max(nxk, 1)))
            P["B"].append(rng.standard_normal((nx1, nuk)) / np.sqrt(max(nuk, 1)))
            P["b"].append(0.1 * rng.standard_normal(nx1))
        G = rng.standard_normal((nxk + nuk, nxk + nuk))
        H = G @ G.T / max(nxk + nuk, 1) + np.eye(nxk + nuk)
        P["R"].append(H[:nuk, :nuk].copy())
        P["S"].append(H[:nuk, nuk:].copy())
        P["Q"].append(H[nuk:, nuk:].copy())
        P["r"].append(0.2 * rng.standard_normal(nuk))
        P["q"].append(0.2 * rng.standard_normal(nxk))
        bu = min(nb_u[k] if isinstance(nb_u, (list, tuple)) else nb_u, nuk)
        bx = min(nb_x[k] if isinstance(nb_x, (list, tuple)) else nb_x, nxk)
        idx = np.r_[np.arange(bu), nuk + np.arange(bx)].astype(np.int32)
        P["hidxb"].append(idx)
        P["nb"].append(len(idx))
        P["lb"].append(-(0.3 + rng.random(len(idx))))
        P["ub"].append(0.3 + rng.random(len(idx)))
        g = ng[k]
        P["C"].append(rng.standard_normal((g, nxk)) / np.sqrt(max(nxk, 1)))
        P["D"].append(rng.standard_normal((g, nuk)) / np.sqrt(max(nuk, 1)) if k < N else np.zeros((g, 0)))
        P["lg"].append(-(0.5 + rng.random(g)))
        P["ug"].append(0.5 + rng.random(g))
    return P


def to_qp(P) -> OCPQP:
    """Interface form -> lib4 OCPQP exactly as the wrappers pack it (fortran_order_interface.c:257-380)."""
    N, nx, nu, ng = P["N"], P["nx"], P["nu"], P["ng"]
    BAbt, RSQ, DCt, d = [], [], [], []
    for k in range(N + 1):
        nuk, nxk = nu[k], nx[k]
        if k < N:
            M = np.zeros((nuk + nxk + 1, nx[k + 1]))
            M[:nuk] = P["B"][k].T
            M[nuk:nuk + nxk] = P["A"][k].T
            M[nuk + nxk] = P["b"][k]
            BAbt.append(pack_lib4(M))
        M = np.zeros((nuk + nxk + 1, nuk + nxk))
        M[:nuk, :nuk] = P["R"][k]
        M[nuk:nuk + nxk, :nuk] = P["S"][k].T
        M[:nuk, nuk:nuk + nxk] = P["S"][k]
        M[nuk:nuk + nxk, nuk:nuk + nxk] = P["Q"][k]
        M[nuk + nxk, :nuk] = P["r"][k]
        M[nuk + nxk, nuk:] = P["q"][k]
        RSQ.append(pack_lib4(M))
        g = ng[k]
        if g:
            Dt = np.zeros((nuk + nxk, g))
            Dt[:nuk] = P["D"][k].T
            Dt[nuk:] = P["C"][k].T
            DCt.append(pack_lib4(Dt))
        else:
            DCt.append(np.zeros(8))
        nbk = P["nb"][k]
        pnb, png = rup(nbk, 4), rup(g, 4)
        dk = np.zeros(max(2 * pnb + 2 * png, 1))
        dk[:nbk] = P["lb"][k]
        dk[pnb:pnb + nbk] = P["ub"][k]
        dk[2 * pnb:2 * pnb + g] = P["lg"][k]
        dk[2 * pnb + png:2 * pnb + png + g] = P["ug"][k]
        d.append(dk)
    return OCPQP(N, np.array(nx, np.int32), np.array(nu, np.int32), np.array(P["nb"], np.int32),
                 np.array(ng, np.int32), [i.copy() for i in P["hidxb"]], BAbt, RSQ, d,
                 DCt if any(ng) else [], None)


def auto_mu0(P):
    """:311-329: mu0 <= 0 -> the largest entry of R, S, Q, r, q (stage N: Q, q)."""
    m = 0.0
    for k in range(P["N"] + 1):
        for key in ("R", "S", "Q", "r", "q"):
            a = np.asarray(P[key][k])
            if a.size:
                m = max(m, float(a.max()))
    return m


def ip_ocp(api, P, N2, k_max=50, mu0=2.0, mu_tol=1e-10, warm=None):
    """fortran_order_d_ip_ocp_hard_tv restated over `api` (the row-major twin computes the same)."""
    N, nx, nu, ng, nb = P["N"], P["nx"], P["nu"], P["ng"], P["nb"]
    qp = to_qp(P)
    if mu0 <= 0:
        mu0 = auto_mu0(P)
    if N2 > N or any(g > 0 for g in ng[:N]):
        N2 = N
    if N2 < N:
        c, _ = api.part_cond(qp.copy(), N2)
        r = api.ipm(c, k_max=k_max, mu0=mu0, mu_tol=mu_tol, alpha_min=1e-8)
        e = api.part_expand(qp, c, r["ux"], r["pi"], r["lam"], r["t"])
        ux, pi, lam, t = e["ux"], e["pi"], e["lam"], e["t"]
    else:
        kw = {}
        if warm is not None:
            kw = dict(warm_start=1, ux=[np.r_[warm["u"][k] if k < N else [], warm["x"][k]] for k in range(N + 1)])
        r = api.ipm(qp.copy(), k_max=k_max, mu0=mu0, mu_tol=mu_tol, alpha_min=1e-8, **kw)
        ux, pi, lam, t = r["ux"], r["pi"], r["lam"], r["t"]
    out = finish(api, P, qp, ux, pi, lam, t)
    out.update(status=r["ret"], kk=r["kk"], stat=r["stat"])
    return out


def finish(api, P, qp, ux, pi, lam, t):
    """Outputs (:590-686): u, x, the equality-box fix, residual infinity norms, pi, compact lam."""
    N, nx, nu, ng, nb = P["N"], P["nx"], P["nu"], P["ng"], P["nb"]
    u = [np.array(ux[k][:nu[k]]) for k in range(N)]
    x = [np.array(ux[k][nu[k]:nu[k] + nx[k]]) for k in range(N + 1)]
    for k in range(N):
        for j in range(nb[k]):
            if P["hidxb"][k][j] >= nu[k]:
                break
            if P["lb"][k][j] == P["ub"][k][j]:
                u[k][P["hidxb"][k][j]] = P["lb"][k][j]
    b, q = bq_from_qp(qp)
    res = api.residuals_plain(qp, b, q, ux, pi, lam, t)
    n0 = max(abs(res["rq"][0][0]), max(float(np.max(np.abs(res["rq"][k][:nu[k] + nx[k]]), initial=0)) for k in range(N)),
             float(np.max(np.abs(res["rq"][N][:nx[N]]), initial=0)))
    n1 = max(abs(res["rb"][0][0]), max(float(np.max(np.abs(res["rb"][k][:nx[k + 1]]), initial=0)) for k in range(N)))
    n2 = abs(res["rd"][0][0])
    for k in range(N + 1):
        pnb, png = rup(nb[k], 4), rup(ng[k], 4)
        idx = np.r_[0:nb[k], pnb:pnb + nb[k], 2 * pnb:2 * pnb + ng[k], 2 * pnb + png:2 * pnb + png + ng[k]].astype(int)
        if idx.size:
            n2 = max(n2, float(np.max(np.abs(res["rd"][k][idx]))))
    lam_c = []
    for k in range(N + 1):
        pnb, png = rup(nb[k], 4), rup(ng[k], 4)
        lam_c.append(np.r_[lam[k][:nb[k]], lam[k][pnb:pnb + nb[k]], lam[k][2 * pnb:2 * pnb + ng[k]],
                           lam[k][2 * pnb + png:2 * pnb + png + ng[k]]])
    return dict(u=u, x=x, pi=[np.array(pi[k][:nx[k + 1]]) for k in range(N)], lam=lam_c,
                inf_norm_res=np.array([n0, n1, n2, res["mu"]]))


def newton_ocp(api, P, ux0, pi0, lam0, t0, k_max=1, mu0=0.1, mu_tol=1e-12):
    """fortran_order_d_ip_ocp_hard_tv_single_newton_step (interfaces/c/fortran_order_interface.c:690-1080): the same
    packing, always the full space (its N2 is computed and never used), d_ip2_res_mpc_hard_tv_single_newton_step from
    the caller's (ux0, pi0, lam0, t0) with the fixed centering target mu0 (no cost-based mu0), then the outputs of the
    IPM wrapper plus t, compact like lam (:1057-1075)."""
    N, nb, ng = P["N"], P["nb"], P["ng"]
    qp = to_qp(P)
    r = api.single_newton(qp.copy(), ux0, pi0, lam0, t0, k_max=k_max, mu0=mu0, mu_tol=mu_tol)
    out = finish(api, P, qp, r["ux"], r["pi"], r["lam"], r["t"])
    t_c = []
    for k in range(N + 1):
        pnb, png = rup(nb[k], 4), rup(ng[k], 4)
        t = r["t"][k]
        t_c.append(np.r_[t[:nb[k]], t[pnb:pnb + nb[k]], t[2 * pnb:2 * pnb + ng[k]], t[2 * pnb + png:2 * pnb + png + ng[k]]])
    out.update(t=t_c, status=r["ret"], kk=r["kk"], stat=r["stat"])
    return out


def kkt_ocp(api, P, P2, k_max=50, mu0=2.0, mu_tol=1e-10):
    """fortran_order_d_ip_ocp_hard_tv on P (full space), then fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv with
    the right-hand sides of P2 (b, q, r, bounds; same matrices): d_kkt_solve_new_rhs_res_mpc_hard_tv on the IPM's
    persisted factor and iterate (d_ip2_res_hard.c:1922-2299), then the wrapper's outputs."""
    qp = to_qp(P)
    r = api.ipm(qp.copy(), k_max=k_max, mu0=mu0 if mu0 > 0 else auto_mu0(P), mu_tol=mu_tol, alpha_min=1e-8)
    qp2 = to_qp(P2)
    b2, q2 = bq_from_qp(qp2)
    k = api.kkt_new_rhs(qp2.copy(), r["work"], b2, q2)
    return finish(api, P2, qp2, k["ux"], k["pi"], k["lam"], k["t"])


def new_rhs(P, seed=1):
    """P with perturbed b, q, r and bounds (the data a KKT re-solve takes)."""
    rng = np.random.default_rng(seed)
    Q = {k: ([np.array(a, copy=True) for a in v] if isinstance(v, list) else v) for k, v in P.items()}
    for key in ("b", "q", "r"):
        Q[key] = [v + 0.05 * rng.standard_normal(v.shape) for v in P[key]]
    for key in ("lb", "lg"):
        Q[key] = [v - 0.05 * rng.random(v.shape) for v in P[key]]
    for key in ("ub", "ug"):
        Q[key] = [v + 0.05 * rng.random(v.shape) for v in P[key]]
    return Q


SHAPES = {"A": lambda P, k: (P["nx"][k + 1], P["nx"][k]), "B": lambda P, k: (P["nx"][k + 1], P["nu"][k]),
          "Q": lambda P, k: (P["nx"][k], P["nx"][k]), "S": lambda P, k: (P["nu"][k], P["nx"][k]),
          "R": lambda P, k: (P["nu"][k], P["nu"][k]), "C": lambda P, k: (P["ng"][k], P["nx"][k]),
          "D": lambda P, k: (P["ng"][k], P["nu"][k])}


def to_flat(P):
    """Interface-form problem -> dict of lists of flat float arrays (golden storage)."""
    out = {}
    for key in ("A", "B", "Q", "S", "R", "C", "D", "b", "q", "r", "lb", "ub", "lg", "ug"):
        out["P_" + key] = [np.asarray(M, dtype=np.float64).reshape(-1) for M in P[key]]
    out["P_hidxb"] = [np.asarray(i, dtype=np.float64) for i in P["hidxb"]]
    if "ns" in P:  # soft constraints
        out["P_Z"] = [np.asarray(v, dtype=np.float64) for v in P["Z"]]
        out["P_z"] = [np.asarray(v, dtype=np.float64) for v in P["z"]]
        out["P_ns"] = [np.asarray(P["ns"], dtype=np.float64)]
    return out


def from_flat(N, nx, nu, nb, ng, inp):
    P = dict(N=N, nx=[int(v) for v in nx], nu=[int(v) for v in nu], nb=[int(v) for v in nb],
             ng=[int(v) for v in ng])
    for key in ("b", "q", "r", "lb", "ub", "lg", "ug"):
        P[key] = [np.array(v) for v in inp["P_" + key]]
    P["hidxb"] = [np.array(v).astype(np.int32) for v in inp["P_hidxb"]]
    for key, shp in SHAPES.items():
        P[key] = [np.array(v).reshape(shp(P, k)) for k, v in enumerate(inp["P_" + key])]
    if "P_ns" in inp:
        P["ns"] = [int(v) for v in inp["P_ns"][0]]
        P["Z"] = [np.array(v) for v in inp["P_Z"]]
        P["z"] = [np.array(v) for v in inp["P_z"]]
    return P


# ------------------------------------------------------------------------------------------------- soft constraints
def random_soft_iface_problem(N, nx, nu, seed=0, Zq=0.5, zl=10.0):
    """Random soft-constrained OCP in interface form, in the reference driver's shape (test_d_ip_soft.c): hard
    boxes on every input of stages 0..N-1 (nb = nu), soft boxes on every state of stages 1..N (ns = nx), penalties
    Z = Zq, z = zl; x0 is stage 0's affine term (nx[0] = 0)."""
    rng = np.random.default_rng(seed)
    nxv = [0] + [nx] * N
    nuv = [nu] * N + [0]
    P = dict(N=N, nx=nxv, nu=nuv, ng=[0] * (N + 1), A=[], B=[], b=[], Q=[], S=[], R=[], q=[], r=[], lb=[], ub=[],
             hidxb=[], nb=[], ns=[], Z=[], z=[], C=[], D=[], lg=[], ug=[])
    x0 = 2.0 * rng.standard_normal(nx)
    for k in range(N + 1):
        nxk, nuk = nxv[k], nuv[k]
        if k < N:
            A = np.eye(nx) + 0.1 * rng.standard_normal((nx, nx)) / np.sqrt(nx)
            B = rng.standard_normal((nx, nuk)) / np.sqrt(max(nuk, 1))
            P["A"].append(A[:, :nxk].copy())
            P["B"].append(B)
            P["b"].append(A @ x0 if k == 0 else 0.05 * rng.standard_normal(nx))
        G = rng.standard_normal((nxk + nuk, nxk + nuk))
        H = 0.5 * G @ G.T / max(nxk + nuk, 1) + 0.5 * np.eye(nxk + nuk)
        P["R"].append(H[:nuk, :nuk].copy())
        P["S"].append(H[:nuk, nuk:].copy())
        P["Q"].append(H[nuk:, nuk:].copy())
        P["r"].append(0.2 * rng.standard_normal(nuk))
        P["q"].append(0.2 * rng.standard_normal(nxk))
        nbk, nsk = nuk, (nxk if k > 0 else 0)
        P["hidxb"].append(np.r_[np.arange(nbk), nuk + np.arange(nsk)].astype(np.int32))
        P["nb"].append(nbk)
        P["ns"].append(nsk)
        P["lb"].append(np.r_[-(0.5 + rng.random(nbk)), -(0.8 + 0.4 * rng.random(nsk))])
        P["ub"].append(np.r_[0.5 + rng.random(nbk), 0.8 + 0.4 * rng.random(nsk)])
        P["Z"].append(np.full(2 * nsk, Zq))
        P["z"].append(np.full(2 * nsk, zl))
        P["C"].append(np.zeros((0, nxk)))
        P["D"].append(np.zeros((0, nuk)))
        P["lg"].append(np.zeros(0))
        P["ug"].append(np.zeros(0))
    return P


def to_soft_qp(P):
    """Interface form -> the SoftQP fortran_order_d_ip_ocp_soft_tv packs (interfaces/c/fortran_order_interface.c:
    1653-1799): the hard OCP blocks as to_qp, Z[k] = [lower | upper] padded to pns, d = [lb | ub | lg | ug | ls | us]
    with the soft bounds read at lb[k][nb + i] / ub[k][nb + i].  z is NOT packed: the reference wrapper never copies
    z into its hz (:1712-1719 fill hZ only), so the IPM sees the zeros of a zeroed work0."""
    from hpmpc_amd.soft import SoftQP

    N = P["N"]
    hard = dict(P, lb=[P["lb"][k][:P["nb"][k]] for k in range(N + 1)], ub=[P["ub"][k][:P["nb"][k]] for k in range(N + 1)],
                hidxb=[P["hidxb"][k][:P["nb"][k]] for k in range(N + 1)])
    qp = to_qp(hard)
    Z, z, d = [], [], []
    for k in range(N + 1):
        nb, ng, ns = P["nb"][k], P["ng"][k], P["ns"][k]
        pnb, png, pns = rup(nb, 4), rup(ng, 4), rup(ns, 4)
        Zk = np.zeros(2 * pns + 4)
        Zk[:ns] = P["Z"][k][:ns]
        Zk[pns:pns + ns] = P["Z"][k][ns:2 * ns]
        Z.append(Zk)
        z.append(np.zeros(2 * pns + 4))
        dk = np.zeros(2 * pnb + 2 * png + 2 * pns + 4)
        dk[:2 * pnb + 2 * png] = qp.d[k][:2 * pnb + 2 * png]
        dk[2 * pnb + 2 * png:2 * pnb + 2 * png + ns] = P["lb"][k][nb:nb + ns]
        dk[2 * pnb + 2 * png + pns:2 * pnb + 2 * png + pns + ns] = P["ub"][k][nb:nb + ns]
        d.append(dk)
    idxb = [np.ascontiguousarray(i, dtype=np.int32) for i in P["hidxb"]]
    return SoftQP(N, qp.nx.copy(), qp.nu.copy(), qp.nb.copy(), np.array(P["ns"], np.int32), idxb, qp.BAbt,
                  qp.RSQrq, d, Z, z, qp.ng.copy(), qp.DCt)


def ip_ocp_soft(api, P, k_max=50, mu0=100.0, mu_tol=1e-8, warm=None):
    """fortran_order_d_ip_ocp_soft_tv (interfaces/c/fortran_order_interface.c:1442-1971): pack (to_soft_qp), mu0 <= 0
    -> the largest entry of R, S, Q, r, q, Z, z (:1723-1740, no absolute value), d_ip2_mpc_soft_tv on the full
    space, then the residuals d_res_mpc_soft_tv and their infinity norms (:1876-1924) and the compact outputs
    (u, x, pi, lam = [lo nb | up nb | lg ng | ug ng | 4 soft blocks of ns]).  The reference wrapper passes its
    residual call's arguments shifted by one (an extra hb after hpBAbt, no hrz: :1880 vs mpc_solvers.h:71), so
    its inf_norm_res is computed on scrambled inputs; this composition (and the product) calls it as declared."""
    N, nx, nu, nb, ng, ns = P["N"], P["nx"], P["nu"], P["nb"], P["ng"], P["ns"]
    sq = to_soft_qp(P)
    if mu0 <= 0:
        m = 0.0
        for k in range(N + 1):
            keys = ("R", "S", "Q", "r", "q", "Z", "z") if k < N else ("Q", "q", "Z", "z")
            for key in keys:
                a = np.asarray(P[key][k])
                if a.size:
                    m = max(m, float(a.max()))
        mu0 = m
    kw = {}
    if warm is not None:
        kw = dict(warm_start=1, ux=[np.r_[warm["u"][k] if k < N else [], warm["x"][k]] for k in range(N + 1)])
    r = api.ipm_soft(sq.copy(), k_max=k_max, mu0=mu0, mu_tol=mu_tol, alpha_min=1e-8, work_extra=1 << 16, **kw)
    ux, pi, lam, t = r["ux"], r["pi"], r["lam"], r["t"]
    q = [np.r_[P["r"][k] if k < N else [], P["q"][k], np.zeros(8)] for k in range(N + 1)]
    res = api.residuals_soft(sq, q, ux, pi, lam, t)
    n0 = max(abs(res["rq"][0][0]), max(float(np.max(np.abs(res["rq"][k][:nu[k] + nx[k]]), initial=0)) for k in range(N)),
             float(np.max(np.abs(res["rq"][N][:nx[N]]), initial=0)))
    n1 = max(abs(res["rb"][0][0]), max(float(np.max(np.abs(res["rb"][k][:nx[k + 1]]), initial=0)) for k in range(N)))
    n2 = abs(res["rd"][0][0])
    lam_c = []
    for k in range(N + 1):
        pnb, png, pns = rup(nb[k], 4), rup(ng[k], 4), rup(ns[k], 4)
        o = 2 * pnb + 2 * png
        idx = np.r_[0:nb[k], pnb:pnb + nb[k], 2 * pnb:2 * pnb + ng[k], 2 * pnb + png:2 * pnb + png + ng[k],
                    o:o + ns[k], o + pns:o + pns + ns[k]].astype(int)
        if idx.size:
            n2 = max(n2, float(np.max(np.abs(res["rd"][k][idx]))))
        lam_c.append(np.concatenate([lam[k][:nb[k]], lam[k][pnb:pnb + nb[k]], lam[k][2 * pnb:2 * pnb + ng[k]],
                                     lam[k][2 * pnb + png:2 * pnb + png + ng[k]]] +
                                    [lam[k][o + s * pns:o + s * pns + ns[k]] for s in range(4)]))
    return dict(u=[np.array(ux[k][:nu[k]]) for k in range(N)], x=[np.array(ux[k][nu[k]:nu[k] + nx[k]]) for k in range(N + 1)],
                pi=[np.array(pi[k][:nx[k + 1]]) for k in range(N)], lam=lam_c,
                inf_norm_res=np.array([n0, n1, n2, res["mu"]]), status=r["ret"], kk=r["kk"], stat=r["stat"])


# ------------------------------------------------------------------------------------------------- legacy MPC wrappers
# fortran_order_d_ip_mpc_hard_tv / c_order_d_ip_mpc_hard_tv (interfaces/c/fortran_order_interface.c:1975-3013,
# c_order_interface.c:1052-2082) and their KKT re-solves (fortran_order_interface.c:3017-3779,
# c_order_interface.c:2083-2848): uniform stage sizes, flat arrays, a time_invariant flag, x0 folded into stage 0
# (nx[0] = 0) and the alternate IPM d_ip2_mpc_hard_tv.  Restated step by step, including the reference's
# deterministic quirks; where the reference reads memory it never wrote or reads past an array, the evident intent
# is taken instead (each case is listed in DESIGN.md §3c and in hpmpc_capi_mpc.cpp).
MPC_KEYS = ("A", "B", "b", "Q", "Qf", "S", "R", "q", "qf", "r", "lb", "ub", "C", "D", "lg", "ug", "Cf", "lgf", "ugf",
            "x0")
MPC_SHAPES = {"A": lambda M: (M["nx"], M["nx"]), "B": lambda M: (M["nx"], M["nu"]), "Q": lambda M: (M["nx"], M["nx"]),
              "S": lambda M: (M["nu"], M["nx"]), "R": lambda M: (M["nu"], M["nu"]), "C": lambda M: (M["ng"], M["nx"]),
              "D": lambda M: (M["ng"], M["nu"])}


def _li(sd, i, j):
    """lib4 index of element (i, j) of a panel-major matrix with panel stride sd."""
    return (i // 4) * 4 * sd + i % 4 + 4 * j


def random_mpc_problem(N, nx, nu, nb, ng, ngN, ti, seed=0, eq=()):
    """Random problem in the legacy flat column-major format.  Time-invariant: one copy of each stage array (lg / ug
    still per stage: the wrapper indexes them by stage either way); time-variant: N copies.  lb / ub hold nb bounds
    per stage ([inputs (nu) | states]), (N + 1) blocks when time-variant (stage N's state bounds at nb N + nu).
    eq: input indices whose bounds are made equal (lb == ub) on every stage."""
    rng = np.random.default_rng(seed)
    S_ = 1 if ti else N
    M = dict(N=N, nx=nx, nu=nu, nb=nb, ng=ng, ngN=ngN, ti=int(ti))
    A, B, b, Q, S, R, q, r, C, D = [], [], [], [], [], [], [], [], [], []
    for _ in range(S_):
        A.append(np.eye(nx) + 0.2 * rng.standard_normal((nx, nx)) / np.sqrt(nx))
        B.append(rng.standard_normal((nx, nu)) / np.sqrt(nu))
        b.append(0.1 * rng.standard_normal(nx))
        G = rng.standard_normal((nx + nu, nx + nu))
        H = G @ G.T / (nx + nu) + np.eye(nx + nu)
        R.append(H[:nu, :nu])
        S.append(H[:nu, nu:])
        Q.append(H[nu:, nu:])
        r.append(0.2 * rng.standard_normal(nu))
        q.append(0.2 * rng.standard_normal(nx))
        C.append(rng.standard_normal((ng, nx)) / np.sqrt(nx))
        D.append(rng.standard_normal((ng, nu)) / np.sqrt(nu))
    G = rng.standard_normal((nx, nx))
    flatF = lambda L: np.concatenate([np.asarray(m, dtype=np.float64).reshape(-1, order="F") for m in L])
    M.update(A=flatF(A), B=flatF(B), b=flatF(b), Q=flatF(Q), S=flatF(S), R=flatF(R), q=flatF(q), r=flatF(r),
             C=flatF(C) if ng else np.zeros(1), D=flatF(D) if ng else np.zeros(1))
    M["Qf"] = flatF([G @ G.T / nx + np.eye(nx)])
    M["qf"] = 0.2 * rng.standard_normal(nx)
    nlb = nb if ti else nb * (N + 1)
    M["lb"] = -(1.0 + rng.random(nlb))
    M["ub"] = 1.0 + rng.random(nlb)
    for blk in range(1 if ti else N + 1):
        for i in eq:
            if i < min(nb, nu):
                M["ub"][blk * nb + i] = M["lb"][blk * nb + i]
    M["lg"] = -(0.5 + rng.random(max(N * ng, 1)))
    M["ug"] = 0.5 + rng.random(max(N * ng, 1))
    M["Cf"] = rng.standard_normal((ngN, nx)).reshape(-1, order="F") / np.sqrt(nx) if ngN else np.zeros(1)
    M["lgf"] = -(0.5 + rng.random(max(ngN, 1)))
    M["ugf"] = 0.5 + rng.random(max(ngN, 1))
    M["x0"] = 0.5 * rng.standard_normal(nx)
    return M


def mpc_new_rhs(M, seed=1):
    """M with perturbed x0, b, r, q, qf and bounds (what the legacy KKT wrapper re-packs; same matrices)."""
    rng = np.random.default_rng(seed)
    M2 = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in M.items()}
    for key in ("x0", "b", "r", "q", "qf"):
        M2[key] = M[key] + 0.05 * rng.standard_normal(M[key].shape)
    for key in ("lb", "lg", "lgf"):
        M2[key] = M[key] - 0.05 * rng.random(M[key].shape)
    for key in ("ub", "ug", "ugf"):
        M2[key] = M[key] + 0.05 * rng.random(M[key].shape)
    return M2


def mpc_to_flat(M):
    """Legacy problem -> golden extras (lists of flat float arrays) and args."""
    return {k: [np.asarray(M[k], dtype=np.float64)] for k in MPC_KEYS}


def mpc_from_flat(args, inp):
    M = {k: int(args[k]) for k in ("N", "nx", "nu", "nb", "ng", "ngN", "ti")}
    for k in MPC_KEYS:
        M[k] = np.asarray(inp[k][0])
    return M


def mpc_sizes(M):
    """Stage sizes the wrapper builds (:2029-2062): x0 folded into stage 0, nbu = min(nb, nu) input boxes on stage 0,
    nb on the middle stages, nb - nu state boxes on stage N, idxb[k] = 0..nbb[k]-1."""
    N, nx, nu, nb, ng, ngN = (M[k] for k in ("N", "nx", "nu", "nb", "ng", "ngN"))
    nbu = min(nb, nu)
    nxx = [0] + [nx] * N
    nuu = [nu] * N + [0]
    nbb = [nbu] + [nb] * (N - 1) + [max(nb - nu, 0)]
    ngg = [ng] * N + [ngN]
    return nbu, nxx, nuu, nbb, ngg


def _mpc_mat(M, key, k):
    """Dense stage-k matrix `key` (time-invariant: the single copy)."""
    m, n = MPC_SHAPES[key](M)
    o = 0 if M["ti"] else k * m * n
    return M[key][o:o + m * n].reshape((m, n), order="F")


def _mpc_vec(M, key, k, n):
    o = 0 if M["ti"] else k * n
    return M[key][o:o + n]


def mpc_pack(M, kkt=False, base=None):
    """The wrapper's lib4 problem (IPM wrapper :2213-2757) or, with kkt=True, the KKT wrapper's re-pack of the
    right-hand sides on top of `base` (the IPM wrapper's packed data, :3248-3366 / time-variant :3480-3560).
    Returns an OCPQP (stage blocks, bounds d) plus hb, hrq (the separate b / q vectors)."""
    N, nx, nu, nb, ng, ngN, ti = (M[k] for k in ("N", "nx", "nu", "nb", "ng", "ngN", "ti"))
    nbu, nxx, nuu, nbb, ngg = mpc_sizes(M)
    pnz, pnx, pnb, png, pngN = rup(nx + nu + 1, 4), rup(nx, 4), rup(nb, 4), rup(ng, 4), rup(ngN, 4)
    cnux, cnu, cnx, cng, cngN = rup(nu + nx, 2), rup(nu, 2), rup(nx, 2), rup(ng, 2), rup(ngN, 2)
    x0 = M["x0"]
    if base is None:
        BAbt = [np.zeros(pnz * cnx + 8) for _ in range(N)]
        RSQ = [np.zeros(pnz * cnux + 8) for _ in range(N + 1)]
        DCt = [np.zeros(pnz * max(cng, cngN, 2) + 8) for _ in range(N + 1)]
    else:
        BAbt, RSQ, DCt = [a.copy() for a in base.BAbt], [a.copy() for a in base.RSQrq], [a.copy() for a in base.DCt]
    hb = [np.zeros(pnx + 4) for _ in range(N)]
    hrq = [np.zeros(pnz + 4) for _ in range(N + 1)]
    d = [np.zeros(2 * pnb + 2 * (png if k < N else pngN) + 4) for k in range(N + 1)]
    # stage 0: b0 = A0 x0 + b0 (:2561-2572), r0 = r0 + S0 x0 (:2628-2639)
    A0, B0 = _mpc_mat(M, "A", 0), _mpc_mat(M, "B", 0)
    hb[0][:nx] = A0 @ x0 + _mpc_vec(M, "b", 0, nx)
    r0 = _mpc_vec(M, "r", 0, nu) + _mpc_mat(M, "S", 0) @ x0
    for i in range(nu):  # B0' into rows 0..nu-1 (the KKT wrapper restores it, :3264)
        for j in range(nx):
            BAbt[0][_li(cnx, i, j)] = B0[j, i]
    if kkt:
        hrq[0][:nu] = r0
    else:
        for j in range(nx):
            BAbt[0][_li(cnx, nu, j)] = hb[0][j]
        R0 = _mpc_mat(M, "R", 0)
        for i in range(nu):
            for j in range(nu):
                RSQ[0][_li(cnu, i, j)] = R0[i, j]
            RSQ[0][_li(cnu, nu, i)] = r0[i]
    for k in range(1, N):
        bk = _mpc_vec(M, "b", k, nx)
        hb[k][:nx] = bk
        rk, qk = _mpc_vec(M, "r", k, nu), _mpc_vec(M, "q", k, nx)
        if kkt:
            hrq[k][:nu], hrq[k][nu:nu + nx] = rk, qk
            continue
        Ak, Bk = _mpc_mat(M, "A", k), _mpc_mat(M, "B", k)
        Rk, Sk, Qk = _mpc_mat(M, "R", k), _mpc_mat(M, "S", k), _mpc_mat(M, "Q", k)
        for j in range(nx):
            for i in range(nu):
                BAbt[k][_li(cnx, i, j)] = Bk[j, i]
            for i in range(nx):
                BAbt[k][_li(cnx, nu + i, j)] = Ak[j, i]
            BAbt[k][_li(cnx, nu + nx, j)] = bk[j]
        for i in range(nu):
            for j in range(nu):
                RSQ[k][_li(cnux, i, j)] = Rk[i, j]
            RSQ[k][_li(cnux, nu + nx, i)] = rk[i]
        for i in range(nx):
            for j in range(nu):
                RSQ[k][_li(cnux, nu + i, j)] = Sk[j, i]
            for j in range(nx):
                RSQ[k][_li(cnux, nu + i, nu + j)] = Qk[i, j]
            RSQ[k][_li(cnux, nu + nx, nu + i)] = qk[i]
    Qf = M["Qf"][:nx * nx].reshape((nx, nx), order="F")
    if kkt:
        hrq[N][:nx] = M["qf"][:nx]
    else:
        for i in range(nx):
            for j in range(nx):
                RSQ[N][_li(cnx, i, j)] = Qf[i, j]
            RSQ[N][_li(cnx, nx, i)] = M["qf"][i]
        if ng > 0:  # general constraints (:2592-2603): [D'; C'] (stage 0: D' only)
            for k in range(N):
                Dk = _mpc_mat(M, "D", k)
                for i in range(nu):
                    for j in range(ng):
                        DCt[k][_li(cng, i, j)] = Dk[j, i]
                if k > 0:
                    Ck = _mpc_mat(M, "C", k)
                    for i in range(nx):
                        for j in range(ng):
                            DCt[k][_li(cng, nu + i, j)] = Ck[j, i]
        if ngN > 0:
            Cf = M["Cf"][:ngN * nx].reshape((ngN, nx), order="F")
            for i in range(nx):
                for j in range(ngN):
                    DCt[N][_li(cngN, i, j)] = Cf[j, i]
    # bounds (:2683-2753).  lb / ub of stage k start at nb k (time-variant) or 0; stage N's state bounds at
    # nb N + nu (the loop index the wrapper leaves at N) or nu.
    lb, ub = M["lb"], M["ub"]
    blk = lambda k: 0 if ti else nb * k
    for k in range(N):
        p0 = rup(nbb[k], 4)
        for i in range(nbu):
            lo, up = lb[i + blk(k)], ub[i + blk(k)]
            if kkt or lo != up:  # the KKT wrapper copies the bounds as they are (:3300-3316)
                d[k][i], d[k][i + p0] = lo, up
            else:  # input equality constraint: folded into b (:2695-2705)
                for ll in range(nx):
                    # the b row is addressed with panel (nxx + nuu) / 4 but in-panel row (nx + nu) % 4 (:2698)
                    BAbt[k][((nxx[k] + nuu[k]) // 4) * cnx * 4 + (nx + nu) % 4 + ll * 4] += BAbt[k][_li(cnx, i, ll)] * lo
                    BAbt[k][_li(cnx, i, ll)] = 0.0
                d[k][i], d[k][i + p0] = lo + 1e3, up - 1e3
    for k in range(1, N):
        p0 = rup(nbb[k], 4)
        for i in range(nu, nbb[k]):
            d[k][i], d[k][i + p0] = lb[i + blk(k)], ub[i + blk(k)]
    p0 = rup(nbb[N], 4)
    for i in range(nbb[N]):
        d[N][i], d[N][i + p0] = lb[nu + i + blk(N)], ub[nu + i + blk(N)]
    if ng > 0:
        for k in range(N):
            p0, g0 = rup(nbb[k], 4), rup(ngg[k], 4)
            # time-invariant: the middle stages share one bound vector, so the last stage's bounds win (:2425-2433)
            kk_ = N - 1 if (ti and k > 0) else k
            for i in range(ng):
                d[k][2 * p0 + i], d[k][2 * p0 + g0 + i] = M["lg"][i + ng * kk_], M["ug"][i + ng * kk_]
    if ngN > 0:
        p0, g0 = rup(nbb[N], 4), rup(ngN, 4)
        for i in range(ngN):
            d[N][2 * p0 + i], d[N][2 * p0 + g0 + i] = M["lgf"][i], M["ugf"][i]
    # the residual's right-hand sides (:2846-2867): b as packed, q = the data's r, q (stage 0: r without S x0)
    if not kkt:
        for k in range(N):
            hrq[k][:nu] = _mpc_vec(M, "r", k, nu)
            if k > 0:
                hrq[k][nu:nu + nx] = _mpc_vec(M, "q", k, nx)
        hrq[N][:nx] = M["qf"][:nx]
    idxb = [np.arange(nbb[k], dtype=np.int32) for k in range(N + 1)]
    qp = OCPQP(N, np.array(nxx, np.int32), np.array(nuu, np.int32), np.array(nbb, np.int32), np.array(ngg, np.int32),
               idxb, BAbt, RSQ, d, DCt, None)
    return qp, hb, hrq


def mpc_mu0(M):
    """mu0 <= 0 (:2320-2340 time-invariant with absolute values, :2659-2675 time-variant without).  The reference
    reads qf[nx] (one past qf) in both, and in the time-invariant case the stage-1 slots R + nu^2, S + nu nx, ... of
    single-stage arrays; here qf[0..nx) and the single stage are read."""
    N, nx, nu, ti = M["N"], M["nx"], M["nu"], M["ti"]
    f = (lambda a: np.abs(a)) if ti else (lambda a: a)
    m = 0.0
    parts = [_mpc_mat(M, "R", 0), _mpc_vec(M, "r", 0, nu)]
    for k in range(1, 2 if ti else N):
        if k < N:
            parts += [_mpc_mat(M, "R", k), _mpc_mat(M, "S", k), _mpc_mat(M, "Q", k), _mpc_vec(M, "r", k, nu),
                      _mpc_vec(M, "q", k, nx)]
    parts += [M["Qf"][:nx * nx], M["qf"][:nx]]
    for p in parts:
        if np.size(p):
            m = max(m, float(np.max(f(np.asarray(p)))))
    return m


def mpc_outputs(M, qp, hb, hrq, ux, pi, lam, t, res, eqfix, gen_norm=True):
    """Outputs (:2802-3007): u, x (stages 1..N), the input-equality fix, inf_norm_res, pi, lam / t in the wrapper's
    layout (stage stride 2 nb + 2 ng; box lower at 0, upper at nb + ng; general lower at nb, upper at 2 nb + ng;
    stage N's boxes at nu + j, upper offset nb + ngN).  The stage-N box term of inf_norm_res[2] reads r_d of stage N
    (the reference reads r_q of stage N there, :2920-2925, partly memory it never wrote).  gen_norm=False: the
    c_order KKT wrapper, whose norm skips the general constraints of stages 0..N-1."""
    N, nx, nu, nb, ng, ngN = (M[k] for k in ("N", "nx", "nu", "nb", "ng", "ngN"))
    nbu, nxx, nuu, nbb, ngg = mpc_sizes(M)
    blk = lambda k: 0 if M["ti"] else nb * k
    u = np.zeros(N * nu)
    x = np.zeros((N + 1) * nx)
    x[:nx] = M["x0"]
    for k in range(N):
        u[k * nu:(k + 1) * nu] = ux[k][:nu]
    for k in range(1, N + 1):
        x[k * nx:(k + 1) * nx] = ux[k][nuu[k]:nuu[k] + nx]
    if eqfix:
        for k in range(N):
            for i in range(nbu):
                if M["lb"][i + blk(k)] == M["ub"][i + blk(k)]:
                    u[i + nu * k] = M["lb"][i + blk(k)]
    rq, rb, rd = res["rq"], res["rb"], res["rd"]
    n0 = max([abs(rq[0][0])] + [abs(v) for v in rq[0][:nu]] +
             [abs(v) for k in range(1, N) for v in rq[k][:nu + nx]] + [abs(v) for v in rq[N][:nx]])
    n1 = max([abs(rb[0][0])] + [abs(v) for k in range(N) for v in rb[k][:nx]])
    n2 = abs(rd[0][0])
    for k in range(N + 1):
        p0 = rup(nbb[k], 4)
        cnt = nbu if k == 0 else (nb if k < N else nbb[N])
        for j in range(cnt):
            n2 = max(n2, abs(rd[k][j]), abs(rd[k][p0 + j]))
    for k in range(N + 1):
        if k < N and not gen_norm:
            continue
        p0, g0 = rup(nbb[k], 4), rup(ngg[k], 4)
        for j in range(2 * p0, 2 * p0 + ngg[k]):
            n2 = max(n2, abs(rd[k][j]), abs(rd[k][g0 + j]))
    pi_o = np.zeros(N * nx)
    for k in range(N):
        pi_o[k * nx:(k + 1) * nx] = pi[k][:nx]
    L = mpc_lam_size(M)
    lam_o, t_o = np.zeros(L), np.zeros(L)
    s = 2 * nb + 2 * ng
    for src, dst in ((lam, lam_o), (t, t_o)):
        for k in range(N):
            p0 = rup(nbb[k], 4)
            for j in range(nbu if k == 0 else nb):
                dst[j + k * s] = src[k][j]
                dst[j + k * s + nb + ng] = src[k][p0 + j]
        p0 = rup(nbb[N], 4)
        for j in range(nbb[N]):
            dst[nu + j + N * s] = src[N][j]
            dst[nu + j + N * s + nb + ngN] = src[N][p0 + j]
        for k in range(N):
            p0, g0 = rup(nbb[k], 4), rup(ngg[k], 4)
            for j in range(ng):
                dst[j + k * s + nb] = src[k][2 * p0 + j]
                dst[j + k * s + nb + ng + nb] = src[k][2 * p0 + g0 + j]
        p0, g0 = rup(nbb[N], 4), rup(ngN, 4)
        for j in range(ngN):
            dst[j + N * s + nb] = src[N][2 * p0 + j]
            dst[j + N * s + nb + ngN + nb] = src[N][2 * p0 + g0 + j]
    return dict(u=u, x=x, pi=pi_o, lam=lam_o, t=t_o, inf_norm_res=np.array([n0, n1, n2, res["mu"]]))


def mpc_lam_size(M):
    """Length of the wrappers' lam / t outputs (the largest index they write, +1)."""
    N, nu, nb, ng, ngN = (M[k] for k in ("N", "nu", "nb", "ng", "ngN"))
    nbN = max(nb - nu, 0)
    s = 2 * nb + 2 * ng
    return N * s + max(s, nu + nbN + nb + ngN, 2 * nb + 2 * ngN)


def ip_mpc(api, M, k_max=50, mu0=2.0, mu_tol=1e-10, warm=None):
    """fortran_order_d_ip_mpc_hard_tv restated over `api`: pack, mu0, warm start (u, x of stages 0..N-1 / 1..N),
    d_ip2_mpc_hard_tv, then the residuals d_res_mpc_hard_tv and the outputs.  Returns the outputs plus the IPM's
    work (for kkt_mpc) and the packed problem."""
    N, nx, nu = M["N"], M["nx"], M["nu"]
    qp, hb, hrq = mpc_pack(M)
    if mu0 <= 0:
        mu0 = mpc_mu0(M)
    kw = {}
    if warm is not None:
        ux0 = [np.r_[warm["u"][k * nu:(k + 1) * nu] if k < N else [], warm["x"][k * nx:(k + 1) * nx] if k > 0 else []]
               for k in range(N + 1)]
        kw = dict(warm_start=1, ux=ux0)
    r = api.ipm(qp.copy(), k_max=k_max, mu0=mu0, mu_tol=mu_tol, alpha_min=1e-8, res=False, **kw)
    res = api.residuals_plain(qp, hb, hrq, r["ux"], r["pi"], r["lam"], r["t"])
    out = mpc_outputs(M, qp, hb, hrq, r["ux"], r["pi"], r["lam"], r["t"], res, eqfix=True)
    out.update(status=r["ret"], kk=r["kk"], stat=r["stat"], work=r["work"], qp=qp, ux=r["ux"])
    return out


def kkt_mpc(api, M, M2, k_max=50, mu0=2.0, mu_tol=1e-10, order="F"):
    """fortran_order_d_ip_mpc_hard_tv on M, then fortran_order_d_solve_kkt_new_rhs_mpc_hard_tv with the
    right-hand sides of M2 (x0, b, r, q, bounds; same matrices): d_kkt_solve_new_rhs_mpc_hard_tv on the IPM's
    work, with stage 0's B' re-packed over the IPM's data and the bounds copied as they are, then the residuals
    and outputs (no input-equality fix; the c_order twin's norm skips the general constraints of stages < N)."""
    ip = ip_mpc(api, M, k_max=k_max, mu0=mu0, mu_tol=mu_tol)
    qp2, hb2, hrq2 = mpc_pack(M2, kkt=True, base=ip["qp"])
    k = api.kkt_new_rhs_plain(qp2, ip["work"], hb2, hrq2, qp2.d, ip["ux"])
    _, _, hrq_res = mpc_pack(M2)
    res = api.residuals_plain(qp2, hb2, hrq_res, k["ux"], k["pi"], k["lam"], k["t"])
    return mpc_outputs(M2, qp2, hb2, hrq_res, k["ux"], k["pi"], k["lam"], k["t"], res, eqfix=False,
                       gen_norm=(order == "F"))
