"""Run a golden case through any library exporting the reference prototypes and compare outputs."""
import numpy as np

from hpmpc_amd.cabi import bq_from_qp

TOL_RIC = 1e-12   # Riccati sv/trf/trs: |a-b| <= TOL * max(1, |ref|)   
TOL_IPM = 1e-10   # IPM ux/pi/lam/t with identical iteration count
TOL_STAT = 1e-9


def run_case(api, case):
    """Execute `case` with `api`; returns dict of outputs keyed like case.out."""
    qp = case.fresh_qp()
    a = case.args
    inp = case.inp
    if case.kind == "sv":
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
    if case.kind == "ipm":
        kw = dict(k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"])
        if a.get("warm_start"):
            kw.update(warm_start=1, ux=inp["ux0"])
        r = api.ipm(qp, **kw)
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    if case.kind == "kkt":
        r = api.ipm(qp, k_max=int(a["k_max"]), mu0=a["mu0"], mu_tol=a["mu_tol"], alpha_min=a["alpha_min"])
        k = api.kkt_new_rhs(qp, r["work"], inp["b2"], inp["q2"])
        return dict(ux=k["ux"], pi=k["pi"], lam=k["lam"], t=k["t"])
    if case.kind == "res":
        r = api.residuals(qp, inp["b"], inp["q"], inp["ux"], inp["pi"], inp["lam"], inp["t"])
        return dict(rq=r["rq"], rb=r["rb"], rd=r["rd"], rm=r["rm"], mu=r["mu"])
    if case.kind == "newton":
        r = api.single_newton(qp, inp["ux0"], inp["pi0"], inp["lam0"], inp["t0"], k_max=int(a["k_max"]),
                              mu0=a["mu0"])
        return dict(ux=r["ux"], pi=r["pi"], lam=r["lam"], t=r["t"], stat=r["stat"], kk=r["kk"], ret=r["ret"])
    raise ValueError(case.kind)


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


def check_case(case, got):
    """Assert parity of `got` against the golden outputs of `case`."""
    out = case.out
    if "kk" in out:
        assert int(got["kk"]) == int(out["kk"]), (case.name, got["kk"], out["kk"])
        assert int(got["ret"]) == int(out["ret"]), (case.name, got["ret"], out["ret"])
    tol = TOL_RIC if case.kind in ("sv", "trf_trs", "res") else TOL_IPM
    for key, ref in out.items():
        if key in ("kk", "ret"):
            continue
        t = TOL_STAT if key == "stat" else tol
        if key in ("BAbt_after", "RSQrq_after"):
            for a, b in zip(got[key], ref):
                np.testing.assert_allclose(np.asarray(a)[: len(b)], b, rtol=0, atol=1e-14, err_msg=case.name + key)
            continue
        e = max_err(case, key, got[key], ref)
        assert e <= t, f"{case.name}: {key} err {e:.3e} > {t:.0e}"
