"""ctypes bindings for the HPMPC hot-path C ABI.

The same marshalling drives three libraries that export the reference's prototypes:

* ``libhpmpc_mi355x.so`` (the product: C-ABI shim + HIP kernels, symbols exactly as named in
  ``include/mpc_solvers.h`` / ``include/lqcp_solvers.h`` of the reference),
* ``oracle/liboracle.so`` (the clean-room CPU restatement, ``orc_`` prefix; test infrastructure),
* ``oracle/_ref/libhpmpc_ref.so`` (the real reference c99 build; dev container only).

This is the ctypes stub a Python maintainer of the reference would write.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .ocp import OCPQP, rup

DP = C.POINTER(C.c_double)
IP = C.POINTER(C.c_int)


def load(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return C.CDLL(path, mode=os.RTLD_LOCAL | getattr(os, "RTLD_NOW", 2))


def _dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous, (a.dtype, a.flags)
    return a.ctypes.data_as(DP)


def dpp(arrs):
    """list of float64 arrays -> double** (keeps no references: caller keeps arrs alive)."""
    return (DP * max(len(arrs), 1))(*[_dptr(a) for a in arrs])


def ipp(arrs):
    return (IP * max(len(arrs), 1))(*[np.ascontiguousarray(a, dtype=np.int32).ctypes.data_as(IP) for a in arrs])


def iv(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return (C.c_int * len(a))(*a.tolist())


def _aligned_copy(a: np.ndarray, align: int = 64) -> np.ndarray:
    buf = np.empty(a.size + align // 8, dtype=np.float64)
    off = (-buf.ctypes.data % align) // 8
    out = buf[off: off + a.size].reshape(a.shape)
    out[...] = a
    return out


class HpmpcAPI:
    """Thin wrapper calling ``<prefix><reference symbol>`` of a loaded library on an OCPQP.

    ``aligned=True`` hands the library 64-byte aligned copies of every double array (and copies them
    back after the call): the reference's X64_AVX helpers use aligned 256-bit loads."""

    def __init__(self, lib: C.CDLL, prefix: str = "", aligned: bool = False):
        self.lib = lib
        self.p = prefix
        self.aligned = aligned
        self._copies = []

    def _pp(self, arrs):
        if not self.aligned:
            return dpp(arrs)
        cps = [_aligned_copy(a) for a in arrs]
        self._copies += list(zip(arrs, cps))
        return dpp(cps)

    def _p(self, a):
        if not self.aligned:
            return _dptr(a)
        c = _aligned_copy(a)
        self._copies.append((a, c))
        return _dptr(c)

    def _sync(self):
        for a, c in self._copies:
            a[...] = c
        self._copies = []

    def fn(self, name: str):
        f = getattr(self.lib, self.p + name)
        return f

    # ---------------------------------------------------------------------------------------------
    def ric_sizes(self, qp: OCPQP):
        N = qp.N
        a = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), iv(qp.ng))
        w = self.fn("d_back_ric_rec_sv_tv_work_space_size_bytes")(*a)
        m = self.fn("d_back_ric_rec_sv_tv_memory_space_size_bytes")(*a)
        return w, m

    def ipm_ws_size(self, qp: OCPQP, res=True):
        N = qp.N
        name = "d_ip2_res_mpc_hard_tv" if res else "d_ip2_mpc_hard_tv"
        return self.fn(name + "_work_space_size_bytes")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), iv(qp.ng))

    # ---------------------------------------------------------------------------------------------
    def ric_sv(self, qp: OCPQP, *, update_b=0, b=None, update_q=0, q=None, bd=None, Qx=None, qx=None,
               compute_pi=1, compute_Pb=0, memory=None, work=None):
        """d_back_ric_rec_sv_tv_res (lqcp_solvers/d_back_ric_rec.c:112).  Returns ux, pi, Pb, memory."""
        N = qp.N
        wsz, msz = self.ric_sizes(qp)
        memory = np.zeros(msz // 8 + 8) if memory is None else memory
        work = np.zeros(wsz // 8 + 8) if work is None else work
        ux = [np.zeros(rup(qp.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        pi = [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        Pb = [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        z = [np.zeros(8)]
        b = b if b is not None else [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        q = q if q is not None else [np.zeros(rup(qp.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        bd = bd if bd is not None else z * (N + 1)
        Qx = Qx if Qx is not None else z * (N + 1)
        qx = qx if qx is not None else z * (N + 1)
        dct = qp.DCt if qp.DCt else z * (N + 1)
        self.fn("d_back_ric_rec_sv_tv_res")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), C.c_int(update_b),
            dpp(qp.BAbt), dpp(b), C.c_int(update_q), dpp(qp.RSQrq), dpp(q), dpp(bd), dpp(dct), dpp(Qx), dpp(qx),
            dpp(ux), C.c_int(compute_pi), dpp(pi), C.c_int(compute_Pb), dpp(Pb), _dptr(memory), _dptr(work))
        return ux, pi, Pb, memory

    def ric_trf(self, qp: OCPQP, *, bd=None, Qx=None, memory=None):
        N = qp.N
        wsz, msz = self.ric_sizes(qp)
        memory = np.zeros(msz // 8 + 8) if memory is None else memory
        work = np.zeros(wsz // 8 + 8)
        z = [np.zeros(8)]
        bd = bd if bd is not None else z * (N + 1)
        Qx = Qx if Qx is not None else z * (N + 1)
        dct = qp.DCt if qp.DCt else z * (N + 1)
        self.fn("d_back_ric_rec_trf_tv_res")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt), dpp(qp.RSQrq),
            dpp(dct), dpp(Qx), dpp(bd), _dptr(memory), _dptr(work))
        return memory

    def ric_trs(self, qp: OCPQP, memory, *, b, q, qx=None, compute_pi=1, compute_Pb=1, Pb=None):
        N = qp.N
        wsz, _ = self.ric_sizes(qp)
        work = np.zeros(wsz // 8 + 8)
        ux = [np.zeros(rup(qp.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        pi = [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        Pb = Pb if Pb is not None else [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        z = [np.zeros(8)]
        qx = qx if qx is not None else z * (N + 1)
        dct = qp.DCt if qp.DCt else z * (N + 1)
        self.fn("d_back_ric_rec_trs_tv_res")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt), dpp(b), dpp(q),
            dpp(dct), dpp(qx), dpp(ux), C.c_int(compute_pi), dpp(pi), C.c_int(compute_Pb), dpp(Pb),
            _dptr(memory), _dptr(work))
        return ux, pi, Pb

    # ---------------------------------------------------------------------------------------------
    def ipm(self, qp: OCPQP, *, k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1,
            ux=None, work=None, res=True):
        """d_ip2_res_mpc_hard_tv (mpc_solvers/d_ip2_res_hard.c:116), or with res=False the alternate IPM
        d_ip2_mpc_hard_tv (mpc_solvers/d_ip2_hard.c:88).  Returns dict."""
        N = qp.N
        nu_N = qp.nu.copy()
        wsz = self.ipm_ws_size(qp, res)
        work = np.zeros(wsz // 8 + 16) if work is None else work
        ux_, pi, lam, t = qp.alloc_solution()
        if ux is not None:
            for k in range(N + 1):
                n = min(len(ux_[k]), len(ux[k]))
                ux_[k][:n] = ux[k][:n]
        stat = np.zeros(5 * k_max + 5)
        kk = C.c_int(0)
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        ret = self.fn("d_ip2_res_mpc_hard_tv" if res else "d_ip2_mpc_hard_tv")(
            C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_double(alpha_min),
            C.c_int(warm_start), self._p(stat), C.c_int(N), iv(qp.nx), iv(nu_N), iv(qp.nb), ipp(qp.idxb),
            iv(qp.ng), self._pp(qp.BAbt), self._pp(qp.RSQrq), self._pp(dct), self._pp(qp.d), self._pp(ux_),
            C.c_int(compute_mult), self._pp(pi), self._pp(lam), self._pp(t), self._p(work))
        self._sync()
        return dict(ret=ret, kk=kk.value, stat=stat[: 5 * kk.value].copy(), ux=ux_, pi=pi, lam=lam, t=t,
                    work=work)

    def ipm_soft(self, sq, *, k_max=50, mu0=100.0, mu_tol=1e-8, alpha_min=1e-8, warm_start=0, compute_mult=1,
                 ux=None, work_extra=0):
        """d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:83) on a SoftQP (hpmpc_amd/soft.py).  Returns dict."""
        N = sq.N
        a = (C.c_int(N), iv(sq.nx), iv(sq.nu), iv(sq.nb), iv(sq.ng), iv(sq.ns))
        wsz = self.fn("d_ip2_mpc_soft_tv_work_space_size_bytes")(*a)
        work = np.zeros(wsz // 8 + 16 + work_extra)
        ux_, pi, lam, t = sq.alloc_solution()
        if ux is not None:
            for k in range(N + 1):
                n = min(len(ux_[k]), len(ux[k]))
                ux_[k][:n] = ux[k][:n]
        stat = np.zeros(5 * k_max + 5)
        kk = C.c_int(0)
        dct = [np.zeros(8)] * (N + 1)
        ret = self.fn("d_ip2_mpc_soft_tv")(
            C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_double(alpha_min),
            C.c_int(warm_start), self._p(stat), C.c_int(N), iv(sq.nx), iv(sq.nu), iv(sq.nb), ipp(sq.idxb),
            iv(sq.ng), iv(sq.ns), self._pp(sq.BAbt), self._pp(sq.RSQrq), self._pp(sq.Z), self._pp(sq.z),
            self._pp(dct), self._pp(sq.d), self._pp(ux_), C.c_int(compute_mult), self._pp(pi), self._pp(lam),
            self._pp(t), self._p(work))
        self._sync()
        return dict(ret=ret, kk=kk.value, stat=stat[: 5 * max(kk.value, 0)].copy(), ux=ux_, pi=pi, lam=lam, t=t)

    def residuals_soft(self, sq, q, ux, pi, lam, t):
        """d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38) at an iterate of a SoftQP (general constraints
        allowed: sq.ng / sq.DCt).  Returns rq, rb, rd, rz, mu."""
        N = sq.N
        pns = [rup(int(sq.ns[k]), 4) for k in range(N + 1)]
        rq = [np.zeros(sq.nux(k) + 8) for k in range(N + 1)]
        rb = [np.zeros(int(sq.nx[k + 1]) + 8) for k in range(N)] + [np.zeros(8)]
        rd = [np.zeros(2 * rup(int(sq.nb[k]), 4) + 2 * rup(int(sq.ng[k]), 4) + 2 * pns[k] + 8) for k in range(N + 1)]
        rz = [np.zeros(2 * pns[k] + 8) for k in range(N + 1)]
        mu = C.c_double(0.0)
        dct = sq.DCt if sq.DCt else [np.zeros(8)] * (N + 1)
        self.fn("d_res_mpc_soft_tv")(
            C.c_int(N), iv(sq.nx), iv(sq.nu), iv(sq.nb), ipp(sq.idxb), iv(sq.ng), iv(sq.ns), self._pp(sq.BAbt),
            self._pp(sq.RSQrq), self._pp(q), self._pp(sq.Z), self._pp(sq.z), self._pp(ux), self._pp(dct),
            self._pp(sq.d), self._pp(pi), self._pp(lam), self._pp(t), self._pp(rq), self._pp(rb), self._pp(rd),
            self._pp(rz), C.byref(mu))
        self._sync()
        return dict(rq=rq, rb=rb[:N], rd=rd, rz=rz, mu=mu.value)

    def prepare_ipm(self, qp: OCPQP, *, k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8):
        """Pre-marshalled d_ip2_res_mpc_hard_tv call: returns (call, kk) where call() runs one cold-start
        solve on private buffers and returns the status; kk.value holds the iteration count.  Used to
        time the CPU baseline without ctypes marshalling in the timed region (the GIL is released during
        the foreign call, so threads run solves concurrently)."""
        N = qp.N
        qp = qp.copy()
        work = np.zeros(self.ipm_ws_size(qp) // 8 + 16)
        ux, pi, lam, t = qp.alloc_solution()
        stat = np.zeros(5 * k_max + 5)
        kk = C.c_int(0)
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        args = (C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_double(alpha_min), C.c_int(0),
                _dptr(stat), C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt),
                dpp(qp.RSQrq), dpp(dct), dpp(qp.d), dpp(ux), C.c_int(1), dpp(pi), dpp(lam), dpp(t), _dptr(work))
        f = self.fn("d_ip2_res_mpc_hard_tv")
        keep = (qp, work, ux, pi, lam, t, stat, dct)

        def call():
            _ = keep
            return f(*args)

        return call, kk

    def single_newton(self, qp: OCPQP, ux0, pi0, lam0, t0, *, k_max=1, mu0=0.0, mu_tol=1e-12, alpha_min=1e-8,
                      compute_mult=1, work=None):
        N = qp.N
        wsz = self.ipm_ws_size(qp)
        work = np.zeros(wsz // 8 + 16) if work is None else work
        ux, pi, lam, t = qp.alloc_solution()
        stat = np.zeros(5 * k_max + 5)
        kk = C.c_int(0)
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        ret = self.fn("d_ip2_res_mpc_hard_tv_single_newton_step")(
            C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_double(alpha_min), C.c_int(0),
            _dptr(stat), C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt),
            dpp(qp.RSQrq), dpp(dct), dpp(qp.d), dpp(ux), C.c_int(compute_mult), dpp(pi), dpp(lam), dpp(t),
            _dptr(work), dpp(ux0), dpp(pi0), dpp(lam0), dpp(t0))
        return dict(ret=ret, kk=kk.value, stat=stat[: 5 * kk.value].copy(), ux=ux, pi=pi, lam=lam, t=t, work=work)

    def kkt_new_rhs(self, qp: OCPQP, work, b, q, compute_mult=1):
        """d_kkt_solve_new_rhs_res_mpc_hard_tv (d_ip2_res_hard.c:1922), re-using ``work`` from ipm()."""
        N = qp.N
        ux, pi, lam, t = qp.alloc_solution()
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        self.fn("d_kkt_solve_new_rhs_res_mpc_hard_tv")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt), dpp(b),
            dpp(qp.RSQrq), dpp(q), dpp(dct), dpp(qp.d), dpp(ux), C.c_int(compute_mult), dpp(pi), dpp(lam), dpp(t),
            _dptr(work))
        return dict(ux=ux, pi=pi, lam=lam, t=t)

    def residuals(self, qp: OCPQP, b, q, ux, pi, lam, t):
        """d_res_res_mpc_hard_tv (mpc_solvers/c99/d_res_ip_res_hard.c:39)."""
        N = qp.N
        rq = [np.zeros(rup(qp.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        rb = [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        rd = [np.zeros(max(qp.nconstr(k), 1) + 4) for k in range(N + 1)]
        rm = [np.zeros(max(qp.nconstr(k), 1) + 4) for k in range(N + 1)]
        work = np.zeros(2 * max([qp.png(k) for k in range(N + 1)] + [1]) + 8)
        mu = C.c_double(0.0)
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        self.fn("d_res_res_mpc_hard_tv")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt), dpp(b),
            dpp(qp.RSQrq), dpp(q), dpp(ux), dpp(dct), dpp(qp.d), dpp(pi), dpp(lam), dpp(t), _dptr(work), dpp(rq),
            dpp(rb), dpp(rd), dpp(rm), C.byref(mu))
        return dict(rq=rq, rb=rb, rd=rd, rm=rm, mu=mu.value)


    def kkt_new_rhs_plain(self, qp: OCPQP, work, b, q, d, ux, compute_mult=1):
        """d_kkt_solve_new_rhs_mpc_hard_tv (mpc_solvers/d_ip2_hard.c:626): re-solve with new b (r_A), q (r_H)
        and bounds d (r_C), re-using ``work`` from ipm(res=False); ``ux`` holds the IPM solution (its
        stage-0 state part is read when nx[0] > 0)."""
        N = qp.N
        ux_, pi, lam, t = qp.alloc_solution()
        for k in range(N + 1):
            n = min(len(ux_[k]), len(ux[k]))
            ux_[k][:n] = ux[k][:n]
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        self.fn("d_kkt_solve_new_rhs_mpc_hard_tv")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), self._pp(qp.BAbt), self._pp(b),
            self._pp(qp.RSQrq), self._pp(q), self._pp(dct), self._pp(d), self._pp(ux_), C.c_int(compute_mult),
            self._pp(pi), self._pp(lam), self._pp(t), self._p(work))
        self._sync()
        return dict(ux=ux_, pi=pi, lam=lam, t=t)

    def residuals_plain(self, qp: OCPQP, b, q, ux, pi, lam, t):
        """d_res_mpc_hard_tv (mpc_solvers/d_res_ip_hard.c:38): r_q, r_b, r_d (no r_m) and mu."""
        N = qp.N
        rq = [np.zeros(rup(qp.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        rb = [np.zeros(rup(int(qp.nx[k + 1]), 4) + 4) for k in range(N)]
        rd = [np.zeros(max(qp.nconstr(k), 1) + 4) for k in range(N + 1)]
        mu = C.c_double(0.0)
        dct = qp.DCt if qp.DCt else [np.zeros(8)] * (N + 1)
        self.fn("d_res_mpc_hard_tv")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), dpp(qp.BAbt), dpp(b),
            dpp(qp.RSQrq), dpp(q), dpp(ux), dpp(dct), dpp(qp.d), dpp(pi), dpp(lam), dpp(t), dpp(rq), dpp(rb),
            dpp(rd), C.byref(mu))
        return dict(rq=rq, rb=rb, rd=rd, mu=mu.value)


    # --------------------------------------------------------------------------------------------- partial condensing
    def part_cond_sizes(self, qp: OCPQP, N2: int):
        """d_part_cond_compute_problem_size (lqcp_solvers/d_part_cond.c:694): condensed stage sizes."""
        N = qp.N
        out = [(C.c_int * (N2 + 1))() for _ in range(4)]
        self.fn("d_part_cond_compute_problem_size")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb),
                                                    iv(qp.ng), C.c_int(N2), *out)
        return [np.array(o[:], dtype=np.int32) for o in out]

    def part_cond(self, qp: OCPQP, N2: int):
        """d_part_cond (d_part_cond.c:926): condense qp into N2 blocks.  Returns the condensed OCPQP (copied out of
        the routine's memory) and the raw memory buffer.  Its last stage is the original's, as d_part_cond sets it
        (:1052-1056); it is taken from qp rather than through the returned pointers because the reference build
        writes one int past `int cnx[N]` (:978-982) and its terminal pointers come back clobbered."""
        N = qp.N
        idxb = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        nx2, nu2, nb2, ng2 = self.part_cond_sizes(qp, N2)
        cn = [iv(a) for a in (nx2, nu2, nb2, ng2)]
        head = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(idxb), iv(qp.ng), C.c_int(N2), *cn)
        wsz = self.fn("d_part_cond_work_space_size_bytes")(*head)
        msz = self.fn("d_part_cond_memory_space_size_bytes")(*head)
        # 2x + 4 KiB headroom: the reference's own work-size formula under-counts for single-block horizons
        # (d_part_cond.c:743-866; N2 = 1 with boxes overruns it)
        memory = np.zeros(2 * (msz // 8) + 512)
        work = np.zeros(2 * (wsz // 8) + 512)
        hidxb2 = (IP * (N2 + 1))()
        pB, pR, pG, pd = ((DP * (N2 + 1))() for _ in range(4))
        dct = qp.DCt if qp.DCt else [np.zeros(8) for _ in range(N + 1)]
        self.fn("d_part_cond")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(idxb), iv(qp.ng), self._pp(qp.BAbt),
                               self._pp(qp.RSQrq), self._pp(dct), self._pp(qp.d), C.c_int(N2), cn[0], cn[1], cn[2],
                               hidxb2, cn[3], pB, pR, pG, pd, self._p(memory), self._p(work))
        self._sync()
        arr = lambda ptr, n: np.ctypeslib.as_array(ptr, shape=(max(n, 1),)).copy() if n > 0 else np.zeros(8)
        BAbt2, RSQ2, DCt2, d2, idx2 = [], [], [], [], []
        for k in range(N2):
            nux = int(nu2[k] + nx2[k])
            if True:
                BAbt2.append(arr(pB[k], rup(nux + 1, 4) * rup(int(nx2[k + 1]), 2)))
            RSQ2.append(arr(pR[k], rup(nux + 1, 4) * rup(nux, 2)))
            DCt2.append(arr(pG[k], rup(nux, 4) * rup(int(ng2[k]), 2)))
            d2.append(arr(pd[k], 2 * rup(int(nb2[k]), 4) + 2 * rup(int(ng2[k]), 4)))
            idx2.append(np.ctypeslib.as_array(hidxb2[k], shape=(int(nb2[k]),)).copy().astype(np.int32)
                        if nb2[k] > 0 else np.zeros(0, np.int32))
        RSQ2.append(qp.RSQrq[N].copy())
        DCt2.append(dct[N].copy())
        d2.append(qp.d[N].copy())
        idx2.append(idxb[N].copy())
        cqp = OCPQP(N2, nx2, nu2, nb2, ng2, idx2, BAbt2, RSQ2, d2, DCt2 if ng2.any() else [], None)
        return cqp, memory

    # the building blocks of one condensing block (d_part_cond.c:214-689): qp's N stages are the block
    @staticmethod
    def gamma_shapes(qp: OCPQP):
        """(rows, cols, lib4 size) of Gamma_j, j < N: rows sum_{i<=j} nu_i + nx_0 + 1, cols nx_{j+1}."""
        out, r = [], int(qp.nx[0]) + 1
        for j in range(qp.N):
            r += int(qp.nu[j])
            c = int(qp.nx[j + 1])
            out.append((r, c, rup(r, 4) * rup(c, 2)))
        return out

    def _cond_work(self, qp: OCPQP):
        nzM = max(int(qp.nu[k] + qp.nx[k]) + 1 for k in range(qp.N + 1))
        g = sum(2 * s for (_, _, s) in self.gamma_shapes(qp))
        return np.zeros(g + 8 * (rup(nzM, 4) + 4) ** 2 + 4096)

    def cond_BAbt(self, qp: OCPQP, fill: float = 0.0):
        """d_cond_BAbt (d_part_cond.c:214): Gamma_0..Gamma_{N-1} (lib4) and BAbt2; outputs pre-filled with fill."""
        N = qp.N
        G = [np.full(s + 8, fill) for (_, _, s) in self.gamma_shapes(qp)]
        r, c, s = self.gamma_shapes(qp)[-1]
        B2 = np.full(s + 8, fill)
        self.fn("d_cond_BAbt")(C.c_int(N), iv(qp.nx), iv(qp.nu), self._pp(qp.BAbt), self._p(self._cond_work(qp)),
                               self._pp(G), self._p(B2))
        self._sync()
        return G, B2

    def cond_RSQrq(self, qp: OCPQP, G, fill: float = 0.0):
        """d_cond_RSQrq (d_part_cond.c:312): the condensed Hessian from the Gammas G; output pre-filled with fill."""
        N = qp.N
        nv = int(np.sum(qp.nu[:N])) + int(qp.nx[0])
        R2 = np.full(rup(nv + 1, 4) * rup(nv, 2) + 8, fill)
        G = [np.ascontiguousarray(g, dtype=np.float64) for g in G] + [np.zeros(8)]
        self.fn("d_cond_RSQrq")(C.c_int(N), iv(qp.nx), iv(qp.nu), self._pp(qp.BAbt), self._pp(qp.RSQrq),
                                self._pp(G), self._p(self._cond_work(qp)), self._p(R2))
        self._sync()
        return R2

    def cond_DCtd(self, qp: OCPQP, G, fill: float = 0.0):
        """d_cond_DCtd (d_part_cond.c:579): DCt2, d2, idxb2 of the block; outputs pre-filled with fill (idxb2: -7)."""
        N = qp.N
        nv = int(np.sum(qp.nu[:N])) + int(qp.nx[0])
        nbb = int(qp.nb[0]) + sum(int(np.sum(qp.idxb[k] < qp.nu[k])) for k in range(1, N))
        nbg = sum(int(np.sum(qp.idxb[k] >= qp.nu[k])) for k in range(1, N))
        DCt2 = np.full(rup(nv, 4) * rup(nbg, 2) + 8, fill)
        d2 = np.full(2 * rup(nbb, 4) + 2 * rup(nbg, 4) + 8, fill)
        idxb2 = np.full(nbb + 4, -7, dtype=np.int32)
        idxb = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        G = [np.ascontiguousarray(g, dtype=np.float64) for g in G] + [np.zeros(8)]
        self.fn("d_cond_DCtd")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(idxb), self._pp(qp.d), self._pp(G),
                               self._p(DCt2), self._p(d2), idxb2.ctypes.data_as(IP))
        self._sync()
        return DCt2, d2, idxb2[:nbb], (nbb, nbg)

    def part_expand(self, qp: OCPQP, cqp: OCPQP, ux2, pi2, lam2, t2):
        """d_part_expand_solution (d_part_cond.c:1103): the full-space solution of qp from the condensed one."""
        N, N2 = qp.N, cqp.N
        b, q = bq_from_qp(qp)
        ux, pi, lam, t = qp.alloc_solution()
        wsz = self.fn("d_part_expand_work_space_size_bytes")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), iv(qp.ng))
        work = np.zeros(wsz // 8 + 16)
        dct = qp.DCt if qp.DCt else [np.zeros(8) for _ in range(N + 1)]
        self.fn("d_part_expand_solution")(
            C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(qp.idxb), iv(qp.ng), self._pp(qp.BAbt), self._pp(b),
            self._pp(qp.RSQrq), self._pp(q), self._pp(dct), self._pp(ux), self._pp(pi), self._pp(lam), self._pp(t),
            C.c_int(N2), iv(cqp.nx), iv(cqp.nu), iv(cqp.nb), ipp(cqp.idxb), iv(cqp.ng), self._pp(ux2), self._pp(pi2),
            self._pp(lam2), self._pp(t2), self._p(work))
        self._sync()
        return dict(ux=ux, pi=pi, lam=lam, t=t)

    def prepare_pcond(self, qp: OCPQP, N2: int):
        """Pre-marshalled configs[4] pipeline for CPU timing: returns call() running d_part_cond ->
        d_back_ric_rec_sv_tv_res (condensed, compute_pi) -> d_part_expand_solution on private buffers with
        ctypes argument tuples built once (the GIL is released inside each foreign call).  The terminal
        condensed pointers are re-pointed at the caller's stage N after every d_part_cond (the reference
        build clobbers them, see part_cond)."""
        N = qp.N
        qp = qp.copy()
        idxb = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        nx2, nu2, nb2, ng2 = self.part_cond_sizes(qp, N2)
        cn = [iv(a) for a in (nx2, nu2, nb2, ng2)]
        head = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(idxb), iv(qp.ng), C.c_int(N2), *cn)
        msz = self.fn("d_part_cond_memory_space_size_bytes")(*head)
        wsz = self.fn("d_part_cond_work_space_size_bytes")(*head)
        memory = np.zeros(2 * (msz // 8) + 512)
        work = np.zeros(2 * (wsz // 8) + 512)
        hidxb2 = (IP * (N2 + 1))()
        pB, pR, pG, pd = ((DP * (N2 + 1))() for _ in range(4))
        dct = qp.DCt if qp.DCt else [np.zeros(8) for _ in range(N + 1)]
        pBAbt, pRSQ, pDCt, pdd, pidx = dpp(qp.BAbt), dpp(qp.RSQrq), dpp(dct), dpp(qp.d), ipp(idxb)
        cond_args = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), pidx, iv(qp.ng), pBAbt, pRSQ, pDCt, pdd,
                     C.c_int(N2), cn[0], cn[1], cn[2], hidxb2, cn[3], pB, pR, pG, pd, _dptr(memory), _dptr(work))
        z1 = (C.c_int * (N2 + 1))()
        mem2 = np.zeros(self.fn("d_back_ric_rec_sv_tv_memory_space_size_bytes")(C.c_int(N2), cn[0], cn[1], z1, z1)
                        // 8 + 64)
        wrk2 = np.zeros(self.fn("d_back_ric_rec_sv_tv_work_space_size_bytes")(C.c_int(N2), cn[0], cn[1], z1, z1)
                        // 8 + 64)
        ux2 = [np.zeros(rup(int(nu2[k] + nx2[k]) + 1, 4)) for k in range(N2 + 1)]
        pi2 = [np.zeros(rup(int(nx2[k + 1]), 4) + 4) for k in range(N2)]
        Pb2 = [np.zeros(rup(int(nx2[k + 1]), 4) + 4) for k in range(N2)]
        dummy = [np.zeros(8) for _ in range(N2 + 1)]
        sv_args = (C.c_int(N2), cn[0], cn[1], z1, hidxb2, z1, C.c_int(0), pB, dpp(dummy), C.c_int(0), pR,
                   dpp(dummy), dpp(dummy), pG, dpp(dummy), dpp(dummy), dpp(ux2), C.c_int(1), dpp(pi2), C.c_int(0),
                   dpp(Pb2), _dptr(mem2), _dptr(wrk2))
        b, q = bq_from_qp(qp)
        ux, pi, lam, t = qp.alloc_solution()
        lam2 = [np.zeros(2 * rup(int(nb2[k]), 4) + 2 * rup(int(ng2[k]), 4) + 4) for k in range(N2 + 1)]
        t2 = [x.copy() for x in lam2]
        wx = np.zeros(self.fn("d_part_expand_work_space_size_bytes")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb),
                                                                    iv(qp.ng)) // 8 + 64)
        ex_args = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), pidx, iv(qp.ng), pBAbt, dpp(b), pRSQ, dpp(q), pDCt,
                   dpp(ux), dpp(pi), dpp(lam), dpp(t), C.c_int(N2), cn[0], cn[1], cn[2], hidxb2, cn[3], dpp(ux2),
                   dpp(pi2), dpp(lam2), dpp(t2), _dptr(wx))
        f_cond, f_sv, f_ex = self.fn("d_part_cond"), self.fn("d_back_ric_rec_sv_tv_res"), \
            self.fn("d_part_expand_solution")
        keep = (qp, idxb, memory, work, mem2, wrk2, ux2, pi2, Pb2, dummy, b, q, ux, pi, lam, t, lam2, t2, wx, dct)
        last = (pRSQ[N], pDCt[N], pdd[N], pidx[N])

        def call():
            _ = keep
            f_cond(*cond_args)
            pR[N2], pG[N2], pd[N2], hidxb2[N2] = last
            f_sv(*sv_args)
            f_ex(*ex_args)

        return call

    def prepare_pcond_ipm(self, qp: OCPQP, N2: int, *, k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8):
        """Pre-marshalled configs[4] IPM pipeline for CPU timing: returns (call, kk) where call() runs d_part_cond ->
        d_ip2_res_mpc_hard_tv on the condensed problem (cold start) -> d_part_expand_solution on private buffers and
        kk.value holds the condensed IPM's iteration count (ctypes argument tuples built once, the GIL released inside
        each foreign call).  The terminal condensed pointers are re-pointed at the caller's stage N after every
        d_part_cond (the reference build clobbers them, see part_cond)."""
        N = qp.N
        qp = qp.copy()
        idxb = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        nx2, nu2, nb2, ng2 = self.part_cond_sizes(qp, N2)
        cn = [iv(a) for a in (nx2, nu2, nb2, ng2)]
        head = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), ipp(idxb), iv(qp.ng), C.c_int(N2), *cn)
        msz = self.fn("d_part_cond_memory_space_size_bytes")(*head)
        wsz = self.fn("d_part_cond_work_space_size_bytes")(*head)
        memory = np.zeros(2 * (msz // 8) + 512)
        work = np.zeros(2 * (wsz // 8) + 512)
        hidxb2 = (IP * (N2 + 1))()
        pB, pR, pG, pd = ((DP * (N2 + 1))() for _ in range(4))
        dct = qp.DCt if qp.DCt else [np.zeros(8) for _ in range(N + 1)]
        pBAbt, pRSQ, pDCt, pdd, pidx = dpp(qp.BAbt), dpp(qp.RSQrq), dpp(dct), dpp(qp.d), ipp(idxb)
        cond_args = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), pidx, iv(qp.ng), pBAbt, pRSQ, pDCt, pdd,
                     C.c_int(N2), cn[0], cn[1], cn[2], hidxb2, cn[3], pB, pR, pG, pd, _dptr(memory), _dptr(work))
        wipm = np.zeros(self.fn("d_ip2_res_mpc_hard_tv_work_space_size_bytes")(C.c_int(N2), *cn) // 8 + 64)
        ux2 = [np.zeros(rup(int(nu2[k] + nx2[k]) + 1, 4) + 4) for k in range(N2 + 1)]
        pi2 = [np.zeros(rup(int(nx2[k + 1]), 4) + 4) for k in range(N2)] + [np.zeros(8)]
        lam2 = [np.zeros(2 * rup(int(nb2[k]), 4) + 2 * rup(int(ng2[k]), 4) + 4) for k in range(N2 + 1)]
        t2 = [x.copy() for x in lam2]
        stat = np.zeros(5 * k_max + 5)
        kk = C.c_int(0)
        ipm_args = (C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_double(alpha_min),
                    C.c_int(0), _dptr(stat), C.c_int(N2), cn[0], cn[1], cn[2], hidxb2, cn[3], pB, pR, pG, pd,
                    dpp(ux2), C.c_int(1), dpp(pi2), dpp(lam2), dpp(t2), _dptr(wipm))
        b, q = bq_from_qp(qp)
        ux, pi, lam, t = qp.alloc_solution()
        wx = np.zeros(self.fn("d_part_expand_work_space_size_bytes")(C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb),
                                                                    iv(qp.ng)) // 8 + 64)
        ex_args = (C.c_int(N), iv(qp.nx), iv(qp.nu), iv(qp.nb), pidx, iv(qp.ng), pBAbt, dpp(b), pRSQ, dpp(q), pDCt,
                   dpp(ux), dpp(pi), dpp(lam), dpp(t), C.c_int(N2), cn[0], cn[1], cn[2], hidxb2, cn[3], dpp(ux2),
                   dpp(pi2), dpp(lam2), dpp(t2), _dptr(wx))
        f_cond, f_ipm, f_ex = self.fn("d_part_cond"), self.fn("d_ip2_res_mpc_hard_tv"), \
            self.fn("d_part_expand_solution")
        keep = (qp, idxb, memory, work, wipm, ux2, pi2, lam2, t2, stat, b, q, ux, pi, lam, t, wx, dct)
        last = (pRSQ[N], pDCt[N], pdd[N], pidx[N])

        def call():
            _ = keep
            f_cond(*cond_args)
            pR[N2], pG[N2], pd[N2], hidxb2[N2] = last
            r = f_ipm(*ipm_args)
            f_ex(*ex_args)
            return r

        return call, kk

    # --------------------------------------------------------------------------------------------- c_interface.h
    def _iface_args(self, P, order):
        """Dense interface-form problem (oracle/iface_oracle.py) -> the wrappers' double** arguments; column-major
        for order 'F' (fortran_order_*), row-major for 'C' (c_order_*)."""
        flat = lambda M: np.ascontiguousarray(np.asarray(M, dtype=np.float64).flatten(order)).reshape(-1)
        pad = lambda v: np.concatenate([np.asarray(v, dtype=np.float64).reshape(-1), np.zeros(4)])
        keep = {}
        for key in ("A", "B", "Q", "S", "R", "C", "D"):
            keep[key] = [pad(flat(M)) for M in P[key]]
        for key in ("b", "q", "r", "lb", "ub", "lg", "ug"):
            keep[key] = [pad(v) for v in P[key]]
        return keep

    def ip_ocp(self, P, N2, *, order="F", k_max=50, mu0=2.0, mu_tol=1e-10, warm=None):
        """fortran_order_d_ip_ocp_hard_tv / c_order_d_ip_ocp_hard_tv (include/c_interface.h:62,65)."""
        N = P["N"]
        nx, nu, nb, ng = iv(P["nx"]), iv(P["nu"]), iv(P["nb"]), iv(P["ng"])
        idx = [np.ascontiguousarray(i, dtype=np.int32) for i in P["hidxb"]]
        a = self._iface_args(P, order)
        x = [np.zeros(P["nx"][k] + 4) for k in range(N + 1)]
        u = [np.zeros(P["nu"][k] + 4) for k in range(N + 1)]
        if warm is not None:
            for k in range(N + 1):
                x[k][:P["nx"][k]] = warm["x"][k]
                if k < N:
                    u[k][:P["nu"][k]] = warm["u"][k]
        pi = [np.zeros(P["nx"][k + 1] + 4) for k in range(N)]
        lam = [np.zeros(2 * P["nb"][k] + 2 * P["ng"][k] + 4) for k in range(N + 1)]
        inf = np.zeros(4)
        stat = np.zeros(5 * k_max + 5)
        wsz = self.fn("hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes")(C.c_int(N), nx, nu, nb, ipp(idx), ng,
                                                                      C.c_int(N2))
        work0 = np.zeros(wsz // 8 + 16)
        kk = C.c_int(0)
        f = self.fn("fortran_order_d_ip_ocp_hard_tv" if order == "F" else "c_order_d_ip_ocp_hard_tv")
        ret = f(C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_int(N), nx, nu, nb, ipp(idx),
                ng, C.c_int(N2), C.c_int(1 if warm is not None else 0), dpp(a["A"]), dpp(a["B"]), dpp(a["b"]),
                dpp(a["Q"]), dpp(a["S"]), dpp(a["R"]), dpp(a["q"]), dpp(a["r"]), dpp(a["lb"]), dpp(a["ub"]),
                dpp(a["C"]), dpp(a["D"]), dpp(a["lg"]), dpp(a["ug"]), dpp(x), dpp(u), dpp(pi), dpp(lam), _dptr(inf),
                _dptr(work0), _dptr(stat))
        nxv, nuv = P["nx"], P["nu"]
        return dict(status=ret, kk=kk.value, stat=stat[:5 * kk.value].copy(), inf_norm_res=inf,
                    u=[u[k][:nuv[k]] for k in range(N)], x=[x[k][:nxv[k]] for k in range(N + 1)],
                    pi=[pi[k][:nxv[k + 1]] for k in range(N)],
                    lam=[lam[k][:2 * P["nb"][k] + 2 * P["ng"][k]] for k in range(N + 1)], work0=work0)

    def ip_ocp_soft(self, P, *, k_max=50, mu0=100.0, mu_tol=1e-8, warm=None):
        """fortran_order_d_ip_ocp_soft_tv (include/c_interface.h:71) on an interface-form problem with ns / Z / z
        (oracle/iface_oracle.py random_soft_iface_problem)."""
        N = P["N"]
        nx, nu, nb, ng, ns = iv(P["nx"]), iv(P["nu"]), iv(P["nb"]), iv(P["ng"]), iv(P["ns"])
        idx = [np.ascontiguousarray(i, dtype=np.int32) for i in P["hidxb"]]
        a = self._iface_args(P, "F")
        Z = [np.concatenate([np.asarray(v, dtype=np.float64), np.zeros(4)]) for v in P["Z"]]
        z = [np.concatenate([np.asarray(v, dtype=np.float64), np.zeros(4)]) for v in P["z"]]
        x = [np.zeros(P["nx"][k] + 4) for k in range(N + 1)]
        u = [np.zeros(P["nu"][k] + 4) for k in range(N + 1)]
        if warm is not None:
            for k in range(N + 1):
                x[k][:P["nx"][k]] = warm["x"][k]
                if k < N:
                    u[k][:P["nu"][k]] = warm["u"][k]
        pi = [np.zeros(P["nx"][k + 1] + 4) for k in range(N)]
        nl = [2 * P["nb"][k] + 2 * P["ng"][k] + 4 * P["ns"][k] for k in range(N + 1)]
        lam = [np.zeros(n + 4) for n in nl]
        inf = np.zeros(4)
        stat = np.zeros(5 * k_max + 5)
        wsz = self.fn("hpmpc_d_ip_ocp_soft_tv_work_space_size_bytes")(C.c_int(N), nx, nu, nb, ipp(idx), ng, ns)
        work0 = np.zeros(wsz // 8 + 16)
        kk = C.c_int(0)
        ret = self.fn("fortran_order_d_ip_ocp_soft_tv")(
            C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_int(N), nx, nu, nb, ipp(idx), ng, ns,
            C.c_int(1 if warm is not None else 0), dpp(a["A"]), dpp(a["B"]), dpp(a["b"]), dpp(a["Q"]), dpp(a["S"]),
            dpp(a["R"]), dpp(a["q"]), dpp(a["r"]), dpp(Z), dpp(z), dpp(a["lb"]), dpp(a["ub"]), dpp(a["C"]),
            dpp(a["D"]), dpp(a["lg"]), dpp(a["ug"]), dpp(x), dpp(u), dpp(pi), dpp(lam), _dptr(inf), _dptr(work0),
            _dptr(stat))
        nxv, nuv = P["nx"], P["nu"]
        return dict(status=ret, kk=kk.value, stat=stat[:5 * max(kk.value, 0)].copy(), inf_norm_res=inf,
                    u=[u[k][:nuv[k]] for k in range(N)], x=[x[k][:nxv[k]] for k in range(N + 1)],
                    pi=[pi[k][:nxv[k + 1]] for k in range(N)], lam=[lam[k][:nl[k]] for k in range(N + 1)])

    def newton_ocp(self, P, ux0, pi0, lam0, t0, *, k_max=1, mu0=0.1, mu_tol=1e-12):
        """fortran_order_d_ip_ocp_hard_tv_single_newton_step (include/c_interface.h:66)."""
        N = P["N"]
        nx, nu, nb, ng = iv(P["nx"]), iv(P["nu"]), iv(P["nb"]), iv(P["ng"])
        idx = [np.ascontiguousarray(i, dtype=np.int32) for i in P["hidxb"]]
        a = self._iface_args(P, "F")
        x = [np.zeros(P["nx"][k] + 4) for k in range(N + 1)]
        u = [np.zeros(P["nu"][k] + 4) for k in range(N + 1)]
        pi = [np.zeros(P["nx"][k + 1] + 4) for k in range(N)]
        lam = [np.zeros(2 * P["nb"][k] + 2 * P["ng"][k] + 4) for k in range(N + 1)]
        t = [np.zeros(2 * P["nb"][k] + 2 * P["ng"][k] + 4) for k in range(N + 1)]
        inf = np.zeros(4)
        stat = np.zeros(5 * k_max + 5)
        wsz = self.fn("hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes")(C.c_int(N), nx, nu, nb, ipp(idx), ng, C.c_int(N))
        work0 = np.zeros(wsz // 8 + 16)
        kk = C.c_int(0)
        ret = self.fn("fortran_order_d_ip_ocp_hard_tv_single_newton_step")(
            C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_int(N), nx, nu, nb, ipp(idx), ng,
            C.c_int(N), C.c_int(0), dpp(a["A"]), dpp(a["B"]), dpp(a["b"]), dpp(a["Q"]), dpp(a["S"]), dpp(a["R"]),
            dpp(a["q"]), dpp(a["r"]), dpp(a["lb"]), dpp(a["ub"]), dpp(a["C"]), dpp(a["D"]), dpp(a["lg"]),
            dpp(a["ug"]), dpp(x), dpp(u), dpp(pi), dpp(lam), dpp(t), _dptr(inf), _dptr(work0), _dptr(stat),
            dpp(ux0), dpp(pi0), dpp(lam0), dpp(t0))
        nxv, nuv = P["nx"], P["nu"]
        n = [2 * P["nb"][k] + 2 * P["ng"][k] for k in range(N + 1)]
        return dict(status=ret, kk=kk.value, stat=stat[:5 * kk.value].copy(), inf_norm_res=inf,
                    u=[u[k][:nuv[k]] for k in range(N)], x=[x[k][:nxv[k]] for k in range(N + 1)],
                    pi=[pi[k][:nxv[k + 1]] for k in range(N)], lam=[lam[k][:n[k]] for k in range(N + 1)],
                    t=[t[k][:n[k]] for k in range(N + 1)])

    def kkt_ocp(self, P, work0, *, order="F"):
        """fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv / c_order_ twin (include/c_interface.h:63,67): new b, q,
        r and bounds of P on the factor ip_ocp left in work0 (full-space solve)."""
        N = P["N"]
        nx, nu, nb, ng = iv(P["nx"]), iv(P["nu"]), iv(P["nb"]), iv(P["ng"])
        idx = [np.ascontiguousarray(i, dtype=np.int32) for i in P["hidxb"]]
        a = self._iface_args(P, order)
        x = [np.zeros(P["nx"][k] + 4) for k in range(N + 1)]
        u = [np.zeros(P["nu"][k] + 4) for k in range(N + 1)]
        pi = [np.zeros(P["nx"][k + 1] + 4) for k in range(N)]
        lam = [np.zeros(2 * P["nb"][k] + 2 * P["ng"][k] + 4) for k in range(N + 1)]
        inf = np.zeros(4)
        f = self.fn("fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv" if order == "F"
                    else "c_order_d_solve_kkt_new_rhs_ocp_hard_tv")
        f(C.c_int(N), nx, nu, nb, ipp(idx), ng, dpp(a["A"]), dpp(a["B"]), dpp(a["b"]), dpp(a["Q"]), dpp(a["S"]),
          dpp(a["R"]), dpp(a["q"]), dpp(a["r"]), dpp(a["lb"]), dpp(a["ub"]), dpp(a["C"]), dpp(a["D"]), dpp(a["lg"]),
          dpp(a["ug"]), dpp(x), dpp(u), dpp(pi), dpp(lam), _dptr(inf), _dptr(work0))
        nxv, nuv = P["nx"], P["nu"]
        return dict(inf_norm_res=inf, u=[u[k][:nuv[k]] for k in range(N)], x=[x[k][:nxv[k]] for k in range(N + 1)],
                    pi=[pi[k][:nxv[k + 1]] for k in range(N)],
                    lam=[lam[k][:2 * P["nb"][k] + 2 * P["ng"][k]] for k in range(N + 1)])


    # --------------------------------------------------------------------------------- legacy c_interface.h wrappers
    @staticmethod
    def _mpc_args(M, order):
        """Legacy flat problem (oracle/iface_oracle.py random_mpc_problem, column-major stage blocks) -> the wrappers'
        double* arguments; each stage block row-major for order 'C' (c_order_*)."""
        nx, nu, ng, ngN = M["nx"], M["nu"], M["ng"], M["ngN"]
        shapes = {"A": (nx, nx), "B": (nx, nu), "Q": (nx, nx), "S": (nu, nx), "R": (nu, nu), "C": (ng, nx),
                  "D": (ng, nu), "Qf": (nx, nx), "Cf": (ngN, nx)}
        a = {}
        for key in ("A", "B", "b", "Q", "Qf", "S", "R", "q", "qf", "r", "lb", "ub", "C", "D", "lg", "ug", "Cf", "lgf",
                    "ugf"):
            v = np.asarray(M[key], dtype=np.float64).reshape(-1)
            if order == "C" and key in shapes and shapes[key][0] * shapes[key][1] > 0:
                m, n = shapes[key]
                nblk = v.size // (m * n)
                v = np.concatenate([v[i * m * n:(i + 1) * m * n].reshape((m, n), order="F").reshape(-1)
                                    for i in range(nblk)] + [v[nblk * m * n:]])
            a[key] = np.concatenate([v, np.zeros(8)])
        return a

    @staticmethod
    def mpc_lam_size(M):
        """Length of the legacy wrappers' lam / t outputs (the largest index they write, +1)."""
        N, nu, nb, ng, ngN = (M[k] for k in ("N", "nu", "nb", "ng", "ngN"))
        s = 2 * nb + 2 * ng
        return N * s + max(s, nu + max(nb - nu, 0) + nb + ngN, 2 * nb + 2 * ngN)

    def _mpc_outs(self, M, x, u, pi, lam, t, inf):
        N, nx, nu = M["N"], M["nx"], M["nu"]
        L = self.mpc_lam_size(M)
        return dict(u=u[:N * nu].copy(), x=x[:(N + 1) * nx].copy(), pi=pi[:N * nx].copy(), lam=lam[:L].copy(),
                    t=t[:L].copy(), inf_norm_res=inf.copy())

    def ip_mpc(self, M, *, order="F", k_max=50, mu0=2.0, mu_tol=1e-10, warm=None, work0=None):
        """fortran_order_d_ip_mpc_hard_tv / c_order_d_ip_mpc_hard_tv (include/c_interface.h:45,52)."""
        N, nx, nu, nb, ng, ngN = (int(M[k]) for k in ("N", "nx", "nu", "nb", "ng", "ngN"))
        a = self._mpc_args(M, order)
        x = np.zeros((N + 1) * nx + 8)
        x[:nx] = M["x0"]
        u = np.zeros(N * nu + 8)
        if warm is not None:
            x[nx:(N + 1) * nx] = warm["x"][nx:(N + 1) * nx]
            u[:N * nu] = warm["u"][:N * nu]
        pi = np.zeros(N * nx + 8)
        L = self.mpc_lam_size(M) + 8
        lam, t = np.zeros(L), np.zeros(L)
        inf = np.zeros(4)
        stat = np.zeros(5 * k_max + 5)
        if work0 is None:
            work0 = np.zeros(self.fn("hpmpc_d_ip_mpc_hard_tv_work_space_size_doubles")(
                C.c_int(N), C.c_int(nx), C.c_int(nu), C.c_int(nb), C.c_int(ng), C.c_int(ngN)) + 16)
        kk = C.c_int(0)
        f = self.fn("fortran_order_d_ip_mpc_hard_tv" if order == "F" else "c_order_d_ip_mpc_hard_tv")
        ret = f(C.byref(kk), C.c_int(k_max), C.c_double(mu0), C.c_double(mu_tol), C.c_int(N), C.c_int(nx), C.c_int(nu),
                C.c_int(nb), C.c_int(ng), C.c_int(ngN), C.c_int(int(M["ti"])), C.c_int(0),
                C.c_int(1 if warm is not None else 0), *[_dptr(a[k]) for k in (
                    "A", "B", "b", "Q", "Qf", "S", "R", "q", "qf", "r", "lb", "ub", "C", "D", "lg", "ug", "Cf", "lgf",
                    "ugf")], _dptr(x), _dptr(u), _dptr(pi), _dptr(lam), _dptr(t), _dptr(inf), _dptr(work0), _dptr(stat))
        out = self._mpc_outs(M, x, u, pi, lam, t, inf)
        out.update(status=ret, kk=kk.value, stat=stat[:5 * max(kk.value, 0)].copy(), work0=work0)
        return out

    def kkt_mpc(self, M2, work0, *, order="F"):
        """fortran_order_d_solve_kkt_new_rhs_mpc_hard_tv / c_order_ twin (include/c_interface.h:46,53): the new
        x0, b, r, q, qf and bounds of M2 on the factor ip_mpc left in work0."""
        N, nx, nu, nb, ng, ngN = (int(M2[k]) for k in ("N", "nx", "nu", "nb", "ng", "ngN"))
        a = self._mpc_args(M2, order)
        x = np.zeros((N + 1) * nx + 8)
        x[:nx] = M2["x0"]
        u = np.zeros(N * nu + 8)
        pi = np.zeros(N * nx + 8)
        L = self.mpc_lam_size(M2) + 8
        lam, t = np.zeros(L), np.zeros(L)
        inf = np.zeros(4)
        f = self.fn("fortran_order_d_solve_kkt_new_rhs_mpc_hard_tv" if order == "F"
                    else "c_order_d_solve_kkt_new_rhs_mpc_hard_tv")
        f(C.c_int(N), C.c_int(nx), C.c_int(nu), C.c_int(nb), C.c_int(ng), C.c_int(ngN), C.c_int(int(M2["ti"])),
          C.c_int(0), *[_dptr(a[k]) for k in ("A", "B", "b", "Q", "Qf", "S", "R", "q", "qf", "r", "lb", "ub", "C", "D",
                                              "lg", "ug", "Cf", "lgf", "ugf")],
          _dptr(x), _dptr(u), _dptr(pi), _dptr(lam), _dptr(t), _dptr(inf), _dptr(work0))
        return self._mpc_outs(M2, x, u, pi, lam, t, inf)

def bq_from_qp(qp: OCPQP):
    """b[k] and q[k] vectors extracted from the augmented rows (as the IPM does, d_ip2_res_hard.c:202-220)."""
    from .ocp import unpack_lib4

    b, q = [], []
    for k in range(qp.N):
        nux = qp.nux(k)
        M = unpack_lib4(qp.BAbt[k], nux + 1, int(qp.nx[k + 1]))
        bb = np.zeros(rup(int(qp.nx[k + 1]), 4) + 4)
        bb[: qp.nx[k + 1]] = M[nux]
        b.append(bb)
    for k in range(qp.N + 1):
        nux = qp.nux(k)
        M = unpack_lib4(qp.RSQrq[k], nux + 1, nux)
        qq = np.zeros(rup(nux + 1, 4) + 4)
        qq[:nux] = M[nux]
        q.append(qq)
    return b, q
