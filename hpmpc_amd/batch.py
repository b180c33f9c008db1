"""Batched, device-resident front end of libhpmpc_mi355x.so (additive API).

A batch is ``nprob`` independent QPs that share stage sizes and box indices.  All arrays live in
HBM as problem-major torch tensors (torch is plumbing here: allocation, streams, events); the solve
itself is one launch of the HIP kernels through the library's C ABI:

    BAbt  (nprob, packB)   lib4 stage blocks, stage k at offB[k]      (d_ip2_res_hard.c pBAbt[k])
    RSQrq (nprob, packR)   lib4 stage blocks, stage k at offR[k]      (pQ[k])
    d     (nprob, N+1, 32) [lb (pnb) | ub (pnb)] per stage            (d[k])
    ux    (nprob, N+1, 16) variable order u..x                        (ux[k])
    pi    (nprob, N+1, 16) over x_{k+1}                               (pi[k])
    lam/t (nprob, N+1, 32) reference padded layout                    (lam[k] / t[k])
    ws    (nprob, ws_doubles) factor + persistent IPM iterate

There is no CPU fallback: constructing a solver without a GPU or without the built library raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .ocp import OCPQP

_LIB = None
# HPMPC_MI355X_LIB: another build of the same library (A/B timing of two builds on one box, tools/gpu_ab.sh)
LIBPATH = os.environ.get("HPMPC_MI355X_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                             "libhpmpc_mi355x.so")


def lib() -> C.CDLL:
    """Load the in-tree HIP library (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIBPATH):
            raise RuntimeError(f"libhpmpc_mi355x.so not built ({LIBPATH}); run __graft_entry__.build()")
        L = C.CDLL(LIBPATH, mode=os.RTLD_LOCAL | getattr(os, "RTLD_NOW", 2))
        vp, i, d, ll = C.c_void_p, C.c_int, C.c_double, C.c_longlong
        L.hpmpc_mi355x_plan_create.restype = vp
        L.hpmpc_mi355x_plan_create.argtypes = [i, vp, vp, vp, vp, vp]
        L.hpmpc_mi355x_plan_destroy.argtypes = [vp]
        L.hpmpc_mi355x_ws_doubles.restype = ll
        L.hpmpc_mi355x_ws_doubles.argtypes = [vp]
        L.hpmpc_mi355x_ipm_solo.restype = i
        L.hpmpc_mi355x_ipm_solo.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i, i, vp,
                                            vp, vp, vp]
        L.hpmpc_mi355x_ipm_batch.restype = i
        L.hpmpc_mi355x_ipm_batch.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i, i, vp,
                                             vp, vp, vp]
        L.hpmpc_mi355x_ipm_pass.restype = i
        L.hpmpc_mi355x_ipm_pass.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i, i, vp,
                                            vp, vp, i, vp]
        L.hpmpc_mi355x_ipm_batch_profiled.restype = i
        L.hpmpc_mi355x_ipm_batch_profiled.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i,
                                                      i, vp, vp, vp, vp, vp]
        L.hpmpc_mi355x_ipm_queue.restype = i
        L.hpmpc_mi355x_ipm_queue.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i, i,
                                             vp, vp, vp, vp, vp, vp]
        L.hpmpc_mi355x_ric_sv_batch.restype = i
        L.hpmpc_mi355x_ric_sv_batch.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, i, i, vp, vp]
        L.hpmpc_mi355x_ric_trf_batch.restype = i
        L.hpmpc_mi355x_ric_trf_batch.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp]
        L.hpmpc_mi355x_ric_trs_batch.restype = i
        L.hpmpc_mi355x_ric_trs_batch.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, i, i, vp, vp]
        L.hpmpc_mi355x_last_error.restype = i
        L.hpmpc_mi355x_version.restype = C.c_char_p
        _LIB = L
    return _LIB


class _Layout(C.Structure):
    _fields_ = [("BAbt_stride", C.c_longlong), ("RSQrq_stride", C.c_longlong),
                ("BAbt_off", C.POINTER(C.c_longlong)), ("RSQrq_off", C.POINTER(C.c_longlong)),
                ("BAbt_shared", C.POINTER(C.c_ubyte)), ("RSQrq_shared", C.POINTER(C.c_ubyte))]


def aliased_layout(qp: OCPQP):
    """The time-invariant / aliased device layout of a batch whose problems differ only in stage 0's BAbt block (its b
    row carries A x0 + b): every other stage block is the same in every problem, and every inner stage the same as
    stage 1 (the reference drivers' aliasing, test_problems/test_d_ip_hard.c:652-662).  Returns the packed arrays
    (BAbt: [shared inner block | stage 0 of problem 0 | stage 0 of problem 1 | ...], RSQrq: [stage 0 | inner | N],
    shared by all problems), the strides, the offsets and the shared flags of hpmpc_mi355x_layout.  Raises
    ValueError when the data do not alias that way."""
    N, P = qp.N, qp.batch
    for k in range(1, N):
        for a, b in ((qp.BAbt[k], qp.BAbt[1]), (qp.RSQrq[k], qp.RSQrq[1])):
            if a.shape != b.shape or not np.array_equal(a, b):
                raise ValueError(f"stage {k} is not stage 1's (time-invariant inner stages needed)")
    for arr in list(qp.BAbt[1:]) + list(qp.RSQrq):
        if not (arr == arr[:1]).all():
            raise ValueError("stage data other than BAbt_0 differ between problems")
    inner = qp.BAbt[1][0] if N > 1 else np.zeros(0)
    b0 = qp.BAbt[0]
    hB = np.concatenate([inner, b0.reshape(-1)])
    offB = np.array([inner.size] + [0] * (N - 1), dtype=np.int64)
    shB = np.array([0] + [1] * (N - 1), dtype=np.uint8)
    r0, r1, rN = qp.RSQrq[0][0], qp.RSQrq[1][0], qp.RSQrq[N][0]
    hR = np.concatenate([r0, r1, rN])
    offR = np.array([0] + [r0.size] * (N - 1) + [r0.size + r1.size], dtype=np.int64)
    shR = np.ones(N + 1, dtype=np.uint8)
    return hB, hR, int(b0.shape[1]), 0, offB, offR, shB, shR


def stage_offsets(qp: OCPQP):
    """Offsets (doubles) of every stage block inside one problem's packed BAbt / RSQrq arrays, and the
    packed lengths: stage k of BAbt at offB[k], of RSQrq at offR[k] (the reference's lib4 blocks, unchanged)."""
    N = qp.N
    offB = np.zeros(N, dtype=np.int64)
    offR = np.zeros(N + 1, dtype=np.int64)
    o = 0
    for k in range(N):
        offB[k] = o
        o += qp.BAbt[k].shape[-1]
    packB = o
    o = 0
    for k in range(N + 1):
        offR[k] = o
        o += qp.RSQrq[k].shape[-1]
    return offB, offR, packB, o


def pack_batch(qp: OCPQP):
    """Problem-major host arrays of a batched OCPQP: BAbt (nprob, packB), RSQrq (nprob, packR), d (nprob, N+1, 32)
    -- the layout BatchSolver keeps in HBM and hpmpc_amd.shard scatters."""
    N = qp.N
    hB = np.ascontiguousarray(np.concatenate([a for a in qp.BAbt], axis=1))
    hR = np.ascontiguousarray(np.concatenate([a for a in qp.RSQrq], axis=1))
    hd = np.zeros((qp.batch, N + 1, 32))
    for k in range(N + 1):
        n = qp.d[k].shape[1]
        hd[:, k, :n] = qp.d[k]
    return hB, hR, hd


def unpack_batch(template: OCPQP, hB, hR, hd) -> OCPQP:
    """Inverse of pack_batch: the batched OCPQP whose stage sizes / idxb are the template's and whose data are
    the packed arrays (numpy or CPU tensors)."""
    hB, hR, hd = (np.asarray(x) for x in (hB, hR, hd))
    offB, offR, _, _ = stage_offsets(template)
    N = template.N
    BAbt = [hB[:, offB[k]:offB[k] + template.BAbt[k].shape[-1]].copy() for k in range(N)]
    RSQrq = [hR[:, offR[k]:offR[k] + template.RSQrq[k].shape[-1]].copy() for k in range(N + 1)]
    d = [hd[:, k, :template.d[k].shape[-1]].copy() for k in range(N + 1)]
    return OCPQP(N, template.nx.copy(), template.nu.copy(), template.nb.copy(), template.ng.copy(),
                 [i.copy() for i in template.idxb], BAbt, RSQrq, d, [], hB.shape[0])


class BatchSolver:
    """Device-resident batch of OCP QPs + the batched HPMPC entry points.

    ``nprob`` given: the batch's data are not uploaded from ``qp`` (which then only supplies stage sizes and
    idxb); BAbt / RSQrq / d are allocated for ``nprob`` problems and filled by the caller, e.g. by the rank-0
    scatter of hpmpc_amd.shard."""

    def __init__(self, qp: OCPQP, device="cuda", k_max: int = 50, nprob: int | None = None, aliased: bool = False):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("BatchSolver needs a GPU (HIP device); there is no CPU fallback")
        assert nprob is not None or qp.batch is not None, "BatchSolver takes a batched OCPQP"
        self.torch = torch
        self.qp = qp
        self.N = N = qp.N
        self.nprob = qp.batch if nprob is None else int(nprob)
        self.k_max = k_max
        self.dev = torch.device(device)
        L = lib()
        self._keep = []
        idx_arrs = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        self._keep.append(idx_arrs)
        idxp = (C.POINTER(C.c_int) * (N + 1))(*[a.ctypes.data_as(C.POINTER(C.c_int)) for a in idx_arrs])
        self._keep.append(idxp)
        ints = lambda a: np.ascontiguousarray(a, dtype=np.int32)
        self._nx, self._nu, self._nb, self._ng = ints(qp.nx), ints(qp.nu), ints(qp.nb), ints(qp.ng)
        self.plan = L.hpmpc_mi355x_plan_create(N, self._nx.ctypes.data, self._nu.ctypes.data, self._nb.ctypes.data,
                                               C.cast(idxp, C.c_void_p), self._ng.ctypes.data)
        if not self.plan:
            raise ValueError(f"unsupported problem sizes for the GPU path (code {L.hpmpc_mi355x_last_error()})")
        # problem-major packed inputs
        f64 = torch.float64
        P = self.nprob
        self.aliased = aliased
        if aliased:  # one copy of every shared stage block (hpmpc_mi355x_layout BAbt_shared / RSQrq_shared)
            assert nprob is None
            hB, hR, sB, sR, offB, offR, shB, shR = aliased_layout(qp)
            self.offB, self.offR, self._sh = offB, offR, (shB, shR)
            u8 = C.POINTER(C.c_ubyte)
            self.layout = _Layout(sB, sR, offB.ctypes.data_as(C.POINTER(C.c_longlong)),
                                  offR.ctypes.data_as(C.POINTER(C.c_longlong)), shB.ctypes.data_as(u8),
                                  shR.ctypes.data_as(u8))
            self.BAbt = torch.from_numpy(hB).to(self.dev)
            self.RSQrq = torch.from_numpy(hR).to(self.dev)
            self.d = torch.from_numpy(pack_batch(qp)[2]).to(self.dev)
        else:
            offB, offR, packB, packR = stage_offsets(qp)
            self.offB, self.offR = offB, offR
            self.layout = _Layout(packB, packR, offB.ctypes.data_as(C.POINTER(C.c_longlong)),
                                  offR.ctypes.data_as(C.POINTER(C.c_longlong)), None, None)
        if aliased:
            pass
        elif nprob is None:
            hB, hR, hd = pack_batch(qp)
            self.BAbt = torch.from_numpy(hB).to(self.dev)
            self.RSQrq = torch.from_numpy(hR).to(self.dev)
            self.d = torch.from_numpy(hd).to(self.dev)
        else:
            self.BAbt = torch.zeros((P, packB), dtype=f64, device=self.dev)
            self.RSQrq = torch.zeros((P, packR), dtype=f64, device=self.dev)
            self.d = torch.zeros((P, N + 1, 32), dtype=f64, device=self.dev)
        self.ux = torch.zeros((P, N + 1, 16), dtype=f64, device=self.dev)
        self.pi = torch.zeros((P, N + 1, 16), dtype=f64, device=self.dev)
        self.lam = torch.zeros((P, N + 1, 32), dtype=f64, device=self.dev)
        self.t = torch.zeros((P, N + 1, 32), dtype=f64, device=self.dev)
        self.Pb = torch.zeros((P, N + 1, 16), dtype=f64, device=self.dev)
        self.wsd = int(L.hpmpc_mi355x_ws_doubles(self.plan))
        self.ws = torch.zeros((P, self.wsd), dtype=f64, device=self.dev)
        self.kk = torch.zeros(P, dtype=torch.int32, device=self.dev)
        self.ret = torch.zeros(P, dtype=torch.int32, device=self.dev)
        self.stat = torch.zeros((P, 5 * k_max), dtype=f64, device=self.dev)

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                lib().hpmpc_mi355x_plan_destroy(self.plan)
        except Exception:
            pass

    def _stream(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def ipm(self, *, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1, p0=0, count=None):
        """Batched d_ip2_res_mpc_hard_tv (asynchronous on torch's current stream)."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ipm_batch(
            self.plan, C.byref(self.layout), self.nprob, p0, count, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            self.d.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.lam.data_ptr(), self.t.data_ptr(),
            self.ws.data_ptr(), self.k_max, mu0, mu_tol, alpha_min, warm_start, compute_mult, self.kk.data_ptr(),
            self.ret.data_ptr(), self.stat.data_ptr(), self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ipm_batch failed ({rc})")

    def ipm_solo(self, *, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1, p0=0, count=None):
        """ipm() as the latency path: each problem's whole solve in one launch (hpmpc_mi355x_ipm_solo)."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ipm_solo(
            self.plan, C.byref(self.layout), self.nprob, p0, count, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            self.d.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.lam.data_ptr(), self.t.data_ptr(),
            self.ws.data_ptr(), self.k_max, mu0, mu_tol, alpha_min, warm_start, compute_mult, self.kk.data_ptr(),
            self.ret.data_ptr(), self.stat.data_ptr(), self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ipm_solo failed ({rc})")

    def ipm_pass(self, pss, *, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1, p0=0,
                 count=None):
        """One pass of the batched IPM (0 init, 1 factorisation, 2 predictor, 3 corrector, 4 update);
        ipm() == pass 0 then k_max rounds of passes 1..4."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ipm_pass(
            self.plan, C.byref(self.layout), self.nprob, p0, count, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            self.d.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.lam.data_ptr(), self.t.data_ptr(),
            self.ws.data_ptr(), self.k_max, mu0, mu_tol, alpha_min, warm_start, compute_mult, self.kk.data_ptr(),
            self.ret.data_ptr(), self.stat.data_ptr(), pss, self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ipm_pass failed ({rc})")

    def ipm_profiled(self, *, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1):
        """ipm() with hipEvents around every pass kernel (synchronous).  Returns the summed device time
        (ms) of passes [init, factorisation, predictor, corrector, update]."""
        out = np.zeros(5)
        rc = lib().hpmpc_mi355x_ipm_batch_profiled(
            self.plan, C.byref(self.layout), self.nprob, 0, self.nprob, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            self.d.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.lam.data_ptr(), self.t.data_ptr(),
            self.ws.data_ptr(), self.k_max, mu0, mu_tol, alpha_min, warm_start, compute_mult, self.kk.data_ptr(),
            self.ret.data_ptr(), self.stat.data_ptr(), out.ctypes.data, self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ipm_batch_profiled failed ({rc})")
        return out

    def queue(self, nq: int, n_slots: int | None = None) -> "IpmQueue":
        """A continuous-batching IPM over this batch's data (entry q solves problem q % nprob)."""
        return IpmQueue(self, nq, self.nprob if n_slots is None else n_slots)

    def ric_sv(self, *, compute_pi=1, compute_Pb=0, p0=0, count=None):
        """Batched d_back_ric_rec_sv_tv_res (nb = ng = 0, no update rows): factor into ws."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ric_sv_batch(
            self.plan, C.byref(self.layout), self.nprob, p0, count, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            self.ux.data_ptr(), self.pi.data_ptr(), self.ws.data_ptr(), compute_pi, compute_Pb,
            self.Pb.data_ptr(), self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ric_sv_batch failed ({rc})")

    def ric_sv_bound(self, stream=None, *, compute_pi=1, compute_Pb=0):
        """ric_sv over the whole batch as a zero-argument callable with every argument marshalled once (a stream
        handle, or the current stream at bind time): a launch loop then costs one foreign call per launch.  The
        callable returns the library's code (0 on success)."""
        fn = lib().hpmpc_mi355x_ric_sv_batch
        st = C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream if stream is None else stream.cuda_stream)
        args = (self.plan, C.byref(self.layout), self.nprob, 0, self.nprob, C.c_void_p(self.BAbt.data_ptr()),
                C.c_void_p(self.RSQrq.data_ptr()), C.c_void_p(self.ux.data_ptr()), C.c_void_p(self.pi.data_ptr()),
                C.c_void_p(self.ws.data_ptr()), compute_pi, compute_Pb, C.c_void_p(self.Pb.data_ptr()), st)
        return lambda: fn(*args)

    def ric_trf(self, *, p0=0, count=None):
        """Batched d_back_ric_rec_trf_tv_res (nb = ng = 0): factor into ws."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ric_trf_batch(self.plan, C.byref(self.layout), self.nprob, p0, count,
                                              self.BAbt.data_ptr(), self.RSQrq.data_ptr(), self.ws.data_ptr(),
                                              self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ric_trf_batch failed ({rc})")

    def ric_trs(self, b, q, *, compute_pi=1, compute_Pb=1, p0=0, count=None):
        """Batched d_back_ric_rec_trs_tv_res with the factor left in ws by ric_sv."""
        count = self.nprob - p0 if count is None else count
        rc = lib().hpmpc_mi355x_ric_trs_batch(
            self.plan, C.byref(self.layout), self.nprob, p0, count, self.BAbt.data_ptr(), self.RSQrq.data_ptr(),
            b.data_ptr(), q.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.ws.data_ptr(), compute_pi,
            compute_Pb, self.Pb.data_ptr(), self._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ric_trs_batch failed ({rc})")


def algorithmic_bytes_per_ip_iter(qp: OCPQP) -> float:
    """Algorithmic HBM bytes of one residual-based IP iteration of one problem:
    sv = BAbt + lower(RSQrq)+row read, L lower+row+inv_diag written, ux/pi written;
    trs = L + BAbt re-read, rhs (q, b) in, (ux, pi) out; res = lower(RSQrq) + BAbt re-read, ux/pi in,
    r_q/r_b out; IPM box vectors 24 doubles per box."""
    tot = 0
    N = qp.N
    for k in range(N + 1):
        nux = qp.nux(k)
        nx1 = int(qp.nx[k + 1]) if k < N else 0
        T = nux * (nux + 1) // 2
        babt = (nux + 1) * nx1
        rsq = T + nux
        L = T + 2 * nux
        sv = babt + rsq + L + nux + nx1
        trs = L + babt + (nux + nx1) + (nux + nx1)
        res = rsq + babt + (nux + nx1) + (nux + nx1)
        tot += sv + trs + res + 24 * int(qp.nb[k])
    return 8.0 * tot


def algorithmic_bytes_per_fact(qp: OCPQP) -> float:
    """Algorithmic HBM bytes of one problem through the IPM factorisation pass (hk_ipm_fact, phase 2,
    residuals fused): BAbt (with its b row) and lower(RSQrq)+q row read, the iterate ux / pi read and
    the residuals r_q / r_b written, box vectors lam, t, r_m, r_d read and t_inv written (10 doubles
    per box), factor L lower + row + inv_diag and P b written."""
    tot = 0
    N = qp.N
    for k in range(N + 1):
        nux = qp.nux(k)
        nx1 = int(qp.nx[k + 1]) if k < N else 0
        T = nux * (nux + 1) // 2
        tot += (nux + 1) * nx1 + (T + nux) + 2 * (nux + nx1) + 10 * int(qp.nb[k]) + (T + 2 * nux) + nx1
    return 8.0 * tot


def algorithmic_bytes_per_pass(qp: OCPQP) -> dict:
    """Algorithmic HBM bytes of one problem-iteration through each IPM pass kernel (phase 2), each datum
    counted once per pass, T = nux(nux+1)/2, per box pair (lower + upper):
    - hk_ipm_fact: algorithmic_bytes_per_fact;
    - hk_ipm_pred: factor L (T + 2 nux), BAbt with r_b in place of its b row; boxes r_d, lam, t read and
      dt, dlam written (10); the step itself is not stored;
    - hk_ipm_corr (trs + forward): L, BAbt + r_b, r_q (nux), stored P b (nx'), ux (nux) and pi (nx')
      written; boxes t, dt, dlam, lam, r_d read, r_m, dt, dlam written (16);
    - hk_ipm_update (queue API: no backups, no r_m store -- nothing in a queue solve reads them): ux, dux
      read, ux written (3 nux), the same for pi (3 nx'); boxes lam, t, dlam, dt, d read, lam, t, r_d
      written (16);
    - hk_ipm_predcorr (the queue's launch of both): hk_ipm_pred + hk_ipm_corr."""
    out = {"hk_ipm_fact": algorithmic_bytes_per_fact(qp), "hk_ipm_pred": 0.0, "hk_ipm_corr": 0.0,
           "hk_ipm_update": 0.0, "hk_ipm_predcorr": 0.0}
    N = qp.N
    for k in range(N + 1):
        nux = qp.nux(k)
        nx1 = int(qp.nx[k + 1]) if k < N else 0
        nb = int(qp.nb[k])
        T = nux * (nux + 1) // 2
        L = T + 2 * nux
        babt = (nux + 1) * nx1
        out["hk_ipm_pred"] += 8.0 * (L + babt + 10 * nb)
        out["hk_ipm_corr"] += 8.0 * (L + babt + nux + nx1 + nux + nx1 + 16 * nb)
        out["hk_ipm_update"] += 8.0 * (3 * nux + 3 * nx1 + 16 * nb)
    out["hk_ipm_predcorr"] = out["hk_ipm_pred"] + out["hk_ipm_corr"]  # the queue's fused launch: both passes' data
    return out


def algorithmic_bytes_per_sv(qp: OCPQP) -> float:
    """8 N [(nux+1)nx' + (T+nux) + (T+2nux) + nux + nx'] (sum over stages)."""
    tot = 0
    N = qp.N
    for k in range(N + 1):
        nux = qp.nux(k)
        nx1 = int(qp.nx[k + 1]) if k < N else 0
        T = nux * (nux + 1) // 2
        tot += (nux + 1) * nx1 + (T + nux) + (T + 2 * nux) + nux + nx1
    return 8.0 * tot


def flops_sv(N, nx, nu):
    """Reference flop count of one sv (test_problems/test_d_ric_mpc.c:578-590), compute_pi included."""
    return ((1 / 3) * nx ** 3 + 1.5 * nx ** 2) + N * ((7 / 3) * nx ** 3 + 4 * nx ** 2 * nu + 2 * nx * nu ** 2 +
                                                    (1 / 3) * nu ** 3 + 6.5 * nx ** 2 + 9 * nx * nu + 2.5 * nu ** 2) \
        - (nx * (nx + nu) + (1 / 3) * nx ** 3 + 1.5 * nx ** 2) + N * 2 * nx ** 2


def flops_ip_iter(N, nx, nu):
    trs = N * (6 * nx ** 2 + 8 * nx * nu + 2 * nu ** 2) + N * 2 * nx ** 2
    res = N * (2 * (nx + nu) ** 2 + 4 * (nx + nu) * nx)
    return flops_sv(N, nx, nu) + trs + res


QUEUE_LANES_MAX = 4  # include/hpmpc_mi355x.h HPMPC_MI355X_QUEUE_LANES_MAX


class IpmQueue:
    """Problem queue over a BatchSolver's data (hpmpc_mi355x_ipm_queue): ``nq`` entries solved by
    ``n_slots`` resident slots; a slot whose problem has finished takes the next entry at the next
    iteration.  Iterates and outputs are per entry, workspaces per slot.  From 2048 slots up the queue runs as
    lanes on their own streams (one per 1024 slots, at most 4; HPMPC_MI355X_QUEUE_LANES) that hand out entries
    from one shared counter, joined back into the caller's stream at the end."""

    def __init__(self, solver: BatchSolver, nq: int, n_slots: int):
        torch = solver.torch
        self.s = solver
        self.nq, self.n_slots = int(nq), int(n_slots)
        N, f64, dev = solver.N, torch.float64, solver.dev
        self.ux = torch.zeros((nq, N + 1, 16), dtype=f64, device=dev)
        self.pi = torch.zeros((nq, N + 1, 16), dtype=f64, device=dev)
        self.lam = torch.zeros((nq, N + 1, 32), dtype=f64, device=dev)
        self.t = torch.zeros((nq, N + 1, 32), dtype=f64, device=dev)
        self.kk = torch.zeros(nq, dtype=torch.int32, device=dev)
        self.ret = torch.zeros(nq, dtype=torch.int32, device=dev)
        self.stat = torch.zeros((nq, 5 * solver.k_max), dtype=f64, device=dev)
        self.ws = torch.zeros((n_slots, solver.wsd), dtype=f64, device=dev)
        # HPMPC_MI355X_QUEUE_CTL_INTS (include/hpmpc_mi355x.h): up to QUEUE_LANES_MAX lane blocks + drain counters
        self.qctl = torch.zeros(6 * QUEUE_LANES_MAX + 2 + 3 * n_slots, dtype=torch.int32, device=dev)

    def lanes(self):
        """The lane split of hpmpc_mi355x_ipm_queue (the C driver's rule): [(control-block offset in qctl, slots)]
        per lane; HPMPC_MI355X_QUEUE_LANES lanes (default 4), at most one per 1024 slots.  The lanes hand out entries
        from one shared counter."""
        L = int(os.environ.get("HPMPC_MI355X_QUEUE_LANES", "4"))
        L = max(1, min(L, self.n_slots // 1024, QUEUE_LANES_MAX, self.nq, self.n_slots))
        out, s0 = [], 0
        for i in range(L):
            ns = self.n_slots // L + (i < self.n_slots % L)
            out.append((6 * i + 3 * s0, ns))
            s0 += ns
        return out

    def finished(self):
        """Entries finished in the last run, over every lane (read after a synchronise)."""
        return sum(int(self.qctl[o + 1].item()) for o, _ in self.lanes())

    def idle(self):
        """Whether every slot of every lane was left without an entry (read after a synchronise)."""
        return all(bool((self.qctl[o + 2:o + 2 + ns] == -1).all()) for o, ns in self.lanes())

    def drained(self):
        """(iterations, problems) the multi-wave drain finished in the last run (read after a synchronise)."""
        o = 6 * QUEUE_LANES_MAX + 3 * self.n_slots
        return int(self.qctl[o].item()), int(self.qctl[o + 1].item())

    # what pass_ms[i] of run(profiled=True) times (include/hpmpc_mi355x.h): a tick is hk_ipm_fact, hk_ipm_predcorr
    # (predictor and corrector back to back) and hk_ipm_update; [3] stays 0
    PASS_KERNELS = ("hk_ipm_init + hk_ipm_qdrain_mw", "hk_ipm_fact", "hk_ipm_predcorr", None, "hk_ipm_update")

    def run(self, *, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, warm_start=0, compute_mult=1, profiled=False):
        """Solve every entry.  Returns (pass_ms[5] or None, ticks): see PASS_KERNELS.  Polls the device once per
        chunk; the caller synchronises before reading results."""
        s = self.s
        out = np.zeros(5)
        ticks = C.c_int(0)
        rc = lib().hpmpc_mi355x_ipm_queue(
            s.plan, C.byref(s.layout), s.nprob, self.nq, self.n_slots, s.BAbt.data_ptr(), s.RSQrq.data_ptr(),
            s.d.data_ptr(), self.ux.data_ptr(), self.pi.data_ptr(), self.lam.data_ptr(), self.t.data_ptr(),
            self.ws.data_ptr(), self.qctl.data_ptr(), s.k_max, mu0, mu_tol, alpha_min, warm_start, compute_mult,
            self.kk.data_ptr(), self.ret.data_ptr(), self.stat.data_ptr(), out.ctypes.data if profiled else None,
            C.byref(ticks), s._stream())
        if rc != 0:
            raise RuntimeError(f"hpmpc_mi355x_ipm_queue failed ({rc})")
        return (out if profiled else None), ticks.value
