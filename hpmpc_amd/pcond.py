"""Device-resident batches of the partial-condensing pipeline (BASELINE configs[4]).

``d_part_cond`` (lqcp_solvers/d_part_cond.c:926) condenses each problem's N stages into N2 blocks, the
Riccati recursion ``d_back_ric_rec_sv_tv_res`` (lqcp_solvers/d_back_ric_rec.c:112) runs on the condensed
(wide) stages, and ``d_part_expand_solution`` (d_part_cond.c:1103) recovers the full-space solution.  All
three are HIP kernels of libhpmpc_mi355x.so (hk_wide.hip); torch only allocates the HBM arrays:

    BAbt, RSQrq, d          (nprob, size)  original lib4 stage blocks / padded bounds at the plan's offsets
    G                       (nprob, size)  Gamma scratch of the condensing
    BAbt2, RSQrq2, DCt2, d2 (nprob, size)  condensed problem
    ws2, ux2, pi2           (nprob, size)  condensed factor and solution
    ux, pi, lam, t          (nprob, size)  expanded solution

There is no CPU fallback: constructing a solver without a GPU raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .batch import lib
from .ocp import OCPQP

_BOUND = False


def _bind():
    global _BOUND
    L = lib()
    if _BOUND:
        return L
    vp, i, ll = C.c_void_p, C.c_int, C.c_longlong
    L.hpmpc_mi355x_pcond_plan_create.restype = vp
    L.hpmpc_mi355x_pcond_plan_create.argtypes = [i, vp, vp, vp, vp, vp, i]
    L.hpmpc_mi355x_pcond_plan_destroy.argtypes = [vp]
    L.hpmpc_mi355x_pcond_sizes.argtypes = [vp, vp]
    L.hpmpc_mi355x_pcond_offsets.argtypes = [vp, i, vp]
    L.hpmpc_mi355x_pcond_batch.restype = i
    L.hpmpc_mi355x_pcond_batch.argtypes = [vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hpmpc_mi355x_pcond_ric_sv_batch.restype = i
    L.hpmpc_mi355x_pcond_ric_sv_batch.argtypes = [vp, i, i, i, vp, vp, vp, vp, vp, i, vp]
    L.hpmpc_mi355x_pexpand_batch.restype = i
    L.hpmpc_mi355x_pexpand_batch.argtypes = [vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hpmpc_mi355x_pcond_wide_plan.restype = vp
    L.hpmpc_mi355x_pcond_wide_plan.argtypes = [vp]
    L.hpmpc_mi355x_wide_sizes.argtypes = [vp, vp]
    L.hpmpc_mi355x_wide_offsets.argtypes = [vp, vp]
    L.hpmpc_mi355x_wide_ipm_batch.restype = i
    d = C.c_double
    L.hpmpc_mi355x_wide_ipm_batch.argtypes = [vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, i, d, d, d, i, i, vp,
                                              vp, vp, vp]
    _ = ll
    _BOUND = True
    return L


class PcondSolver:
    """A batch of OCP QPs (shared sizes), condensed into N2 blocks and solved by the condensed Riccati."""

    def __init__(self, qp: OCPQP, N2: int, device="cuda"):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("PcondSolver needs a GPU (HIP device); there is no CPU fallback")
        assert qp.batch is not None, "PcondSolver takes a batched OCPQP"
        self.torch = torch
        self.qp = qp
        self.N, self.N2, self.nprob = qp.N, N2, qp.batch
        self.dev = torch.device(device)
        L = _bind()
        N = qp.N
        idx = [np.ascontiguousarray(i, dtype=np.int32) for i in qp.idxb]
        idxp = (C.POINTER(C.c_int) * (N + 1))(*[a.ctypes.data_as(C.POINTER(C.c_int)) for a in idx])
        ints = lambda a: np.ascontiguousarray(a, dtype=np.int32)
        self._keep = [idx, idxp]
        nx, nu, nb, ng = ints(qp.nx), ints(qp.nu), ints(qp.nb), ints(qp.ng)
        self.plan = L.hpmpc_mi355x_pcond_plan_create(N, nx.ctypes.data, nu.ctypes.data, nb.ctypes.data,
                                                     C.cast(idxp, C.c_void_p), ng.ctypes.data, N2)
        if not self.plan:
            raise ValueError(f"unsupported partial condensing (code {L.hpmpc_mi355x_last_error()})")
        sz = (C.c_longlong * 15)()
        L.hpmpc_mi355x_pcond_sizes(self.plan, sz)
        self.sizes = [int(v) for v in sz]
        o0 = (C.c_longlong * (6 * (N + 1)))()
        o1 = (C.c_longlong * (6 * (N2 + 1)))()
        L.hpmpc_mi355x_pcond_offsets(self.plan, 0, o0)
        L.hpmpc_mi355x_pcond_offsets(self.plan, 1, o1)
        self.off = np.array(o0[:], dtype=np.int64).reshape(N + 1, 6)
        self.off2 = np.array(o1[:], dtype=np.int64).reshape(N2 + 1, 6)
        P = self.nprob
        s = self.sizes
        hB = np.zeros((P, s[0]))
        hR = np.zeros((P, s[1]))
        hd = np.zeros((P, s[2]))
        for k in range(N + 1):
            if k < N:
                n = qp.BAbt[k].shape[1]
                hB[:, self.off[k, 0]:self.off[k, 0] + n] = qp.BAbt[k]
            n = qp.RSQrq[k].shape[1]
            hR[:, self.off[k, 1]:self.off[k, 1] + n] = qp.RSQrq[k]
            if qp.nb[k] + qp.ng[k] > 0:
                n = qp.d[k].shape[1]
                hd[:, self.off[k, 2]:self.off[k, 2] + n] = qp.d[k]
        f64 = torch.float64
        z = lambda n: torch.zeros((P, max(n, 1)), dtype=f64, device=self.dev)
        self.BAbt = torch.from_numpy(hB).to(self.dev)
        self.RSQrq = torch.from_numpy(hR).to(self.dev)
        self.d = torch.from_numpy(hd).to(self.dev)
        self.G = z(s[12])
        self.BAbt2, self.RSQrq2, self.DCt2, self.d2 = z(s[5]), z(s[6]), z(s[7]), z(s[8])
        self.ux2, self.pi2, self.ws2 = z(s[9]), z(s[10]), z(s[11])
        self.lam2, self.t2 = z(s[8]), z(s[8])
        self.ux, self.pi, self.lam, self.t = z(s[3]), z(s[4]), z(s[2]), z(s[2])

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                _bind().hpmpc_mi355x_pcond_plan_destroy(self.plan)
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed (code {rc})")

    def condense(self, p0=0, count=None):
        count = self.nprob - p0 if count is None else count
        p = self._p
        self._check(_bind().hpmpc_mi355x_pcond_batch(self.plan, self.nprob, p0, count, p(self.BAbt), p(self.RSQrq),
                                                     p(self.d), p(self.G), p(self.BAbt2), p(self.RSQrq2),
                                                     p(self.DCt2), p(self.d2), self._stream()), "pcond")

    def riccati(self, p0=0, count=None, compute_pi=1):
        count = self.nprob - p0 if count is None else count
        p = self._p
        self._check(_bind().hpmpc_mi355x_pcond_ric_sv_batch(self.plan, self.nprob, p0, count, p(self.BAbt2),
                                                            p(self.RSQrq2), p(self.ws2), p(self.ux2), p(self.pi2),
                                                            compute_pi, self._stream()), "condensed sv")

    def expand(self, p0=0, count=None):
        count = self.nprob - p0 if count is None else count
        p = self._p
        self._check(_bind().hpmpc_mi355x_pexpand_batch(self.plan, self.nprob, p0, count, p(self.BAbt), p(self.RSQrq),
                                                       p(self.ux2), p(self.pi2), p(self.lam2), p(self.t2), p(self.ux),
                                                       p(self.pi), p(self.lam), p(self.t), self._stream()), "expand")

    def solve(self):
        """condense -> condensed Riccati -> expand for the whole batch (asynchronous on the current stream)."""
        self.condense()
        self.riccati()
        self.expand()

    def ipm(self, k_max=50, mu0=2.0, mu_tol=1e-12, alpha_min=1e-8, p0=0, count=None):
        """d_ip2_res_mpc_hard_tv on the condensed problems (hpmpc_mi355x_wide_ipm_batch, the wide-stage IPM: one
        workgroup per problem, one launch): ux2 / pi2 / lam2 / t2, and kk2 / ret2 / stat2 per problem."""
        L = _bind()
        torch = self.torch
        if not getattr(self, "wplan", None):
            self.wplan = L.hpmpc_mi355x_pcond_wide_plan(self.plan)
            if not self.wplan:
                raise ValueError(f"no wide IPM plan for the condensed problem (code {L.hpmpc_mi355x_last_error()})")
            ws = (C.c_longlong * 8)()
            L.hpmpc_mi355x_wide_sizes(self.wplan, ws)
            self.wsizes = [int(v) for v in ws]
            # the wide IPM indexes the condensed arrays with its own layout: it must be the condensing carve's
            # (the library also checks every stage offset when it creates the plan)
            s = self.sizes
            assert self.wsizes[:6] == [s[5], s[6], s[7], s[8], s[9], s[10]], (self.wsizes, self.sizes)
            wo = (C.c_longlong * (6 * (self.N2 + 1)))()
            L.hpmpc_mi355x_wide_offsets(self.wplan, wo)
            wo = np.array(wo[:], dtype=np.int64).reshape(self.N2 + 1, 6)  # oB oR oG oD oU oP
            assert np.array_equal(wo[:, [0, 1, 3, 4, 5]], self.off2[:, [0, 1, 2, 3, 4]]), (wo, self.off2)
        P = self.nprob
        if getattr(self, "_kmax", None) != k_max:
            self.work2 = torch.zeros((P, self.wsizes[6]), dtype=torch.float64, device=self.dev)
            self.kk2 = torch.zeros(P, dtype=torch.int32, device=self.dev)
            self.ret2 = torch.zeros(P, dtype=torch.int32, device=self.dev)
            self.stat2 = torch.zeros((P, 5 * max(k_max, 1)), dtype=torch.float64, device=self.dev)
            self._kmax = k_max
        count = self.nprob - p0 if count is None else count
        p = self._p
        self._check(L.hpmpc_mi355x_wide_ipm_batch(self.wplan, P, p0, count, p(self.BAbt2), p(self.RSQrq2),
                                                  p(self.DCt2), p(self.d2), p(self.ux2), p(self.pi2), p(self.lam2),
                                                  p(self.t2), p(self.work2), k_max, mu0, mu_tol, alpha_min, 0, 1,
                                                  p(self.kk2), p(self.ret2), p(self.stat2), self._stream()),
                    "condensed IPM")

    def cond_sizes(self):
        """Stage sizes of the condensed problem (lists of N2+1): nx, nu, nb, ng."""
        N, N2, qp = self.N, self.N2, self.qp
        nx = [int(v) for v in qp.nx]
        nu = [int(v) for v in qp.nu]
        nb = [int(v) for v in qp.nb]
        ng = [int(v) for v in qp.ng]
        blocks = _blocks(N, N2)
        c = dict(nx=[], nu=[], nb=[], ng=[])
        s = 0
        for T in blocks:  # d_part_cond_compute_problem_size (d_part_cond.c:694-741)
            c["nx"].append(nx[s])
            c["nu"].append(sum(nu[s + j] for j in range(T)))
            inner_u = sum(sum(1 for v in qp.idxb[s + j] if v < nu[s + j]) for j in range(1, T))
            inner_x = sum(sum(1 for v in qp.idxb[s + j] if v >= nu[s + j]) for j in range(1, T))
            c["nb"].append(nb[s] + inner_u)
            c["ng"].append(sum(ng[s + j] for j in range(T)) + inner_x)
            s += T
        c["nx"].append(nx[N])
        c["nu"].append(0)
        c["nb"].append(nb[N])
        c["ng"].append(ng[N])
        return c

    def solve_ipm(self, **kw):
        """condense -> IPM on the condensed problems -> expand (solution and multipliers), asynchronous."""
        self.condense()
        self.ipm(**kw)
        self.expand()

    def multipliers(self, p: int):
        """Problem p's expanded lam[k], t[k] (the padded [lb | ub | lg | ug] vectors) as numpy lists."""
        lam = self.lam[p].cpu().numpy()
        t = self.t[p].cpu().numpy()
        qp = self.qp
        n = [qp.nconstr(k) for k in range(self.N + 1)]
        return ([lam[self.off[k, 2]:self.off[k, 2] + n[k]].copy() for k in range(self.N + 1)],
                [t[self.off[k, 2]:self.off[k, 2] + n[k]].copy() for k in range(self.N + 1)])

    def solution(self, p: int):
        """Problem p's expanded ux[k] (nu+nx) and pi[k] (nx_{k+1}) as numpy lists."""
        ux = self.ux[p].cpu().numpy()
        pi = self.pi[p].cpu().numpy()
        qp = self.qp
        U = [ux[self.off[k, 3]:self.off[k, 3] + qp.nux(k)].copy() for k in range(self.N + 1)]
        Pi = [pi[self.off[k, 4]:self.off[k, 4] + int(qp.nx[k + 1])].copy() for k in range(self.N)]
        return U, Pi


# ------------------------------------------------------------------------------------------------
# Algorithmic work of the pipeline (SURVEY.md §8d accounting: each datum once per kernel pass, fp64)
# ------------------------------------------------------------------------------------------------
def _tri(n):
    return n * (n + 1) // 2


def pcond_algorithmic_bytes(qp: OCPQP, N2: int):
    """Bytes per problem of [hk_pcond, hk_wide_sv (condensed), hk_pexpand]:
    condense: BAbt and lower(RSQrq)+gradient row of every stage in, BAbt2 and lower(RSQrq2)+row out;
    condensed sv: BAbt2, lower(RSQrq2)+row in; packed L + 1/diag, ux2, pi2 out;
    expand: BAbt, lower(RSQrq)+row of the inner stages, ux2, pi2 in; ux, pi out."""
    N = qp.N
    nux = [qp.nux(k) for k in range(N + 1)]
    nx = [int(v) for v in qp.nx]
    bB = sum((nux[k] + 1) * nx[k + 1] for k in range(N))
    bR = sum(_tri(nux[k]) + nux[k] for k in range(N + 1))
    blocks = _blocks(N, N2)
    nv, nx2 = [], []
    s = 0
    for T in blocks:
        nv.append(sum(int(qp.nu[s + j]) for j in range(T)) + nx[s])
        nx2.append(nx[s + T])
        s += T
    b2B = sum((nv[i] + 1) * nx2[i] for i in range(N2))
    b2R = sum(_tri(nv[i]) + nv[i] for i in range(N2)) + _tri(nux[N]) + nux[N]
    fac = sum(_tri(nv[i]) + nv[i] + nv[i] for i in range(N2)) + _tri(nux[N]) + 2 * nux[N]
    u2 = sum(nv) + nux[N]
    p2 = sum(nx2)
    cond = 8.0 * (bB + bR + b2B + b2R)
    sv = 8.0 * (b2B + b2R + fac + u2 + p2)
    expand = 8.0 * (bB + bR + u2 + p2 + sum(nux) + sum(nx[1:]))
    return cond, sv, expand


def wide_ipm_algorithmic_bytes(nx, nu, nb, ng):
    """Bytes of ONE IP iteration of the wide-stage IPM (hk_wide_ipm) on a problem with stage sizes nx, nu, nb, ng
    (lists of N+1; the condensed problem at configs[4]), SURVEY.md §8d's rule -- each datum once per pass -- applied to
    the passes of an iteration: the factorisation (BAbt, lower RSQrq + row and DCt in; packed L + row + 1/diag out),
    the predictor and corrector solves (L, BAbt and DCt in; ux, pi out), the residuals (lower RSQrq, BAbt, DCt, ux,
    pi in; r_q, r_b out) and 24 doubles per constraint pair (the element-wise IPM vectors, as the narrow IPM's
    accounting)."""
    N = len(nx) - 1
    nux = [int(nu[k]) + int(nx[k]) for k in range(N + 1)]
    B = sum((nux[k] + 1) * int(nx[k + 1]) for k in range(N))
    R = sum(_tri(n) + n for n in nux)
    L = sum(_tri(n) + 2 * n for n in nux)
    D = sum(nux[k] * int(ng[k]) for k in range(N + 1))
    u, p = sum(nux), sum(int(nx[k + 1]) for k in range(N))
    fact = B + R + D + L
    solve = L + B + D + u + p
    res = R + B + D + 2 * (u + p)
    vec = 24 * sum(int(nb[k]) + int(ng[k]) for k in range(N + 1))
    return 8.0 * (fact + 2 * solve + res + vec)


def _blocks(N, N2):
    N1, R1 = N // N2, N - N2 * (N // N2)
    return [N1 + 1 if i < R1 else N1 for i in range(N2)]


def pcond_flops(qp: OCPQP, N2: int):
    """Flops per problem of [condense, condensed sv, expand] by the restated algorithm (d_part_cond.c,
    lqcp_solvers/d_back_ric_rec.c; sv by the reference's closed form test_d_ric_mpc.c:578-590 on the condensed
    sizes)."""
    from .batch import flops_sv

    N = qp.N
    nx = [int(v) for v in qp.nx]
    nu = [int(v) for v in qp.nu]
    cond = 0.0
    s = 0
    nv_l, nx2_l = [], []
    for T in _blocks(N, N2):
        rows = nx[s] + 1
        for j in range(T):
            rows += nu[s + j]
            if j > 0:  # Gamma_j = Gamma_{j-1} A_j
                cond += 2.0 * (rows - nu[s + j]) * nx[s + j] * nx[s + j + 1]
        rows = nx[s] + 1 + nu[s]
        for j in range(1, T):  # state cost-to-go propagation + cross terms per stage
            st = s + j
            nxs, nus, nuxp = nx[st], nu[st], nu[st - 1] + nx[st - 1]
            r_prev = nx[s] + 1 + sum(nu[s:st])
            cond += 2.0 * r_prev * nxs * nus + nxs ** 3 / 3.0 + (nuxp + 1) * nxs * nxs + (nuxp + 1) * nuxp * nxs
        nv_l.append(sum(nu[s:s + T]) + nx[s])
        nx2_l.append(nx[s + T])
        s += T
    nv = int(round(np.mean(nv_l[1:] if len(nv_l) > 1 else nv_l)))
    sv = flops_sv(N2, nx2_l[-1], nv - nx2_l[-1])
    expand = sum(2.0 * (nu[k] + nx[k]) * nx[k + 1] * 2 + 2.0 * nx[k] * (nu[k] + nx[k]) for k in range(N))
    return cond, sv, expand
