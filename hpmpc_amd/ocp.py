"""Host-side description of the box-constrained linear MPC QP that HPMPC's hot path solves.

The data layout is HPMPC's own (so the same buffers can be handed to the reference, the oracle and
the MI355X C-ABI unchanged):

* every stage matrix is a lib4 panel-major array (bs = D_MR = 4 rows per panel, panel stride
  ``sd`` = column count padded to D_NCL = 2; element (i, j) at ``(i//4)*4*sd + i%4 + 4*j``,
  ``include/block_size.h:62-72``, ``auxiliary/d_aux_lib4.c:1310``);
* ``BAbt[k]`` is ``(nu_k+nx_k+1) x nx_{k+1}`` = ``[B'; A'; b']`` (augmented last row);
* ``RSQrq[k]`` is ``(nu_k+nx_k+1) x (nu_k+nx_k)`` = ``[[R S]; [S' Q]; [r' q']]`` (lower part used);
* ``d[k]`` is the padded ``[lb | ub | lg | ug]`` bound vector (``pnb``/``png`` strides);
* ``nx[0] = 0`` (x0 folded into ``b0 = A x0 + b``) and ``nu[N] = 0``.

The mass-spring generator restates ``test_problems/test_d_ric_mpc.c:61-142`` and the problem set-up
of ``test_problems/test_d_ip_hard.c:288-521`` (Ts = 0.5, b = 0.1, Q = I, R = 2I, S = 0, q = 0.1,
r = 0.2, u in [-0.5, 0.5], first nx/2 states in [-4, 4]).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

BS = 4   # D_MR   (include/block_size.h, TARGET_C99_4X4)
NCL = 2  # D_NCL


def rup(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def lib4_size(m: int, n: int) -> int:
    """Doubles in an m x n lib4 matrix (rows padded to 4, cols padded to 2)."""
    return rup(m, BS) * rup(n, NCL)


def pack_lib4(A: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
    """Dense (m, n) -> flat lib4 buffer (d_cvt_mat2pmat, auxiliary/d_aux_lib4.c:1310)."""
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    sd = rup(n, NCL)
    pm = rup(m, BS)
    buf = np.zeros((pm // BS, sd, BS)) if out is None else out.reshape(pm // BS, sd, BS)
    Ap = np.zeros((pm, sd))
    Ap[:m, :n] = A
    buf[...] = Ap.reshape(pm // BS, BS, sd).transpose(0, 2, 1)
    return buf.reshape(-1)


def unpack_lib4(buf: np.ndarray, m: int, n: int) -> np.ndarray:
    """Flat lib4 buffer -> dense (m, n) (d_cvt_pmat2mat, auxiliary/d_aux_lib4.c:1686)."""
    sd = rup(n, NCL)
    pm = rup(m, BS)
    b = np.asarray(buf)[..., : pm * sd]
    lead = b.shape[:-1]
    P = b.reshape(*lead, pm // BS, sd, BS)
    P = np.swapaxes(P, -1, -2).reshape(*lead, pm, sd)
    return P[..., :m, :n]


@dataclass
class OCPQP:
    """One (or a batch of) box-constrained OCP QP(s) on lib4 data.

    Batched arrays carry a leading problem axis: ``BAbt[k].shape == (B, size_k)``.  All problems of a
    batch share the stage sizes and ``idxb`` (the batched solver's contract).
    """

    N: int
    nx: np.ndarray
    nu: np.ndarray
    nb: np.ndarray
    ng: np.ndarray
    idxb: list
    BAbt: list
    RSQrq: list
    d: list
    DCt: list = field(default_factory=list)
    batch: int | None = None

    # --- sizes ------------------------------------------------------------------------------------
    def nux(self, k: int) -> int:
        return int(self.nu[k] + self.nx[k])

    def pnb(self, k: int) -> int:
        return rup(int(self.nb[k]), BS)

    def png(self, k: int) -> int:
        return rup(int(self.ng[k]), BS)

    def nconstr(self, k: int) -> int:
        return 2 * self.pnb(k) + 2 * self.png(k)

    def problem(self, p: int) -> "OCPQP":
        """Extract problem p of a batch as a single (unbatched) problem (copies)."""
        assert self.batch is not None
        return OCPQP(self.N, self.nx.copy(), self.nu.copy(), self.nb.copy(), self.ng.copy(),
                     [i.copy() for i in self.idxb], [a[p].copy() for a in self.BAbt],
                     [a[p].copy() for a in self.RSQrq], [a[p].copy() for a in self.d],
                     [a[p].copy() for a in self.DCt] if self.DCt else [], None)

    def copy(self) -> "OCPQP":
        return OCPQP(self.N, self.nx.copy(), self.nu.copy(), self.nb.copy(), self.ng.copy(),
                     [i.copy() for i in self.idxb], [a.copy() for a in self.BAbt],
                     [a.copy() for a in self.RSQrq], [a.copy() for a in self.d],
                     [a.copy() for a in self.DCt], self.batch)

    # --- solution buffers (padded like the reference drivers) ---------------------------------------
    def alloc_solution(self):
        N = self.N
        lead = () if self.batch is None else (self.batch,)
        ux = [np.zeros(lead + (rup(self.nux(k) + 1, BS),)) for k in range(N + 1)]
        pi = [np.zeros(lead + (rup(int(self.nx[k + 1]), BS),)) for k in range(N)]
        lam = [np.zeros(lead + (max(self.nconstr(k), 1),)) for k in range(N + 1)]
        t = [np.zeros(lead + (max(self.nconstr(k), 1),)) for k in range(N + 1)]
        return ux, pi, lam, t


def mass_spring_dynamics(nx: int, nu: int, Ts: float = 0.5):
    """A, B of the sampled mass-spring chain (test_d_ric_mpc.c:61-142)."""
    from scipy.linalg import expm

    pp = nx // 2
    T = -2.0 * np.eye(pp) + np.eye(pp, k=1) + np.eye(pp, k=-1)
    Ac = np.zeros((nx, nx))
    Ac[:pp, pp:] = np.eye(pp)
    Ac[pp:, :pp] = T
    Bc = np.zeros((nx, nu))
    Bc[pp:pp + nu, :] = np.eye(nu)
    A = expm(Ts * Ac)
    B = np.linalg.solve(Ac, (A - np.eye(nx)) @ Bc)
    return A, B


def default_x0(nx: int) -> np.ndarray:
    x0 = np.zeros(nx)
    x0[:2] = 2.5
    return x0


def batch_x0(nx: int, batch: int, seed_base: int = 20261015, start: int = 0) -> np.ndarray:
    """Initial states of global problems start .. start+batch-1: problem 0 uses the driver's x0, problem
    p>0 ~ U(-2.5, 2.5) from PCG64(seed_base + p)."""
    X = np.empty((batch, nx))
    for i, p in enumerate(range(start, start + batch)):
        X[i] = default_x0(nx) if p == 0 else \
            np.random.Generator(np.random.PCG64(seed_base + p)).uniform(-2.5, 2.5, nx)
    return X


def pack_lib4_batch(M: np.ndarray) -> np.ndarray:
    """(..., m, n) dense -> (..., lib4_size(m, n)) lib4 buffers (vectorised pack_lib4)."""
    m, n = M.shape[-2:]
    sd, pm = rup(n, NCL), rup(m, BS)
    lead = M.shape[:-2]
    P = np.zeros(lead + (pm, sd))
    P[..., :m, :n] = M
    P = P.reshape(lead + (pm // BS, BS, sd))
    return np.ascontiguousarray(np.swapaxes(P, -1, -2)).reshape(lead + (pm * sd,))


def _perturbations(N: int, nx: int, nu: int, problem_ids, seed: int):
    """Per-problem stage perturbations drawn from a stream of the problem's own: PCG64([seed, p]) for global
    problem p.  Returns dA (B, N, nx, nx), dB (B, N, nx, nu) and G (B, N, nx, nx) (G[:, k-1] perturbs Q_k,
    k = 1..N), all already scaled by 1e-3.  A problem's data are then a function of (seed, p) alone, so a
    shard of the global batch is bitwise the same block whatever the world size."""
    ids = np.asarray(problem_ids, dtype=np.int64)
    dA = np.empty((ids.size, N, nx, nx))
    dB = np.empty((ids.size, N, nx, nu))
    G = np.empty((ids.size, N, nx, nx))
    for i, p in enumerate(ids):
        rng = np.random.Generator(np.random.PCG64([int(seed), int(p)]))
        dA[i] = rng.standard_normal((N, nx, nx))
        dB[i] = rng.standard_normal((N, nx, nu))
        G[i] = rng.standard_normal((N, nx, nx))
    return 1e-3 * dA, 1e-3 * dB, 1e-3 * G


def mass_spring_qp(N: int, nx: int, nu: int, *, boxes: bool = True, x0=None, batch: int | None = None,
                   time_variant: bool = False, seed: int = 0, problem_ids=None) -> OCPQP:
    """The reference drivers' mass-spring MPC QP (nx[0] = 0, nu[N] = 0).

    ``batch`` stacks ``batch`` problems that differ in x0 (problem 0 = the drivers' x0) and, with
    ``time_variant``, in a seeded perturbation of every stage's A, B (1e-3 N(0,1)) and Q (+ G G',
    G ~ 1e-3 N(0,1)) so that no two stage buffers alias (SURVEY.md §8d roofline accounting).

    With ``problem_ids`` (the global indices of the batch's problems) each problem's perturbations come from
    its own stream ``PCG64([seed, p])`` (`_perturbations`), so the data of global problem p do not depend on
    which batch or rank it is generated in.  Without it the perturbations come from one stream over the whole
    batch (``PCG64(seed)``, the layout the committed goldens were generated with).
    """
    A, B = mass_spring_dynamics(nx, nu)
    b = np.full(nx, 0.1)
    Q = np.eye(nx)
    R = 2.0 * np.eye(nu)
    q = np.full(nx, 0.1)
    r = np.full(nu, 0.2)
    Bn = 1 if batch is None else batch
    if x0 is None:
        X0 = batch_x0(nx, Bn) if batch is not None else default_x0(nx)[None]
    else:
        X0 = np.atleast_2d(np.asarray(x0, dtype=np.float64))
        assert X0.shape == (Bn, nx)
    rng = np.random.Generator(np.random.PCG64(seed))
    per_problem = None
    if time_variant and problem_ids is not None:
        assert len(problem_ids) == Bn, (len(problem_ids), Bn)
        per_problem = _perturbations(N, nx, nu, problem_ids, seed)

    nxv = np.array([0] + [nx] * N, dtype=np.int32)
    nuv = np.array([nu] * N + [0], dtype=np.int32)
    if boxes:
        nbv = np.array([nu] + [nu + nx // 2] * (N - 1) + [nx // 2], dtype=np.int32)
    else:
        nbv = np.zeros(N + 1, dtype=np.int32)
    ngv = np.zeros(N + 1, dtype=np.int32)

    BAbt, RSQrq, dv, idxb = [], [], [], []
    for k in range(N + 1):
        nuk, nxk = int(nuv[k]), int(nxv[k])
        nux = nuk + nxk
        if k < N:
            nx1 = int(nxv[k + 1])
            Ak = np.broadcast_to(A, (Bn, nx, nx))
            Bk = np.broadcast_to(B, (Bn, nx, nu))
            if per_problem is not None:
                Ak = A + per_problem[0][:, k]
                Bk = B + per_problem[1][:, k]
            elif time_variant:
                Ak = A + 1e-3 * rng.standard_normal((Bn, nx, nx))
                Bk = B + 1e-3 * rng.standard_normal((Bn, nx, nu))
            M = np.zeros((Bn, nux + 1, nx1))
            M[:, :nuk, :] = np.swapaxes(Bk, 1, 2)
            if k == 0:
                M[:, nuk, :] = np.einsum("pij,pj->pi", Ak, X0) + b  # b0 = A x0 + b (test_d_ip_hard.c:306-322)
            else:
                M[:, nuk:nux, :] = np.swapaxes(Ak, 1, 2)
                M[:, nux, :] = b
            BAbt.append(pack_lib4_batch(M))
        M = np.zeros((Bn, nux + 1, nux))
        M[:, :nuk, :nuk] = R[:nuk, :nuk]
        Qk = np.broadcast_to(Q[:nxk, :nxk], (Bn, nxk, nxk))
        if per_problem is not None and nxk > 0:
            G = per_problem[2][:, k - 1]
            Qk = Q[:nxk, :nxk] + G @ np.swapaxes(G, 1, 2)
        elif time_variant and nxk > 0:
            G = 1e-3 * rng.standard_normal((Bn, nxk, nxk))
            Qk = Q[:nxk, :nxk] + G @ np.swapaxes(G, 1, 2)
        M[:, nuk:nux, nuk:nux] = Qk
        M[:, nux, :nuk] = r[:nuk]
        M[:, nux, nuk:nux] = q[:nxk]
        RSQrq.append(pack_lib4_batch(M))
        # boxes: u in [-0.5, 0.5]; first nx/2 states in [-4, 4]  (test_d_ip_hard.c:359-405)
        nbk = int(nbv[k])
        pnb = rup(nbk, BS)
        dk = np.zeros(max(2 * pnb, 1))
        for j in range(nbk):
            if j < nuk:
                dk[j], dk[pnb + j] = -0.5, 0.5
            else:
                dk[j], dk[pnb + j] = -4.0, 4.0
        idxb.append(np.arange(nbk, dtype=np.int32))
        dv.append(np.broadcast_to(dk, (Bn, dk.size)).copy())

    qp = OCPQP(N, nxv, nuv, nbv, ngv, idxb, BAbt, RSQrq, dv, [], batch)
    if batch is None:
        qp.BAbt = [a[0].copy() for a in qp.BAbt]
        qp.RSQrq = [a[0].copy() for a in qp.RSQrq]
        qp.d = [a[0].copy() for a in qp.d]
    return qp
