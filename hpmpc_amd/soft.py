"""Soft-constrained MPC problems for d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:83-547).

Data contract of the reference (test_problems/test_d_ip_soft.c:277-640):

* ``idxb[k]`` lists the nb[k] hard boxes followed by the ns[k] soft boxes;
* ``d[k]`` = [lb (pnb) | ub (pnb) | ls (pns) | us (pns)] (no general constraints);
* ``Z[k]``, ``z[k]`` = quadratic / linear slack penalties [lower (pns) | upper (pns)];
* ``lam[k]``, ``t[k]`` = [lower (pnb) | upper (pnb) | 4 soft blocks of pns]; ``nu[N] = 0``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .ocp import mass_spring_dynamics, pack_lib4_batch, rup


@dataclass
class SoftQP:
    N: int
    nx: np.ndarray
    nu: np.ndarray
    nb: np.ndarray
    ns: np.ndarray
    idxb: list
    BAbt: list
    RSQrq: list
    d: list
    Z: list
    z: list
    ng: np.ndarray = field(default=None)
    DCt: list = field(default_factory=list)

    def __post_init__(self):
        if self.ng is None:
            self.ng = np.zeros(self.N + 1, dtype=np.int32)

    def nux(self, k: int) -> int:
        return int(self.nu[k] + self.nx[k])

    def ncv(self, k: int) -> int:
        """length of lam[k] / t[k]: [lower, upper (pnb) | general lower, upper (png) | 4 soft blocks (pns)]"""
        return 2 * rup(int(self.nb[k]), 4) + 2 * rup(int(self.ng[k]), 4) + 4 * rup(int(self.ns[k]), 4)

    def copy(self) -> "SoftQP":
        cp = lambda L: [np.array(a, copy=True) for a in L]
        return SoftQP(self.N, self.nx.copy(), self.nu.copy(), self.nb.copy(), self.ns.copy(), cp(self.idxb),
                      cp(self.BAbt), cp(self.RSQrq), cp(self.d), cp(self.Z), cp(self.z), self.ng.copy(), cp(self.DCt))

    @staticmethod
    def from_case(case) -> "SoftQP":
        """SoftQP of a golden case of kind "soft" (tests/golden/make_golden.py soft)."""
        q = case.qp
        ns = np.asarray(case.inp["ns"][0], dtype=np.float64).astype(np.int32)
        return SoftQP(q.N, q.nx.copy(), q.nu.copy(), q.nb.copy(), ns, [a.copy() for a in q.idxb],
                      [a.copy() for a in q.BAbt], [a.copy() for a in q.RSQrq], [a.copy() for a in q.d],
                      [a.copy() for a in case.inp["Z"]], [a.copy() for a in case.inp["z"]], q.ng.copy(),
                      [a.copy() for a in q.DCt])

    def alloc_solution(self):
        N = self.N
        ux = [np.zeros(rup(self.nux(k) + 1, 4) + 4) for k in range(N + 1)]
        pi = [np.zeros(rup(int(self.nx[k + 1]), 4) + 4) for k in range(N)]
        lam = [np.zeros(self.ncv(k) + 4) for k in range(N + 1)]
        t = [np.zeros(self.ncv(k) + 4) for k in range(N + 1)]
        return ux, pi, lam, t


def mass_spring_soft(N: int, nx: int, nu: int, *, x0=None, Zq: float = 0.0, zl: float = 100.0, Q_diag: float = 0.0,
                     soft_bounds=(-1.0, 1.0), hard_u=(-0.5, 0.5), time_variant: bool = False, seed: int = 0,
                     hard_last: int = 0, soft: bool = True, hard: bool = True) -> SoftQP:
    """The reference's soft-constraint driver problem (test_d_ip_soft.c:160-640): mass-spring dynamics, b = 0,
    x0 = [3.5, 3.5, 0, ...], Q = Q_diag I (0 in the driver), R = 2 I, q = 0.1, r = 0.2; hard input boxes at
    stages 0..N-1 (nb = nu), soft state boxes at stages 1..N (ns = nx), Z = Zq, z = zl.
    ``soft`` / ``hard`` = False drop the soft / hard boxes.
    ``hard_last`` > 0 puts hard boxes on the first ``hard_last`` states of the terminal stage and soft ones on
    the others (a shape the driver does not use: it exercises the reference's soft-gradient index for nb > 0
    at k = N, whose write lands in Zl / zl of stage 1)."""
    A, B = mass_spring_dynamics(nx, nu)
    rng = np.random.Generator(np.random.PCG64(seed))
    if x0 is None:
        x0 = np.zeros(nx)
        x0[0] = x0[1] = 3.5
    b = np.zeros(nx)
    R = 2.0 * np.eye(nu)
    q = np.full(nx, 0.1)
    r = np.full(nu, 0.2)
    nxv = np.array([0] + [nx] * N, dtype=np.int32)
    nuv = np.array([nu] * N + [0], dtype=np.int32)
    nbv = np.array([nu if hard else 0] * N + [hard_last], dtype=np.int32)
    nsv = np.array([0] + [nx if soft else 0] * (N - 1) + [(nx - hard_last) if soft else 0], dtype=np.int32)
    BAbt, RSQrq, dv, idxb, Zv, zv = [], [], [], [], [], []
    for k in range(N + 1):
        nuk, nxk = int(nuv[k]), int(nxv[k])
        nux = nuk + nxk
        if k < N:
            Ak, Bk = A, B
            if time_variant:
                Ak = A + 1e-3 * rng.standard_normal(A.shape)
                Bk = B + 1e-3 * rng.standard_normal(B.shape)
            M = np.zeros((nux + 1, nx))
            M[:nuk, :] = Bk.T
            if k == 0:
                M[nuk, :] = Ak @ x0 + b
            else:
                M[nuk:nux, :] = Ak.T
                M[nux, :] = b
            BAbt.append(pack_lib4_batch(M[None])[0].copy())
        M = np.zeros((nux + 1, nux))
        M[:nuk, :nuk] = R[:nuk, :nuk]
        M[nuk:nux, nuk:nux] = Q_diag * np.eye(nxk)
        M[nux, :nuk] = r[:nuk]
        M[nux, nuk:nux] = q[:nxk]
        RSQrq.append(pack_lib4_batch(M[None])[0].copy())
        nbk, nsk = int(nbv[k]), int(nsv[k])
        pnb, pns = rup(nbk, 4), rup(nsk, 4)
        ib = list(range(min(nuk, nbk))) + [nuk + j for j in range(nbk - min(nuk, nbk))]
        ib += [nuk + nxk - nsk + j for j in range(nsk)]  # soft boxes on the last nsk states (no variable twice)
        idxb.append(np.array(ib, dtype=np.int32) if ib else np.zeros(1, dtype=np.int32))
        dk = np.zeros(2 * pnb + 2 * pns + 4)
        for j in range(nbk):
            lo, hi = hard_u if ib[j] < nuk else (-4.0, 4.0)
            dk[j], dk[pnb + j] = lo, hi
        for j in range(nsk):
            dk[2 * pnb + j], dk[2 * pnb + pns + j] = soft_bounds
        dv.append(dk)
        Zk = np.zeros(2 * pns + 4)
        zk = np.zeros(2 * pns + 4)
        Zk[:nsk] = Zq
        Zk[pns:pns + nsk] = Zq
        zk[:nsk] = zl
        zk[pns:pns + nsk] = zl
        Zv.append(Zk)
        zv.append(zk)
    return SoftQP(N, nxv, nuv, nbv, nsv, idxb, BAbt, RSQrq, dv, Zv, zv)
