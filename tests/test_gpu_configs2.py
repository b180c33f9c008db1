"""configs[2] at its own batch (BASELINE.json): 1024 x mass-spring N=50 nx=8 nu=3, Riccati only -- the
hk_ric_sv launch bench.py times.  Oracle parity on problems spread over the batch (0, 1, 511, 1023), and
launch splitting is bitwise identical to the whole launch; the same for trf + trs with new right-hand
sides.  Tolerance: TOL_RIC (1e-12 relative to max(1, |ref|))."""
import os

import numpy as np
import pytest

from helpers import TOL_RIC

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAMPLE = (0, 1, 511, 1023)


def _oracle():
    from hpmpc_amd.cabi import HpmpcAPI, load

    return HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")


@pytest.fixture(scope="module")
def solver():
    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    qp = make_shard(50, 8, 3, 0, 1, 1024, boxes=False)
    return BatchSolver(qp, k_max=1)


def test_sv_full_batch(solver):
    import torch

    s, qp = solver, solver.qp
    s.ric_sv(compute_pi=1, compute_Pb=1)
    torch.cuda.synchronize()
    ux1, pi1, Pb1 = s.ux.clone(), s.pi.clone(), s.Pb.clone()
    s.ux.zero_()
    s.pi.zero_()
    s.Pb.zero_()
    s.ric_sv(compute_pi=1, compute_Pb=1, p0=0, count=333)
    s.ric_sv(compute_pi=1, compute_Pb=1, p0=333, count=691)
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux1) and torch.equal(s.pi, pi1) and torch.equal(s.Pb, Pb1)
    ux, pi, Pb = (x.cpu().numpy() for x in (ux1, pi1, Pb1))
    orc = _oracle()
    for p in SAMPLE:
        u2, p2, b2, _ = orc.ric_sv(qp.problem(p), compute_pi=1, compute_Pb=1)
        for k in range(51):
            n = qp.nux(k)
            np.testing.assert_allclose(ux[p, k, :n], u2[k][:n], rtol=TOL_RIC, atol=TOL_RIC)
            if k < 50:
                np.testing.assert_allclose(pi[p, k, :8], p2[k][:8], rtol=TOL_RIC, atol=TOL_RIC)
                np.testing.assert_allclose(Pb[p, k, :8], b2[k][:8], rtol=TOL_RIC, atol=TOL_RIC)


def test_trf_trs_full_batch(solver):
    import torch

    s, qp = solver, solver.qp
    rng = np.random.default_rng(7)
    b = torch.from_numpy(rng.standard_normal((1024, 51, 16))).cuda()
    q = torch.from_numpy(rng.standard_normal((1024, 51, 16))).cuda()
    s.ric_trf()
    s.ric_trs(b, q)
    torch.cuda.synchronize()
    ux1 = s.ux.clone()
    s.ux.zero_()
    s.ric_trf(p0=0, count=512)
    s.ric_trf(p0=512, count=512)
    s.ric_trs(b, q, p0=0, count=100)
    s.ric_trs(b, q, p0=100, count=924)
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux1)
    ux = ux1.cpu().numpy()
    orc = _oracle()
    for p in SAMPLE:
        one = qp.problem(p)
        mem = orc.ric_trf(one)
        u2, _, _ = orc.ric_trs(one, mem, b=[b[p, k].cpu().numpy().copy() for k in range(50)],
                               q=[q[p, k].cpu().numpy().copy() for k in range(51)])
        for k in range(51):
            n = qp.nux(k)
            np.testing.assert_allclose(ux[p, k, :n], u2[k][:n], rtol=TOL_RIC, atol=TOL_RIC)
