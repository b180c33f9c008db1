"""The two-wave Riccati sv kernel (hk_ric2.hip: tile recursion on one wave, fetch / row half / stores on the other)
against the one-wave kernel (hpmpc_kernels.hip hk_ric_sv, HPMPC_MI355X_RIC_WAVES=1) and the CPU oracle.

Both kernels run the same hk_riccati.h routines on the same operands, so they agree to rounding (the compiler may
contract a few products into FMAs differently once the bodies are split over waves, hk_mw.h); each is held to the
oracle at TOL_RIC (1e-12 relative to max(1, |ref|)), on:
  * the benchmark shapes (compiled stage classes (4, 12) and (3, 8)) at their full batch sizes, launch splitting
    bitwise identical to the whole launch;
  * generic shapes (DynSh stages, full factor on stage 0 with nx[0] > 0), short horizons N = 1, 2, 3;
  * the reference's inner x-pivot clamp (xclamp_qp variants, the stages the clamp certificate rejects);
  * the aliased (time-invariant) layout.
The one-wave kernel is the product's (the two-wave one measured slower), and the two-wave kernel lives
only in the ric2 build variant (hpmpc_amd.build.build_ric2, hpmpc_amd/lib/ab/libric2.so): test_two_wave_suite runs this
module in a child process on that library (HPMPC_MI355X_LIB); the tests below run only there.  test_sv_goldens_two_wave
runs the sv goldens (update_b / update_q with box terms, the clamp goldens) through the drop-in entry point on the
two-wave kernel."""
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import TOL_RIC, random_qp, stack_qps as stack, xclamp_qp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(ROOT, "hpmpc_amd", "lib", "ab", "libric2.so")
ON_VARIANT = os.path.abspath(os.environ.get("HPMPC_MI355X_LIB", "") or ".") == VARIANT
variant_only = pytest.mark.skipif(not ON_VARIANT, reason="runs on the ric2 build variant (test_two_wave_suite)")


@pytest.mark.skipif(ON_VARIANT, reason="the child process itself")
def test_two_wave_suite():
    """This module's tests on the ric2 variant library, in a child process (the product library has no two-wave sv)."""
    assert os.path.exists(VARIANT), "build the variant: hpmpc_amd.build.build_ric2()"
    env = dict(os.environ, HPMPC_MI355X_LIB=VARIANT)
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.abspath(__file__), "-m", "gpu", "-x", "-q",
                        "-p", "no:cacheprovider"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "11 passed" in r.stdout, r.stdout[-2000:]


def _oracle():
    from hpmpc_amd.cabi import HpmpcAPI, load

    return HpmpcAPI(load(os.path.join(ROOT, "oracle", "liboracle.so")), "orc_")


def run_sv(s, waves, **kw):
    import torch

    os.environ["HPMPC_MI355X_RIC_WAVES"] = str(waves)
    try:
        s.ux.zero_()
        s.pi.zero_()
        s.Pb.zero_()
        s.ric_sv(compute_pi=1, compute_Pb=1, **kw)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("HPMPC_MI355X_RIC_WAVES", None)
    return s.ux.clone(), s.pi.clone(), s.Pb.clone()


def relerr(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


def check_oracle(qp, ux, pi, Pb, sample, tol=TOL_RIC):
    orc = _oracle()
    ux, pi, Pb = (x.cpu().numpy() for x in (ux, pi, Pb))
    N = qp.N
    worst = 0.0
    for p in sample:
        u2, p2, b2, _ = orc.ric_sv(qp.problem(p), compute_pi=1, compute_Pb=1)
        for k in range(N + 1):
            n = qp.nux(k)
            worst = max(worst, relerr(ux[p, k, :n], u2[k][:n]))
            if k < N:
                m = int(qp.nx[k + 1])
                worst = max(worst, relerr(pi[p, k, :m], p2[k][:m]), relerr(Pb[p, k, :m], b2[k][:m]))
    assert worst <= tol, worst
    return worst


@variant_only
@pytest.mark.parametrize("N,nx,nu,batch", [(100, 12, 4, 1024), (50, 8, 3, 1024)])
def test_two_wave_benchmark_shapes(N, nx, nu, batch):
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.shard import make_shard

    qp = make_shard(N, nx, nu, 0, 1, batch, boxes=False)
    s = BatchSolver(qp, k_max=1)
    ux1, pi1, Pb1 = run_sv(s, 1)
    ux2, pi2, Pb2 = run_sv(s, 2)
    # the two kernels agree to rounding
    for a, b in ((ux2, ux1), (pi2, pi1), (Pb2, Pb1)):
        assert relerr(a.cpu().numpy(), b.cpu().numpy()) <= 1e-13
    # launch splitting is bitwise the whole launch
    s.ux.zero_()
    s.pi.zero_()
    s.Pb.zero_()
    s.ric_sv(compute_pi=1, compute_Pb=1, p0=0, count=333)
    s.ric_sv(compute_pi=1, compute_Pb=1, p0=333, count=batch - 333)
    torch.cuda.synchronize()
    assert torch.equal(s.ux, ux2) and torch.equal(s.pi, pi2) and torch.equal(s.Pb, Pb2)
    check_oracle(qp, ux2, pi2, Pb2, (0, 1, batch // 2 - 1, batch - 1))


@variant_only
@pytest.mark.parametrize("N,nx,nu", [(1, 6, 2), (2, 5, 3), (3, 12, 4), (20, 10, 3), (17, 7, 5), (30, 12, 3)])
def test_two_wave_generic_shapes(N, nx, nu):
    from hpmpc_amd.batch import BatchSolver

    nxs = [nx] * (N + 1)
    nxs[0] = 3 if N > 2 else nx  # x_0 as a variable: stage 0 keeps the full factor
    qps = [random_qp(N, nxs, [nu] * (N + 1), nb=[0] * (N + 1), seed=100 + i) for i in range(8)]
    qp = stack(qps)
    s = BatchSolver(qp, k_max=1)
    ux1, pi1, Pb1 = run_sv(s, 1)
    ux2, pi2, Pb2 = run_sv(s, 2)
    for a, b in ((ux2, ux1), (pi2, pi1), (Pb2, Pb1)):
        assert relerr(a.cpu().numpy(), b.cpu().numpy()) <= 1e-12
    check_oracle(qp, ux2, pi2, Pb2, range(8))


@variant_only
def test_two_wave_clamp_variants():
    """Stages the clamp certificate rejects (the reference clamps an inner x pivot): the tile wave factorises the x
    block and hands the x factor over; the row wave adds its row half and p_eff."""
    from hpmpc_amd.batch import BatchSolver

    from helpers import XCLAMP as variants

    qps = [xclamp_qp(N=12, nx=8, nu=3, d=d, off=o, r=r) for d, o, r in variants]
    qp = stack(qps)
    s = BatchSolver(qp, k_max=1)
    ux2, pi2, Pb2 = run_sv(s, 2)
    check_oracle(qp, ux2, pi2, Pb2, range(len(variants)))


@variant_only
def test_two_wave_aliased_layout():
    import torch

    from hpmpc_amd.batch import BatchSolver
    from hpmpc_amd.ocp import mass_spring_qp

    qp = mass_spring_qp(40, 12, 4, boxes=False, batch=64)
    a = BatchSolver(qp, k_max=1, aliased=True)
    b = BatchSolver(qp, k_max=1)
    r_a = run_sv(a, 2)
    r_b = run_sv(b, 2)
    for x, y in zip(r_a, r_b):
        assert torch.equal(x, y)
    check_oracle(qp, *r_b, (0, 63))


@variant_only
def test_sv_goldens_two_wave(product):
    """The drop-in d_back_ric_rec_sv_tv_res on the two-wave kernel (HPMPC_MI355X_RIC_WAVES=2), every sv golden."""
    from hpmpc_amd.golden import load_all
    from helpers import check_case, run_case

    cases = [c for c in load_all() if c.kind in ("sv", "sv_xclamp")]
    assert len(cases) >= 8
    os.environ["HPMPC_MI355X_RIC_WAVES"] = "2"
    try:
        for case in cases:
            check_case(case, run_case(product, case))
    finally:
        os.environ.pop("HPMPC_MI355X_RIC_WAVES", None)
