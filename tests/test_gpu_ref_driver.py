"""The reference's own driver, unchanged, on the MI355X.

test_problems/test_d_ric_mpc.c (with test_problems/tools.c) is compiled unchanged from the reference sources and
linked against the reference archive minus the files libhpmpc_mi355x.so replaces plus -lhpmpc_mi355x
(tools/relink/Makefile, in the build container; the binary travels to the GPU box as oracle/_ref/drivers/).  Run
here, its 1000 sv + 1000 trf + 1000 trs calls go through the drop-in boundary to the GPU, and the ux / pi it
prints (d_print_mat, "%9.5f") must be what the same driver linked against the whole reference prints on the
host (tests/golden/drivers/test_d_ric_mpc.npz, make_golden.py driver()).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "oracle", "_ref", "drivers", "test_d_ric_mpc")


def test_unchanged_reference_driver_on_gpu(tmp_path):
    assert os.path.exists(DRV), "relinked reference driver not built (tools/relink/Makefile drivers)"
    from helpers import parse_ric_driver

    (tmp_path / "test_problems" / "results").mkdir(parents=True)
    # The driver allocates hpi[0] with pnx_v[0] = 0 doubles (test_d_ric_mpc.c:498) and every sv / trs call then
    # writes pi_0 (nx[1] = 8 doubles) into it -- the reference itself does (d_back_ric_rec.c forward loop from
    # nn = 0), a heap overflow that the all-CPU run survives only by heap layout, while the HIP runtime's own heap
    # traffic trips glibc's chunk checks ("corrupted size vs. prev_size").  With every allocation in its own
    # mmap'd pages the overflow stays inside the page's slack and the driver runs unchanged.
    tun = "glibc.malloc.mmap_threshold=0"
    env = dict(os.environ, GLIBC_TUNABLES=(os.environ["GLIBC_TUNABLES"] + ":" + tun) if os.environ.get(
        "GLIBC_TUNABLES") else tun)
    r = subprocess.run([DRV], cwd=tmp_path, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "hpmpc_mi355x" not in r.stderr, r.stderr[-2000:]  # no error line from the shim
    b = parse_ric_driver(r.stdout)
    z = np.load(os.path.join(ROOT, "tests", "golden", "drivers", "test_d_ric_mpc.npz"))
    ux = np.concatenate([np.asarray(x) for x in b["ux"]])
    assert ux.shape == z["ux"].shape and np.asarray(b["pi"]).shape == z["pi"].shape
    # same numbers at the printed precision (one unit of the 5th decimal covers a rounding-boundary flip)
    np.testing.assert_allclose(ux, z["ux"], rtol=0, atol=1.01e-5)
    np.testing.assert_allclose(np.asarray(b["pi"]), z["pi"], rtol=0, atol=1.01e-5)
    print(r.stdout.strip().splitlines()[-1])  # the driver's own timing line (sv / trf / trs through the GPU)


RELINK = os.path.join(ROOT, "oracle", "_ref", "drivers", "relink_driver")
# gates per printed quantity (tests/helpers.py): Riccati 1e-12; the residual IPM, its KKT re-solve and residuals
# 1e-10; the alternate IPM (no residual correction, stopped at mu_tol 1e-8) and its re-solve TOL_KKT2
GATES = {"sv": 1e-12, "trs": 1e-12, "ipm": 1e-10, "kkt": 1e-10, "res": 1e-10, "ipm2": 1e-8, "kkt2": 1e-8,
         "res2": 1e-8}


def _parse_relink(text):
    vals, heads = {}, []
    for line in text.splitlines():
        w = line.split()
        if not w:
            continue
        if w[0] in ("ipm", "ipm2") and w[1] == "status":
            heads.append((w[0], int(w[2]), int(w[4])))
        elif "." in w[0]:
            vals[(w[0], int(w[1]))] = np.array([float(x) for x in w[2:]])
    return heads, vals


def test_relinked_ipm_driver_on_gpu():
    """tools/relink/relink_driver.c -- the low-level call sequence of test_problems/test_d_ip_hard.c (IPM, KKT re-solve,
    residuals, the alternate IPM and its re-solve) and test_d_ric_mpc.c (sv, trf, trs) through the reference's own
    headers and auxiliary objects -- linked against the reference archive minus the replaced files plus
    -lhpmpc_mi355x, run on the MI355X: every number it prints against the same driver linked against the whole
    reference (tests/golden/drivers/relink_driver.txt): status and kk identical, values at the gates above."""
    assert os.path.exists(RELINK), "relinked driver not built (tools/relink/Makefile drivers)"
    r = subprocess.run([RELINK], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "hpmpc_mi355x" not in r.stderr, r.stderr[-2000:]
    heads, vals = _parse_relink(r.stdout)
    rheads, rvals = _parse_relink(open(os.path.join(ROOT, "tests", "golden", "drivers", "relink_driver.txt")).read())
    assert heads == rheads and len(heads) == 2
    assert vals.keys() == rvals.keys()
    # kkt2 and its residuals res2 against the reference's default-target build (make_golden.py driver(): the c99
    # build's alternate KKT re-solve mis-binds its gradient helper and ends 8.3e-8 from every other build here)
    kkt2 = np.load(os.path.join(ROOT, "tests", "golden", "drivers", "relink_kkt2_avx.npz"))
    for key, ref in rvals.items():
        tag = key[0].split(".")[0]
        tol = 1e-9 if key[0] == "ipm.stat" else GATES[tag]
        if tag in ("kkt2", "res2"):
            ref = kkt2[f"{key[0].split('.')[1]}_{key[1]}"]
        got = vals[key]
        assert got.shape == ref.shape, key
        e = float(np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref)), initial=0.0))
        assert e <= tol, (key, e)
