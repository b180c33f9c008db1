"""Link-level drop-in proof (CPU, build container only).

tools/relink/Makefile compiles the reference's own sources where they lie (only when /root/reference exists)
into an archive WITHOUT the files libhpmpc_mi355x.so replaces (d_back_ric_rec.c, d_part_cond.c,
d_ip2_res_hard.c, d_ip2_hard.c, d_res_ip_hard.c, d_ip2_soft.c, c99/d_res_ip_res_hard.c) and links
tools/relink/relink_driver.c -- the call sequence of test_problems/test_d_ip_hard.c and test_d_ric_mpc.c, which
themselves need the absent BLASFEO headers -- against it plus -lhpmpc_mi355x.  The link must succeed, every
replaced entry point the driver calls must be undefined in the driver and the reference archive and defined by
the shim, and the executable must bind them dynamically from libhpmpc_mi355x.so.  The binary is never run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("HPMPC_REF", "/root/reference")
OUT = os.path.join(ROOT, "oracle", "_ref", "relink")
LIB = os.path.join(ROOT, "hpmpc_amd", "lib", "libhpmpc_mi355x.so")

# the reference entry points the drop-in boundary replaces (the driver calls all of them)
REPLACED = [
    "d_ip2_res_mpc_hard_tv_work_space_size_bytes", "d_ip2_res_mpc_hard_tv", "d_kkt_solve_new_rhs_res_mpc_hard_tv",
    "d_res_res_mpc_hard_tv", "d_ip2_mpc_hard_tv", "d_kkt_solve_new_rhs_mpc_hard_tv", "d_res_mpc_hard_tv",
    "d_back_ric_rec_sv_tv_work_space_size_bytes", "d_back_ric_rec_sv_tv_memory_space_size_bytes",
    "d_back_ric_rec_sv_tv_res", "d_back_ric_rec_trf_tv_res", "d_back_ric_rec_trs_tv_res",
    "d_part_cond_compute_problem_size", "d_part_cond_work_space_size_bytes", "d_part_expand_work_space_size_bytes",
]

pytestmark = pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("nm") is None or not os.path.exists(LIB),
                                reason="needs the reference sources (build container), nm and the built product")


def _nm(*args):
    return subprocess.run(["nm", *args], check=True, capture_output=True, text=True).stdout


def _syms(text, kinds):
    out = set()
    for line in text.splitlines():
        parts = line.split()
        if len(parts) >= 2 and parts[-2] in kinds:
            out.add(parts[-1])
    return out


@pytest.fixture(scope="module")
def relinked():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "relink"), f"REF={REF}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(OUT, "relink_driver")


def test_link_succeeds(relinked):
    assert os.path.exists(relinked)


def test_replaced_symbols_resolve_to_the_shim(relinked):
    driver_undef = _syms(_nm(os.path.join(OUT, "relink_driver.o")), {"U"})
    archive_def = _syms(_nm(os.path.join(OUT, "libhpmpc_ref_minus.a")), {"T", "D", "B", "R"})
    shim_def = _syms(_nm("-D", "--defined-only", LIB), {"T"})
    exe_undef = _syms(_nm("-D", "--undefined-only", relinked), {"U"})
    for s in REPLACED:
        assert s in driver_undef, s              # the driver calls it
        assert s not in archive_def, s           # no reference object left defines it
        assert s in shim_def, s                  # libhpmpc_mi355x.so exports it
        assert s in exe_undef, s                 # the executable binds it dynamically (from the shim)


def test_reference_auxiliaries_still_come_from_the_reference(relinked):
    """The driver's lib4 helpers (d_zeros_align, d_cvt_mat2pmat) are the reference's own objects, linked
    statically from the archive: the shim replaces the solvers only."""
    exe_def = _syms(_nm(relinked), {"T"})
    assert {"d_zeros_align", "d_cvt_mat2pmat"} <= exe_def
    shim_def = _syms(_nm("-D", "--defined-only", LIB), {"T"})
    assert not ({"d_zeros_align", "d_cvt_mat2pmat"} & shim_def)


def test_driver_needs_the_shim_library(relinked):
    r = subprocess.run(["readelf", "-d", relinked], check=True, capture_output=True, text=True).stdout
    assert "libhpmpc_mi355x.so" in r


# ------------------------------------------------------------------ the reference's own driver, unchanged
DRV = os.path.join(ROOT, "oracle", "_ref", "drivers", "test_d_ric_mpc")
RIC_SYMS = ["d_back_ric_rec_sv_tv_res", "d_back_ric_rec_trf_tv_res", "d_back_ric_rec_trs_tv_res",
            "d_back_ric_rec_sv_tv_work_space_size_bytes", "d_back_ric_rec_sv_tv_memory_space_size_bytes"]


@pytest.fixture(scope="module")
def drivers():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "relink"), f"REF={REF}", "drivers"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return DRV


def test_unchanged_reference_driver_relinks(drivers):
    """test_problems/test_d_ric_mpc.c and tools.c compile unchanged (gcc -DTARGET_C99_4X4) and link against the
    reference archive minus the replaced objects plus -lhpmpc_mi355x: every Riccati entry point it calls is
    undefined in its object, defined by the shim, and bound dynamically by the executable."""
    drv_undef = _syms(_nm(os.path.join(OUT, "drv", "test_d_ric_mpc.o")), {"U"})
    shim_def = _syms(_nm("-D", "--defined-only", LIB), {"T"})
    exe_undef = _syms(_nm("-D", "--undefined-only", drivers), {"U"})
    for s in RIC_SYMS:
        assert s in drv_undef and s in shim_def and s in exe_undef, s


def test_reference_driver_output_is_the_golden(drivers):
    """The same unchanged driver linked against the whole reference, run here on the host, prints exactly the
    ux / pi that tests/golden/drivers/test_d_ric_mpc.npz holds (what the GPU-relinked run is compared with)."""
    import sys
    import tempfile

    import numpy as np

    from helpers import parse_ric_driver

    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "test_problems", "results"))
        text = subprocess.run([os.path.join(OUT, "test_d_ric_mpc_ref")], cwd=d, check=True, capture_output=True,
                              text=True, timeout=300).stdout
    b = parse_ric_driver(text)
    z = np.load(os.path.join(ROOT, "tests", "golden", "drivers", "test_d_ric_mpc.npz"))
    np.testing.assert_array_equal(np.concatenate([np.asarray(r) for r in b["ux"]]), z["ux"])
    np.testing.assert_array_equal(np.asarray(b["pi"]), z["pi"])
