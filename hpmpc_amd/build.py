"""Build recipes for the in-tree native artefacts (no JIT cache: the .so files travel with the repo).

* hpmpc_amd/lib/libhpmpc_mi355x.so -- HIP kernels for gfx950 + the reference-named C ABI (product)
* oracle/liboracle.so              -- clean-room CPU restatement (test infrastructure)
* oracle/_ref/libhpmpc_ref.so      -- the real reference c99 path (only when /root/reference exists)
"""
from __future__ import annotations

import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hpmpc_amd", "csrc")
LIBDIR = os.path.join(ROOT, "hpmpc_amd", "lib")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HPMPC_ARCH", "gfx950")
SOURCES = ["hpmpc_kernels.hip", "hk_wide.hip", "hk_wide_ipm.hip", "hk_soft.hip", "hpmpc_capi.cpp", "hpmpc_capi_wide.cpp",
           "hpmpc_capi_wide_ipm.cpp", "hpmpc_capi_iface.cpp", "hpmpc_capi_mpc.cpp"]
HEADERS = ["hpmpc_api.h", "hk_ipm_body.h", "hk_prims.h", "hk_riccati.h", "hk_ipm.h", "hk_mw.h", "hpmpc_kargs.h", "hk_wide_args.h", "hk_wide_core.h", "hk_wide_host.h", "hk_soft_args.h", "hk_launch_guard.h"]
# MFMA accumulators stay in ordinary VGPRs: the stage tile is read and written by VALU code between
# MFMAs, and the AGPR form costs 8 v_accvgpr moves each way per MFMA group.
KFLAGS = ["-mllvm", "-amdgpu-mfma-vgpr-form"] + os.environ.get("HK_EXTRA_FLAGS", "").split()
# Per-source flags.  The narrow IPM / Riccati passes use the memory-clause machine scheduler: a same-box A/B
# (tools/gpu_ab.sh, profiles/ab_sched_max_memory_clause/) measured hk_ipm_corr 3.161 -> 3.125 ms per step with
# the other passes unchanged (max-ilp instead slowed the factorisation by 8 %).
SRC_FLAGS = {"hpmpc_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]}


EXPORTS = os.path.join(CSRC, "exports.map")


def _newer(out, deps):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in deps)


def _deps(src, hdrs_all):
    """The headers a source reaches through its quoted #include lines (transitively, within csrc/ and include/)."""
    import re
    seen, todo = set(), [os.path.join(CSRC, src)]
    while todo:
        path = todo.pop()
        try:
            text = open(path).read()
        except OSError:
            continue
        for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
            for cand in (os.path.join(os.path.dirname(path), name), os.path.join(CSRC, name),
                         os.path.join(ROOT, "include", os.path.basename(name))):
                if os.path.exists(cand) and cand not in seen:
                    seen.add(cand)
                    todo.append(cand)
                    break
    return sorted(seen | {h for h in hdrs_all if os.path.basename(h) == "hpmpc_mi355x.h"})


def build_hip(force: bool = False, verbose: bool = False, variant: str | None = None, extra=(), sources=()) -> str:
    """Each source compiles to its own object under build/ (rebuilt when it or a header is newer), then one
    link; a one-file change recompiles one translation unit.  variant: an A/B build with `extra` compiler flags,
    objects under build/obj_<variant>, library hpmpc_amd/lib/ab/lib<variant>.so (tools/gpu_ab.sh)."""
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(ROOT, "build", "obj" if variant is None else f"obj_{variant}")
    os.makedirs(objdir, exist_ok=True)
    out = os.path.join(LIBDIR, "libhpmpc_mi355x.so")
    if variant is not None:
        os.makedirs(os.path.join(LIBDIR, "ab"), exist_ok=True)
        out = os.path.join(LIBDIR, "ab", f"lib{variant}.so")
    hdrs_all = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "hpmpc_mi355x.h")]
    # -fvisibility=hidden: only include/hpmpc_mi355x.h's functions are exported (csrc/hpmpc_api.h)
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-function"] + KFLAGS + list(extra)
    objs, procs = [], []
    for src in SOURCES + list(sources):
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        if force or not _newer(obj, [os.path.join(CSRC, src)] + _deps(src, hdrs_all)):
            cmd = common + SRC_FLAGS.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((src, subprocess.Popen(cmd)))
    for src, pr in procs:
        if pr.wait() != 0:
            raise subprocess.CalledProcessError(pr.returncode, src)
    if procs or force or not _newer(out, objs + [EXPORTS]):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", f"-Wl,--version-script={EXPORTS}"] + objs + \
              ["-o", out]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


def build_stamps(verbose: bool = False, force: bool = False) -> str:
    """Diagnostic variant with s_memtime stamps (tools/stamps.py) and the multi-wave kernel's lost-hand-over hook
    (tests/test_gpu_parity.py test_multiwave_expired_wait_drains); never loaded by the product."""
    out = build_hip(force=force, verbose=verbose, variant="stamps", extra=["-DHK_STAMPS"])
    dst = os.path.join(LIBDIR, "libhpmpc_mi355x_stamps.so")
    if not _newer(dst, [out]):
        import shutil

        shutil.copy2(out, dst)
    return dst


def build_ric2(verbose: bool = False, force: bool = False) -> str:
    """The two-wave Riccati sv (hk_ric2.hip, a measured negative result) is not in the product
    library: this variant links it (-DHK_RIC2, HPMPC_MI355X_RIC_WAVES=2 selects it), for tests/test_gpu_ric2.py."""
    return build_hip(force=force, verbose=verbose, variant="ric2", extra=["-DHK_RIC2"], sources=["hk_ric2.hip"])


def build_calib(verbose: bool = False) -> str:
    """HBM counter calibration kernel (tools/hbm_calib.hip; profiling tool, not part of the product)."""
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, "libhbm_calib.so")
    src = os.path.join(ROOT, "tools", "hbm_calib.hip")
    if _newer(out, [src, os.path.join(CSRC, "hk_prims.h")]):
        return out
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", src, "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out


def build_oracle(force: bool = False) -> None:
    odir = os.path.join(ROOT, "oracle")
    targets = ["oracle", "oracle_fma"]  # oracle_fma: the build spread that gates the configs[4] IPM test
    if os.path.isdir(os.environ.get("HPMPC_REF", "/root/reference")):
        targets += ["ref", "ref_avx"]  # ref_avx: the alternate IPM's goldens (make_golden.py)
    subprocess.run(["make", "-s", "-C", odir] + (["-B"] if force else []) + targets, check=True)
    if "ref" in targets:  # the reference's own test_d_ric_mpc.c, unchanged, relinked against the product
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "relink"), "drivers"], check=True)


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hip(force=force, verbose=verbose)
    build_stamps(verbose=verbose, force=force)
    build_ric2(verbose=verbose, force=force)
    build_calib(verbose=verbose)
    build_oracle(force=force)


if __name__ == "__main__":
    build_all(force=True, verbose=True)
