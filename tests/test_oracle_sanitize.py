"""The parity checker must itself be free of undefined behaviour: the oracle is rebuilt
with -fsanitize=address,undefined (oracle/Makefile `asan`) and the whole golden suite runs through it in a
child python with the sanitizer runtimes preloaded.  A heap overflow or UB report fails the test."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_goldens_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not (asan and ubsan):
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "oracle_sanitize_run.py"),
                        os.path.join(ROOT, "oracle", "liboracle_asan.so")], env=env, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0 and "sanitized goldens ok" in r.stdout, (r.stdout[-2000:] + r.stderr[-4000:])
