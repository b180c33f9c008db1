"""Child process of tests/test_oracle_sanitize.py: every golden case through the sanitizer build of the
oracle (oracle/liboracle_asan.so), under libasan/libubsan preloaded by the parent.  Any out-of-bounds
access or undefined behaviour aborts the process with a sanitizer report."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from hpmpc_amd.cabi import HpmpcAPI, load  # noqa: E402
from hpmpc_amd.golden import load_all  # noqa: E402
from helpers import check_case, run_case  # noqa: E402

api = HpmpcAPI(load(sys.argv[1]), "orc_")
n = 0
for case in load_all():
    check_case(case, run_case(api, case))
    n += 1
print(f"sanitized goldens ok: {n}")
