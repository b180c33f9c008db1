"""The CPU oracle (clean-room restatement) against the golden vectors of the real reference.

This pins the oracle: every GPU parity test compares against the oracle, which is itself
checked here against outputs of the reference c99 build (tests/golden/make_golden.py).
"""
import pytest

from hpmpc_amd.golden import load_all
from helpers import check_case, run_case

CASES = load_all()


def test_goldens_present():
    kinds = {c.kind for c in CASES}
    assert {"sv", "trf_trs", "ipm", "kkt", "res", "newton", "ipm2", "kkt2", "res2", "pcond", "pcond_sv", "cond_parts", "iface", "iface_kkt", "soft"} <= kinds, kinds
    assert len(CASES) >= 20


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_oracle_matches_reference(oracle, case):
    check_case(case, run_case(oracle, case))
