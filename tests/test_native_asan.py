"""The engine's host code under AddressSanitizer + UBSan (tests/native/asan_driver.cpp,
built by tests/native/Makefile from __graft_entry__.build()): a seeded churn through every
C-ABI entry point, with the match modes checked against each other."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "native", "asan_driver")


@pytest.mark.gpu
def test_host_code_under_asan_ubsan():
    if not os.path.exists(DRIVER):
        pytest.fail("tests/native/asan_driver not built (run __graft_entry__.build())")
    env = dict(os.environ)
    # the HIP runtime keeps allocations until exit: leak reports are not ours to judge
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    p = subprocess.run([DRIVER], capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "asan driver ok" in p.stdout
    assert "runtime error" not in p.stderr  # UBSan findings
