"""The C oracle (and with it the CPU baseline) under AddressSanitizer +
UndefinedBehaviorSanitizer, including leak checks: every entry
point over edge sizes, short inputs and non-finite values
(oracle/sanitize_main.c).  Host code only -- GPU sanitizers are not available
on this pool."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_is_asan_ubsan_clean():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize: clean" in r.stdout
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
