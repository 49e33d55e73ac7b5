"""the CPU restatement's C code (oracle/nrk_oracle.c) built with
AddressSanitizer + UndefinedBehaviorSanitizer and driven over every entry
point by oracle/asan_check.c (random cases plus the reference's edges).
Host-only (no GPU); the checker itself, not the product."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(ORACLE, "_asan", "asan_check")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan_check OK" in r.stdout
