"""The CPU oracle is the checker of every physics test: build it with AddressSanitizer +
UndefinedBehaviorSanitizer (oracle/Makefile `sanitize`) and step every robot under every
physics-rule switch, single-threaded and with OpenMP; any sanitizer report fails the test."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_oracle_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               OMP_NUM_THREADS="2", OMP_STACKSIZE="64M")  # ASan redzones inflate the Atlas-sized frames
    out = subprocess.run([os.path.join(ORACLE, "_san", "pbg_oracle_san"), "12"], capture_output=True, text=True,
                         timeout=600, env=env)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    assert "sanitize ok" in out.stdout
    assert "runtime error" not in out.stderr, out.stderr[-4000:]
