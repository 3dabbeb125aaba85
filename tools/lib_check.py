"""Dev tool: run one of the float64 teacher-forced parity checks of tests/test_f64.py against a given
build of libpbg_amd.so (an A/B variant), in its own process per library.
  python tools/lib_check.py LIB ENV_ID N STEPS [kernel=K] ...
Prints the parity record and PASS / FAIL."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
lib, env_id, n, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
opts = {k: int(v) for k, v in (a.split("=") for a in sys.argv[5:])}
import pybulletgym_amd  # noqa: E402,F401
from pybulletgym_amd import _native  # noqa: E402
_native.LIB_PATH = os.path.abspath(lib)
import test_f64  # noqa: E402
try:
    test_f64._teacher_forced64(env_id, n, steps, name=f"{os.path.basename(lib)}:{env_id}:{opts}", **opts)
    print("PASS", os.path.basename(lib), env_id, opts)
except AssertionError as e:
    print("FAIL", os.path.basename(lib), env_id, opts, str(e)[:300])
