"""Sanitizer runs of the CPU-side code: the oracle restatement and the
host driver built with AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile.san), run here
on the CPU.  The oracle harness (oracle/san_main.c) drives every restated kernel, both spread forms
and the cilia kinematics with points on the lattice's x edges and walls; the driver runs its argument
checks and its no-device path.  Any sanitizer finding aborts the program (-fno-sanitize-recover)."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "oracle", "_san")


@pytest.fixture(scope="module")
def san_build():
    r = subprocess.run(["make", "-s", "-f", os.path.join(REPO, "oracle", "Makefile.san")], capture_output=True,
                       text=True, cwd=REPO)
    assert r.returncode == 0, r.stdout + r.stderr
    return SAN


def run(args, **env):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    e.update({k: str(v) for k, v in env.items()})
    return subprocess.run(args, capture_output=True, text=True, timeout=600, env=e)


def clean(r):
    return "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr and "LeakSanitizer" not in r.stderr


def test_oracle_under_asan_ubsan(san_build):
    r = run([os.path.join(san_build, "oracle_san")])
    assert r.returncode == 0 and clean(r), r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and abs(out["delta_sum"] - 0.5) < 1e-4  # phi sums to ~1 over a row; x-only row at y offset 0.5


def test_driver_under_asan_ubsan(san_build, tmp_path):
    app = os.path.join(san_build, "IBLB_san")
    env = {"ASAN_OPTIONS": "detect_leaks=0"}  # the HIP runtime's own allocations are not ours to audit
    r = run([app, "1", "2", "3"], **env)
    assert r.returncode == 1 and "Too few arguments" in r.stdout and clean(r), r.stdout + r.stderr
    r = run([app, "1", "6", "48", "1.0", "1", "1", "1", "0", "0", "1"], **env)  # P_num = 0 (main.cu:301 divides by it)
    assert r.returncode == 1 and "Output interval is zero" in r.stdout and clean(r), r.stdout + r.stderr
    r = run([app, "1", "2", "48", "1.0", "1", "1", "1", "10", "0", "1"], **env)  # XDIM 96 < 2 LENGTH (main.cu:303)
    assert r.returncode == 1 and "not enough cilia" in r.stdout and clean(r), r.stdout + r.stderr
    r = run([app, "1", "6", "48", "1.0", "1", "2", "0.1", "10", "0", "1"], IBLB_DATA_DIR=str(tmp_path) + "/", **env)
    assert clean(r), r.stdout + r.stderr
    if "no HIP device" in r.stdout + r.stderr:  # this container: the HIP path fails loudly, no CPU fallback
        assert r.returncode != 0
    else:
        assert r.returncode == 0, r.stdout + r.stderr
