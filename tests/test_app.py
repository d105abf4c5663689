"""The drop-in driver `cuda_iblb_11_amd/bin/IBLB` (cuda_iblb_11_amd/app/iblb_main.cpp) against the
reference driver's contract (main.cu:263-1065): argument handling on the CPU, and on the GPU the
files of a short run compared with the same run of the restated reference (tests/app_model.py).

Text parity: every line of every file must match the oracle's text, except that a number may
differ in its last printed digit when the GPU value and the oracle value (≤ 1e-13 apart in f64)
straddle a rounding boundary of the 6-significant-digit output; such numbers must agree to 1e-5
relative (f64).  With f32 storage every number must be within 1e-4 of its column's largest
magnitude (the field-level f32 tolerance of SURVEY §8c).
"""
import os
import subprocess

import numpy as np
import pytest

import app_model as M

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(REPO, "cuda_iblb_11_amd", "bin", "IBLB")
# 288 x 192, the reference's cilia scenario (6 cilia, 48 apart, T = 1e5) for 20 iterations,
# output every 10 (P_num = 2), BigData on.  Kept short: the reference's penalty IB diverges in this
# scenario after ~30 iterations.
ARGS = ["1", "6", "48", "1.0", "1", "5", "0.0002", "2", "0", "1"]


def run_app(args, tmp_path, timeout=600, **env):
    e = dict(os.environ, IBLB_DATA_DIR=str(tmp_path) + "/", **{k: str(v) for k, v in env.items()})
    return subprocess.run([APP] + list(args), capture_output=True, text=True, timeout=timeout, env=e,
                          cwd=str(tmp_path))


def read(root, rel):
    with open(str(root) + "/" + rel) as f:
        return f.read()


def compare_text(got: str, exp: str, rtol: float, name: str, field: bool = False) -> int:
    """Line-by-line equality, numbers within tolerance where the text differs (relative to the
    number, floored at 1e-4 of the column's largest magnitude; field=True: relative to the
    column's largest magnitude, the north star's field-level f32 metric).  Returns the number
    of lines that differed textually."""
    gl, el = got.split("\n"), exp.split("\n")
    assert len(gl) == len(el), f"{name}: {len(gl)} lines vs {len(el)} expected"
    rows = [ln.split("\t") for ln in el if ln]
    width = max((len(r) for r in rows), default=0)
    colmax = np.zeros(width)
    for r in rows:
        for i, t in enumerate(r):
            colmax[i] = max(colmax[i], abs(float(t)))
    ndiff = 0
    for n, (a, b) in enumerate(zip(gl, el)):
        if a == b:
            continue
        ndiff += 1
        fa, fb = a.split("\t"), b.split("\t")
        assert len(fa) == len(fb), f"{name}:{n + 1}: {a!r} vs {b!r}"
        for i, (x, y) in enumerate(zip(fa, fb)):
            x, y = float(x), float(y)
            scale = colmax[i] if field else max(abs(y), colmax[i] * 1e-4)
            assert abs(x - y) <= rtol * scale + 1e-300, f"{name}:{n + 1}: {a!r} vs {b!r}"
    return ndiff


# ---- CPU: argument handling (no device touched) ---------------------------------------------------

def test_app_built():
    assert os.access(APP, os.X_OK), "build the driver: make (or __graft_entry__.build())"


def test_too_few_arguments(tmp_path):
    p = run_app(["1", "6", "48"], tmp_path, timeout=60)
    assert p.returncode == 1
    assert p.stdout == "Too few arguments! 3 entered of 10 required. \n"  # main.cu:284-289


def test_not_enough_cilia(tmp_path):
    p = run_app(["1", "3", "48", "1.0", "1", "5", "1", "100", "0", "0"], tmp_path, timeout=60)
    assert p.returncode == 1  # XDIM = 144 < 2 * LENGTH (main.cu:303-308)
    assert p.stdout == "not enough cilia in simulation! Cilia spacing of 48 requires at least 4 cilia\n"


def test_zero_output_interval_refused(tmp_path):
    # ITERATIONS / P_num == 0: the reference takes `it % 0` (crash); the driver refuses
    p = run_app(["1", "6", "48", "1.0", "1", "1", "1", "100", "0", "0"], tmp_path, timeout=60)
    assert p.returncode == 1 and "Output interval is zero" in p.stdout


def test_parameters_match_reference_defaults():
    from cuda_iblb_11_amd import workloads as W
    p = M.params(["1", "6", "48", "1.0", "1", "5", "1", "100", "0", "0"])
    assert p["XDIM"] == 288 and p["T"] == 100000 and p["ITERATIONS"] == 100000 and p["INTERVAL"] == 1000
    assert p["TAU"] == W.TAU and p["TAU2"] == W.TAU2
    q = M.params(ARGS)
    assert q["ITERATIONS"] == 20 and q["INTERVAL"] == 10
    assert M.paths(q)["flux"] == "/Flux/1_6_48_1_1x5-flux.dat"


def test_no_device_fails_loudly(tmp_path):
    """Without a GPU the driver stops at context creation: there is no CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    p = run_app(ARGS, tmp_path, timeout=120)
    assert p.returncode == 1 and "iblb_create failed (-7)" in p.stderr


# ---- GPU: file parity with the restated reference ---------------------------------------------------

@pytest.fixture(scope="module")
def expected():
    return M.expected_run(ARGS)


def check_simlog(text, p):
    lines = text.split("\n")
    exp = M.simlog_lines(p)
    for n, e in enumerate(exp):
        if e is not None:
            assert lines[n] == e, (n, lines[n], e)
    rest = lines[len(exp):]
    # it == INTERVAL is reached (ITERATIONS > INTERVAL): completion estimate, then the runtime
    assert rest[0] == "" and rest[1].startswith("Completion time: ")
    assert rest[-2].startswith("Total runtime: ") and rest[-1] == ""


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_app_matches_reference_files(gpu, tmp_path, expected, precision):
    p, files = expected
    r = run_app(ARGS, tmp_path, IBLB_PRECISION=precision)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Initialising...\n" in r.stdout and "Running Simulation...\n" in r.stdout
    for rel, text in files.items():
        if precision == "f64":
            compare_text(read(tmp_path, rel), text, 1e-5, rel)
        else:  # f32 storage: max |a - b| / max |b| <= 1e-4 per column
            compare_text(read(tmp_path, rel), text, 1e-4, rel, field=True)
    check_simlog(read(tmp_path, M.paths(p)["simlog"]), p)


@pytest.mark.gpu
def test_app_restart_continues_the_run(gpu, tmp_path, expected):
    """IBLB_CHECKPOINT / IBLB_RESTART: 10 iterations, checkpoint, then the 20-iteration run resumed
    from it writes the same it = 10 fields and final flux as the uninterrupted reference run."""
    p, files = expected
    first = ARGS[:6] + ["0.0001", "1"] + ARGS[8:]  # ITERATIONS = 10, one output interval
    assert M.params(first)["ITERATIONS"] == 10
    ck = str(tmp_path / "ck")
    r = run_app(first, tmp_path, IBLB_CHECKPOINT=ck, IBLB_CHECKPOINT_EVERY=10)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(ck + ".rank0")
    os.remove(str(tmp_path) + "/" + M.paths(p)["raw"] + "0-fluid.dat")
    r = run_app(ARGS, tmp_path, IBLB_RESTART=ck)
    assert r.returncode == 0, r.stdout + r.stderr
    rel = M.paths(p)["raw"] + "10-fluid.dat"
    compare_text(read(tmp_path, rel), files[rel], 1e-5, rel)
    assert not os.path.exists(str(tmp_path) + "/" + M.paths(p)["raw"] + "0-fluid.dat")
    last_got = read(tmp_path, M.paths(p)["flux"]).strip().split("\n")[-1]
    last_exp = files[M.paths(p)["flux"]].strip().split("\n")[-1]
    compare_text(last_got, last_exp, 1e-5, "final flux")


@pytest.mark.gpu
def test_app_stops_a_diverged_run(gpu, tmp_path):
    """The reference's own scenario diverges by iteration ~40 (penalty IB gain) and
    the reference writes NaN fields on; the driver checks the populations at every output
    iteration (iblb_count_nonfinite, collective) and stops with status 3 instead."""
    args = ARGS[:6] + ["0.001", "10"] + ARGS[8:]  # 100 iterations, output every 10
    p = M.params(args)
    assert p["ITERATIONS"] == 100
    r = run_app(args, tmp_path)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "the run diverged" in r.stderr, r.stderr
    # the diverged iteration's output is written as the reference writes it (NaN fields), then the
    # run stops: the flux file ends at that iteration (no final line)
    it = int(r.stderr.split("populations at iteration ")[1].split()[0])
    assert 10 <= it < 100 and it % 10 == 0, r.stderr
    fluid = read(tmp_path, M.paths(p)["raw"] + f"{it}-fluid.dat")
    assert "nan" in fluid.lower()
    assert not os.path.exists(str(tmp_path) + "/" + M.paths(p)["raw"] + f"{it + 10}-fluid.dat")
    assert len(read(tmp_path, M.paths(p)["flux"]).strip().split("\n")) == it // 10 + 1


@pytest.mark.gpu
def test_app_nan_guard_off_keeps_reference_behaviour(gpu, tmp_path):
    """IBLB_NAN_GUARD=0: the diverged run goes on to the end as the reference's does (NaN fields
    written at every output iteration, the final flux line), with one warning."""
    args = ARGS[:6] + ["0.001", "10"] + ARGS[8:]
    p = M.params(args)
    r = run_app(args, tmp_path, IBLB_NAN_GUARD=0)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stderr.count("the run diverged") == 1, r.stderr
    assert os.path.exists(str(tmp_path) + "/" + M.paths(p)["raw"] + "90-fluid.dat")
    assert len(read(tmp_path, M.paths(p)["flux"]).strip().split("\n")) == 11
