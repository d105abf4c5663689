"""bench.py's N > 1 branch end to end (VERDICT r2 missing #2): two ranks launched by
torch.distributed.run exactly as the driver launches the scaling runs, here on one GPU
(--same-device: gloo process group, every rank its slab as an RCCL self ring), through the
process-group init, the prime broadcast, the barrier-bracketed timed region, the MAX reductions
of the time and of the launch timing, and the JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world=2, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--same-device", "--prime-seconds", "0.2", "--no-cpu-baseline"] + args
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("workload", ["M", "K5"])
def test_bench_two_ranks(gpu, workload):
    d = _run(["--workload", workload, "--steps", "40", "--warmup", "5"])
    assert d["n_gpus"] == 2 and d["steps"] == 40 and d["state_finite"]
    assert d["config"]["parallelism"].startswith("x-slab x2")
    assert d["value"] > 0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["frac"] is not None and r["achieved"] > 0 and r["launch_ms"] > 0
    assert r["kernel"].startswith("sweepk_kernel<K=") and "slab interior" in r["kernel"], r["kernel"]
    assert "MAX over ranks" in r["launch_timing"]
    assert "wave(s) per SIMD at" in r["limiter"] and "MODE" in r["limiter"], r["limiter"]  # the build that ran
    if workload == "K5":
        assert d["ib_band"] is not None and d["ib_band"]["deep_ms_per_cycle"] > 0  # the band cycle ran
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"bench_n2_{workload}.json"), "w") as f:
        json.dump(d, f)


def test_bench_labels_without_events(gpu):
    d = _run(["--workload", "M", "--steps", "20", "--warmup", "5", "--no-profile-events"])
    r = d["roofline"]
    assert r["frac"] is None and r["kernel"].startswith("sweepk_kernel<K=") and "not timed" in r["kernel"]
    assert r["launch_timing"].startswith("none")
