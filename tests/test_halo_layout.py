"""The halo slot maps on the CPU: a host build of iblb_device.h / iblb_kernels.h checks that
every halo (one-step, 2-step, IB, deep K = 3..6) carries exactly what the boundary kernels pull,
once each, and that sender and receiver agree (tests/native/halo_layout_check.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_halo_slot_maps(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "halo_layout_check")
    src = os.path.join(HERE, "native", "halo_layout_check.cpp")
    inc = os.path.join(REPO, "cuda_iblb_11_amd", "csrc")
    subprocess.run([hipcc, "-std=c++17", "-O1", "-x", "hip", "--offload-arch=gfx950", "-I", inc, src, "-o", exe],
                   check=True, capture_output=True, timeout=300)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and "halo layout: ok" in p.stdout, p.stdout + p.stderr
