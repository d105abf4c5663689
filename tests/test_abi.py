"""The drop-in boundary on CPU: libiblb.so loads, exports every function include/iblb.h
declares, and refuses to run without a HIP device (no CPU fallback)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import cuda_iblb_11_amd as P
from cuda_iblb_11_amd import _lib as L


def test_library_exports_every_header_symbol():
    names = L.header_functions()
    assert len(names) >= 30
    lib = L.load()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes signature table covers exactly the header
    assert sorted(L._SIGS) == names


def test_exports_are_c_abi():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for n in L.header_functions():
        assert n in exported, f"{n} not exported unmangled"


def test_library_is_gfx950():
    data = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_config_default_matches_reference_defaults():
    cfg = L.Config()
    assert L.load().iblb_config_default(C.byref(cfg)) == 0
    assert (cfg.nx, cfg.ny) == (288, 192)                 # main.cu:270-271 (c_num 6 x c_space 48)
    assert abs(cfg.tau - 2.806798146151282) < 1e-15        # main.cu:320
    assert abs(cfg.tau2 - 0.5361251085069444) < 1e-15      # main.cu:321
    assert cfg.flux_norm == 192.0 and cfg.flux_column == 283  # ImmersedBoundary.cu:259-261
    assert L.load().iblb_version().decode().startswith("iblb")


def test_create_without_device_fails_loudly():
    if L.device_count() > 0:
        pytest.skip("a HIP device is visible here")
    with pytest.raises(P.IblbError) as e:
        P.Lattice(64, 32)
    assert e.value.code == L.IBLB_ERR_NODEVICE
    assert "no HIP device" in str(e.value)


def test_argument_validation_without_device():
    lib = L.load()
    cfg = L.Config()
    lib.iblb_config_default(C.byref(cfg))
    h = C.c_void_p()
    cfg.ny = 1
    assert lib.iblb_create(C.byref(cfg), C.byref(h)) == L.IBLB_ERR_ARG
    cfg.ny, cfg.tau = 192, 0.4
    assert lib.iblb_create(C.byref(cfg), C.byref(h)) == L.IBLB_ERR_ARG
    assert lib.iblb_equilibrium(None, None, None, None, None, 4, 4, 1.0, None) == L.IBLB_ERR_ARG
    assert lib.iblb_step(None, 1) == L.IBLB_ERR_ARG
    assert lib.iblb_streaming(None, None, 0, 4, None) == L.IBLB_ERR_ARG


def test_slab_plan():
    assert P.plan_slabs(4096, 8) == [(512 * r, 512) for r in range(8)]
    plan = P.plan_slabs(90, 4)
    assert sum(c for _, c in plan) == 90 and plan[0][0] == 0
    assert all(plan[i][0] + plan[i][1] == plan[i + 1][0] for i in range(3))
    with pytest.raises(ValueError):
        P.plan_slabs(3, 4)


def test_split_helpers_roundtrip():
    nx, ny = 10, 4
    rho = np.arange(nx * ny, dtype=float)
    parts = [P.split_state(rho, 1, nx, ny, xb, xc) for xb, xc in P.plan_slabs(nx, 3)]
    back = np.concatenate([p.reshape(ny, -1) for p in parts], axis=1).ravel()
    assert np.array_equal(back, rho)
    f = np.arange(9 * nx * ny, dtype=float)
    fp = [P.split_populations(f, nx, ny, xb, xc) for xb, xc in P.plan_slabs(nx, 2)]
    back = np.concatenate([p.reshape(ny, -1, 9) for p in fp], axis=1).ravel()
    assert np.array_equal(back, f)


def test_struct_layouts_match_the_header(tmp_path):
    """The Python mirror's ctypes structs (cuda_iblb_11_amd/_lib.py) against the C header: size and
    every field's offset of iblb_config, iblb_timing and iblb_cilia, from a C program compiled
    with gcc against include/iblb.h (no device needed)."""
    import shutil
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"iblb_config": L.Config, "iblb_timing": L.Timing, "iblb_cilia": L.Cilia}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "iblb.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'    printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'    printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ['    return 0;', '}']
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(repo, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {(ln.split()[0], ln.split()[1]): int(ln.split()[2]) for ln in out if ln.strip()}
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_abi_version_matches_header():
    """IBLB_ABI_VERSION of include/iblb.h is what the library was built with (a struct crossing the ABI
    changed layout: the version moves), and iblb_get_timing_ex exists for callers of older headers."""
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "iblb.h")).read()
    v = int(re.search(r"#define IBLB_ABI_VERSION (\d+)", hdr).group(1))
    lib = L.load()
    assert lib.iblb_abi_version() == v
    assert f"abi {v}" in lib.iblb_version().decode()
    assert lib.iblb_get_timing_ex(None, None, 0, 0) == L.IBLB_ERR_ARG


def test_bench_limiter_names_the_build():
    """bench.py's roofline.limiter is built from the deep build the library reports
    for its last deep launch (iblb_timing deep_mode / deep_vs / deep_waves_per_simd / deep_vgprs) and the
    SQ passes' VALU issue share, not from a fixed string."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    f32 = bench.deep_limiter({"deep_mode": 593, "deep_vs": 2, "deep_waves_per_simd": 3, "deep_vgprs": 165},
                             {"valu_issue_share": 0.27}, "f32")
    assert "3 wave(s) per SIMD at 165 VGPRs" in f32 and "LDS window" in f32 and "packed" in f32, f32
    assert "27 %" in f32 and "~81 %" in f32 and "(hbm)" in f32, f32
    f64 = bench.deep_limiter({"deep_mode": 785, "deep_vs": 2, "deep_waves_per_simd": 1, "deep_vgprs": 239}, None, "f64")
    assert "1 wave(s) per SIMD at 239 VGPRs" in f64 and "preshift" in f64 and "packed" not in f64, f64
    assert "dependent latency" in bench.deep_limiter({}, None, "f64")
