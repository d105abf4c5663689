#!/bin/bash
# Cilia tests (band cycle with on-device kinematics) and timings.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03cil}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "cilia or checkpoint or band" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python3 scripts/r03_cilia.py 6 48 192 500 > "$OUT/cilia_ref.log" 2>&1 && tail -1 "$OUT/cilia_ref.log" || { tail -5 "$OUT/cilia_ref.log"; exit 1; }
timeout -k 10 200 python3 scripts/r03_cilia.py 64 128 192 500 > "$OUT/cilia_64.log" 2>&1 && tail -1 "$OUT/cilia_64.log" || { tail -5 "$OUT/cilia_64.log"; exit 1; }
timeout -k 10 200 python3 scripts/r03_cilia.py 64 128 2048 200 f32 > "$OUT/cilia_64_2048.log" 2>&1 && tail -1 "$OUT/cilia_64_2048.log" || { tail -5 "$OUT/cilia_64_2048.log"; exit 1; }
