#!/bin/bash
# Deep-sweep rewrite: bit-identity tests, then an interleaved A/B of depth / cells per lane / width.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02b}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py -k "sweep_deep or sweep_two or channel_no_ib or channel_shapes or fused_variants or band_cycle or boot" \
  > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python -u scripts/tune_fused.py --rounds 4 --steps 100 --envs "${ENVS}" > "$OUT/tune.log" 2>&1 || exit 1
grep config "$OUT/tune.log"
