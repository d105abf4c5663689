#!/bin/bash
# Bit-identity of the deep sweeps on the product build, then the same A/B on each library build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02c}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py -k "(sweep_deep or sweep_two or channel_no_ib or channel_shapes or fused_variants or band_cycle or boot or explicit)" \
  > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 1; }
for lib in "" ${LIBS}; do
  tag=${lib:-main}
  IBLB_LIB=${lib:+cuda_iblb_11_amd/lib/variants/libiblb_$lib.so} timeout -k 10 300 python -u scripts/tune_fused.py --rounds 3 --steps 100 --envs "${ENVS}" > "$OUT/tune_$tag.log" 2>&1 || exit 1
  echo "== $tag"; grep config "$OUT/tune_$tag.log" | python3 -c 'import sys,json; [print(round(d["median_ms_per_iter"],5), round(d["mlups"]), d["bitwise_equal_to_first"], d["config"]) for d in map(json.loads, sys.stdin)]'
done
