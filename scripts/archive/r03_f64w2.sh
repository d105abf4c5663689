#!/bin/bash
# (IBLB_BND_VS and the two-wave f64 variant were temporary experiment hooks, removed after these runs: profiles/r03bv, r03w2)
# f64 deep sweep built for two waves per SIMD without the software prefetch (IBLB_DEEP_VARIANT=5)
# vs the default one-wave build (1): bit-identity tests, then M f64 alternated.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03w2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "sweep_deep_bit_identical and f64" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50"
for rep in 1 2 3; do
  for v in 1 5; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 120 $B > "$OUT/M_v${v}_$rep.json" 2> "$OUT/M_v${v}_$rep.err" || { tail -5 "$OUT/M_v${v}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" "$OUT/M_v${v}_$rep.json" "M f64 variant $v rep $rep"
  done
done
echo "== done"
