#!/bin/bash
# (IBLB_DEEP_WALLX4 was a temporary tuning hook, removed after these runs: profiles/r03s1)
# f32 wall split with one-cell wall chunks: bit-identity tests, then M f32 for wall sweeps per inner
# sweep IBLB_DEEP_WALLX4 / 4 vs the two-wave build (variant 1), alternated.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03s1}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "sweep_deep_bit_identical" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50 --precision f32"
for rep in 1 2; do
  for cfg in "1 3" "3 2" "3 3" "3 4" "3 6"; do
    set -- $cfg
    IBLB_DEEP_VARIANT=$1 IBLB_DEEP_WALLX4=$2 timeout -k 10 120 $B > "$OUT/M_v$1_w$2_$rep.json" 2> "$OUT/M_v$1_w$2_$rep.err" || { tail -5 "$OUT/M_v$1_w$2_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" "$OUT/M_v$1_w$2_$rep.json" "M f32 variant $1 wallx4 $2 rep $rep"
  done
done
echo "== done"
