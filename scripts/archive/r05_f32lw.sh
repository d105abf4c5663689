#!/bin/bash
# f32 deep sweep with two of the three moving populations in LDS, three waves per SIMD (IBLB_DEEP_VARIANT
# 139 = 11 | 128): bit identity, then M f32 and K5 alternated with the default (11), two passes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05f32lw}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    -k "sweep_deep_bit_identical and f32" > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "passed|failed" "$OUT/pytest.log" | tail -3; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
  [ $rc -eq 0 ] || exit 1
}
B="python3 bench.py --no-cpu-baseline"
for rep in 1 2; do
  for v in 11 139; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 300 $B --precision f32 > "$OUT/M_f32_v$v.$rep.json" 2> "$OUT/M.err" || { tail -5 "$OUT/M.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('M f32 v$v', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])" "$OUT/M_f32_v$v.$rep.json"
  done
done
for v in 11 139; do
  IBLB_DEEP_VARIANT=$v timeout -k 10 300 $B --workload K5 > "$OUT/K5_v$v.json" 2> "$OUT/K5.err" || { tail -5 "$OUT/K5.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('K5 v$v', d['value'], d['roofline']['launch_ms'], d['ms_per_step'])" "$OUT/K5_v$v.json"
done
echo "== done"
