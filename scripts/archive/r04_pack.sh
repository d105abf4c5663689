#!/bin/bash
# Packed f32 collide (round 4): deep-sweep bit-identity tests, then M f32 and K5 with the deep variants
# 3 (three-wave wall split, scalar collide: the round-3 default), 11 (packed inner chunks + wall split,
# two waves) and 9 (packed, two waves, no split), alternated twice on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04p}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu tests \
  -k "${TESTK:-sweep_deep_bit_identical and f32 or sweep_two_iterations}" > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -E "^FAILED|Error" "$OUT/pytest.log" | head
[ $rc -ne 0 ] && exit 1
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'), (d.get('ib_band') or {}).get('deep_ms_per_cycle'))" "$2" "$1"; }
for rep in 1 2; do
  for v in ${VARIANTS:-3 11 9}; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --precision f32 --steps 500 > "$OUT/Mf32_v${v}_$rep.json" 2> "$OUT/Mf32_v${v}_$rep.err" && one "M f32 variant $v" "$OUT/Mf32_v${v}_$rep.json" || exit 1
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --workload K5 --steps 300 --warmup 30 > "$OUT/K5_v${v}_$rep.json" 2> "$OUT/K5_v${v}_$rep.err" && one "K5 variant $v" "$OUT/K5_v${v}_$rep.json" || exit 1
  done
done
echo "== done"
