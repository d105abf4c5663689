#!/bin/bash
# f32 collide order A/B (round 4): the f32 parity tests on the current tree, then M f32 and K5
# benches alternating the current library and the round-3 collide order (IBLB_LIB variant r03dev,
# scripts/build_variant.sh with the round-3 iblb_device.h).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  -k "f32 or k5 or K5" > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -E "^FAILED" "$OUT/pytest.log" | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
cp gpurun_out/parity_f32.json "$OUT/" 2>/dev/null
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in cur r03; do
    L=""; [ $v = r03 ] && L="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_r03dev.so"
    env $L timeout -k 10 200 $B --precision f32 --steps 500 > "$OUT/Mf32_${v}_$rep.json" 2> "$OUT/Mf32_${v}_$rep.err" && one "M f32 $v" "$OUT/Mf32_${v}_$rep.json" || exit 1
    env $L timeout -k 10 200 $B --workload K5 --steps 300 --warmup 30 > "$OUT/K5_${v}_$rep.json" 2> "$OUT/K5_${v}_$rep.err" && one "K5 $v" "$OUT/K5_${v}_$rep.json" || exit 1
  done
done
echo "== done"
