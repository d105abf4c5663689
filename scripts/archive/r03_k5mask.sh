#!/bin/bash
# (the band deep sweep took the f32 wall split under a CU-masked chain for these runs only; reverted: profiles/r03km)
# K5 (8192 x 2048 f32, 6144 moving points): the band chain on 32 / 64 CUs of its own with the deep
# sweep's f32 wall split on the others, vs the default (both streams unmasked, the two-wave deep
# sweep); the band stream tests first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03km}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "stream_arrangements or band_cycle_matches" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --workload K5"
for rep in 1 2; do
  for cus in default 32 64 16; do
    env=""; [ "$cus" != default ] && env="IBLB_BAND_CUS=$cus"
    env $env timeout -k 10 120 $B > "$OUT/K5_${cus}_$rep.json" 2> "$OUT/K5_${cus}_$rep.err" || { tail -5 "$OUT/K5_${cus}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/K5_${cus}_$rep.json" "K5 cus=$cus rep $rep"
  done
done
echo "== done"
