#!/bin/bash
# Experiment: CUs of the IB band chain's stream (IBLB_BAND_CUS; default = one XCD's worth, two
# when the trapezoids hold > 5 % of the updates; -2 = unmasked high-priority stream; 0 = one
# stream in sequence) on K3, K5 and the K5-width slab with filaments on the edge / mid-slab.
set -o pipefail
OUT=gpurun_out/${TAG:-r03c}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for cus in default 8 16 -2 0; do
  env=""; [ "$cus" != default ] && env="IBLB_BAND_CUS=$cus"
  for w in "K3" "K5" "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5"; do
    tag=$(echo "$w" | tr -d ' -')
    env $env timeout -k 10 120 $B --workload $w > "$OUT/${tag}_$cus.json" 2> "$OUT/${tag}_$cus.err" || { tail -5 "$OUT/${tag}_$cus.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/${tag}_$cus.json" "cus=$cus $w"
  done
done
# f32 deep sweep with 4 cells per lane (IBLB_DEEP_VS=4) vs the default 2
for vs in 2 4; do
  IBLB_DEEP_VS=$vs timeout -k 10 120 python3 bench.py --no-cpu-baseline --precision f32 > "$OUT/Mf32_vs$vs.json" 2> "$OUT/Mf32_vs$vs.err" || { tail -5 "$OUT/Mf32_vs$vs.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'])" "$OUT/Mf32_vs$vs.json" "M f32 vs=$vs"
done
