#!/bin/bash
# (the polled iblb_synchronize measured here was reverted: no difference, profiles/r03sy)
# iblb_synchronize polling a marker event (current) vs a blocking hipStreamSynchronize (variant
# build `oldsync`: the previous iblb_ctx.hip): the driver's command (20 steps, 5 warmup) and 500
# steps, alternated.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03sy}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in new old; do
    env=""; [ $v = old ] && env="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_oldsync.so"
    for st in "20 5" "500 50"; do
      set -- $st
      env $env timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps $1 --warmup $2 > "$OUT/M_${v}_$1_$rep.json" 2> "$OUT/M_${v}_$1_$rep.err" || { tail -5 "$OUT/M_${v}_$1_$rep.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'])" "$OUT/M_${v}_$1_$rep.json" "$v steps $1 rep $rep"
    done
  done
done
echo "== done"
