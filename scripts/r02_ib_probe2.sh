#!/bin/bash
# K5-width slab (1024 x 2048 f32, 8 moving filaments), lone: band cycle breakdown per variant.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ab}
mkdir -p "$OUT"
B="python3 bench.py --nx 1024 --ny 2048 --precision f32 --steps 300 --warmup 30 --no-cpu-baseline --workload K5"
for cfg in ${CFGS:-"rows:" "cols:IBLB_BAND_ROWS=0" "rows_r0:IBLB_BAND_RESERVE_CUS=0" "cols_r0:IBLB_BAND_ROWS=0 IBLB_BAND_RESERVE_CUS=0"}; do
  lab=${cfg%%:*}; ev=${cfg#*:}
  env $ev timeout -k 10 120 $B $EXTRA > "$OUT/$lab.json" 2> "$OUT/$lab.err" || { tail -5 "$OUT/$lab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('ib_band'))" "$OUT/$lab.json" "$lab"
done
