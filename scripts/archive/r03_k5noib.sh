#!/bin/bash
# The K5-width slab (1024 x 2048 f32) without IB, lone and on the RCCL self ring: the no-IB time
# the band cycle's slab is compared with (<= 1.3x).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03kn}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --nx 1024 --ny 2048 --precision f32"
for r in "" "--rccl-self"; do
  tag=plain$(echo "$r" | tr -d ' -')
  timeout -k 10 120 $B $r > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'])" "$OUT/$tag.json" "1024x2048 f32 no IB $r"
done
