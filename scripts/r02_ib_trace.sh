#!/bin/bash
# Kernel + HIP API trace of the K5-width lone slab band cycle (1024 x 2048 f32, moving filaments).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ad}
mkdir -p "$OUT"
for cfg in ${CFGS:-"rows:"}; do
  lab=${cfg%%:*}; ev=${cfg#*:}
  env $ev timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/$lab" -o trace \
    -- python3 bench.py --nx 1024 --ny 2048 --precision f32 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --workload K5 \
    > "$OUT/$lab.json" 2> "$OUT/$lab.err" || { tail -20 "$OUT/$lab.err"; exit 1; }
  python3 scripts/band_timeline.py "$OUT/$lab" | tee "$OUT/${lab}_timeline.txt"
done
