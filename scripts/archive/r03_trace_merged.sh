#!/bin/bash
# Kernel timelines of the K5-width slab (1024 x 2048 f32, 8 moving filaments, mid-slab and on the
# slab edge) with the merged band chain (the default there) and the chained one (IBLB_BAND_MERGE=0).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03tm}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 300 --warmup 30"
for off in ${OFFS:-0.5 0}; do
  for m in ${MERGE:-1 0}; do
    n=k5slab${SUFFIX}_${off}_m$m
    IBLB_BAND_MERGE=$m timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o trace -- $B --filament-offset $off $EXTRA \
      > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
    echo "== $n"; python3 scripts/band_timeline.py "$OUT/$n" | head -24 | tee "$OUT/${n}_timeline.txt"
  done
done
