#!/bin/bash
# K5 at N = 1 (8192 x 2048 f32, 64 filaments on every slab edge): kernel timeline of the band cycle
# (band_timeline.py: median cycle, median duration per kernel kind, one cycle's kernels by queue).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06k5tl}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload ${WL:-K5} --steps 280 --warmup 28"
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o trace -- $B \
  > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -20 "$OUT/tl.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/tl" > "$OUT/tl_timeline.txt"; cat "$OUT/tl_timeline.txt"
echo "== done"
