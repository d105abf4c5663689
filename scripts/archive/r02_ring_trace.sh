#!/bin/bash
# Kernel timeline of the 512 x 4096 strong-scaling slab on the RCCL self ring and alone
# (rocprofv3 --kernel-trace, scripts/slab_timeline.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ar}
mkdir -p "$OUT"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ring" -o trace -- python3 bench.py --nx 512 --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events --rccl-self \
  > "$OUT/ring.json" 2> "$OUT/ring.err" || { tail -20 "$OUT/ring.err"; exit 1; }
python3 scripts/slab_timeline.py "$OUT/ring" | tee "$OUT/ring_timeline.txt"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/plain" -o trace -- python3 bench.py --nx 512 --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
  > "$OUT/plain.json" 2> "$OUT/plain.err" || { tail -20 "$OUT/plain.err"; exit 1; }
python3 scripts/slab_timeline.py "$OUT/plain" | tee "$OUT/plain_timeline.txt"
