#!/bin/bash
# K5-width slab (1024 x 2048 f32, 8 filaments on the slab edges) repeatability: 7 timed regions that
# follow the beat vs 7 regions with the same points (--same-phase), lone and on the RCCL self ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04ph}
mkdir -p "$OUT"
for args in "--k5 0" "--k5 0 --same-phase" "--k5 0 --ring" "--k5 0 --ring --same-phase"; do
  timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 $args >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
  tail -1 "$OUT/reps.jsonl"
done
