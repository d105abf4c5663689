#!/bin/bash
# A/B of the collide-stream kernel variants and plane padding / buffer gap (one process per sweep).
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tune3
mkdir -p "$OUT"
timeout -k 10 600 python scripts/tune_fused.py --variants 5 --pads 128,256,320,384,640 --gaps 0,160,320,2048 \
  --rounds 4 > "$OUT/f64_v5.log" 2>&1
grep variant "$OUT/f64_v5.log"
timeout -k 10 600 python scripts/tune_fused.py --precision f32 --variants 2 --pads 256,512,768,1024 --gaps 0,320,4096 \
  --rounds 4 > "$OUT/f32_v2.log" 2>&1
grep variant "$OUT/f32_v2.log"
