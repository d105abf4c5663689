#!/bin/bash
# A/B: planar (default) vs interleaved population layout, f64 variant 5 and f32 variant 2.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}/tune_layout
mkdir -p "$OUT"
E64="IBLB_FUSED_VARIANT=5"
for cp in 0 64 256 1024; do for pp in 0 64; do
  E64="$E64;IBLB_FUSED_VARIANT=5 IBLB_LAYOUT=1 IBLB_COL_PAD=$cp IBLB_PLANE_PAD=$pp"
done; done
timeout -k 10 600 python scripts/tune_fused.py --envs "$E64" --rounds 4 > "$OUT/f64.log" 2>&1
grep median "$OUT/f64.log"
E32="IBLB_FUSED_VARIANT=2"
for cp in 0 256 1024; do for pp in 0 128; do
  E32="$E32;IBLB_FUSED_VARIANT=2 IBLB_LAYOUT=1 IBLB_COL_PAD=$cp IBLB_PLANE_PAD=$pp"
done; done
timeout -k 10 600 python scripts/tune_fused.py --precision f32 --envs "$E32" --rounds 4 > "$OUT/f32.log" 2>&1
grep median "$OUT/f32.log"
