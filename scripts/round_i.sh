#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01i
mkdir -p "$OUT"
timeout -k 10 300 python scripts/bench_dropin.py > "$OUT/dropin.log" 2> "$OUT/dropin.err" || { tail -20 "$OUT/dropin.err"; exit 1; }
cat "$OUT/dropin.log"
E=""
for v in 0 1 2 3 4 5 6 7; do E="$E;IBLB_FUSED_VARIANT=$v"; done
E="${E#;};IBLB_FUSED_VARIANT=5 IBLB_COL_PAD=0;IBLB_FUSED_VARIANT=5 IBLB_COL_PAD=128;IBLB_FUSED_VARIANT=5 IBLB_COL_PAD=192;IBLB_FUSED_VARIANT=5 IBLB_BUF_GAP=0;IBLB_FUSED_VARIANT=5 IBLB_BUF_GAP=2048"
timeout -k 10 600 python scripts/tune_fused.py --envs "$E" --rounds 4 > "$OUT/tune_f64.log" 2>&1
grep median "$OUT/tune_f64.log"
