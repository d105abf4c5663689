#!/bin/bash
# The multi-GPU rehearsal slabs (scripts/ring_reps.py, 7 regions in one process each): N = 1 (4096^2 f64),
# the 512-column f64 slab lone and on the RCCL self ring, the K5-width f32 slab with edge filaments,
# lone and ring, and without IB.  ARGS_EXTRA (env) goes to every run; OUT under gpurun_out/$TAG.
set -o pipefail
OUT=gpurun_out/${TAG:-rings}
mkdir -p "$OUT"
LIST=${LIST:-"4096 4096 f64|512 4096 f64|512 4096 f64 --ring|1024 2048 f32 --ring|1024 2048 f32 --k5 0|1024 2048 f32 --k5 0 --ring"}
IFS='|' read -ra RUNS <<< "$LIST"
for args in "${RUNS[@]}"; do
  timeout -k 10 150 python3 scripts/ring_reps.py $args $ARGS_EXTRA >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
  tail -1 "$OUT/reps.jsonl"
done
echo "== done"
