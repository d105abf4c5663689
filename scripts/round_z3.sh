#!/bin/bash
# Three iterations per launch: one cell per lane (two ghost lanes per edge) against two/four.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01z3}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 250 \
  --timeout-method thread -k "three_iterations" > "$OUT/pytest_sweep3.log" 2>&1 || { tail -30 "$OUT/pytest_sweep3.log"; exit 1; }
tail -1 "$OUT/pytest_sweep3.log"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:62s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP_DEPTH=2"
for w in 16 24 32 48 64; do E="$E;IBLB_SWEEP_DEPTH=3 IBLB_SWEEP3_W=$w IBLB_SWEEP3_VS=1"; done
for w in 40 48 64 96; do E="$E;IBLB_SWEEP_DEPTH=3 IBLB_SWEEP3_W=$w IBLB_SWEEP3_VS=2"; done
echo "-- f64 4096^2"
timeout -k 10 400 python -u scripts/tune_fused.py --steps 96 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
E="IBLB_SWEEP_DEPTH=2"
for w in 16 24 32 48; do E="$E;IBLB_SWEEP_DEPTH=3 IBLB_SWEEP3_W=$w IBLB_SWEEP3_VS=1"; done
for w in 20 28 40; do E="$E;IBLB_SWEEP_DEPTH=3 IBLB_SWEEP3_W=$w IBLB_SWEEP3_VS=2"; done
echo "-- f32 4096^2"
timeout -k 10 300 python -u scripts/tune_fused.py --precision f32 --steps 96 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
echo "== done"
