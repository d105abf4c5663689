#!/bin/bash
# Folded-constant collide + Newton reciprocal: parity suite, then step times.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01g}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:62s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP=0;IBLB_SWEEP_DEPTH=2"
for c in "4 2 96" "5 2 96" "5 1 64" "6 2 96" "6 1 96"; do set -- $c; E="$E;IBLB_SWEEP_DEPTH=$1 IBLB_DEEP_VS=$2 IBLB_DEEP_W=$3"; done
echo "-- f64 4096^2"
timeout -k 10 500 python -u scripts/tune_fused.py --steps 120 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
E="IBLB_SWEEP=0;IBLB_SWEEP_DEPTH=2"
for c in "5 1 64" "5 2 64" "6 1 64" "6 2 96"; do set -- $c; E="$E;IBLB_SWEEP_DEPTH=$1 IBLB_DEEP_VS=$2 IBLB_DEEP_W=$3"; done
echo "-- f32 4096^2"
timeout -k 10 400 python -u scripts/tune_fused.py --precision f32 --steps 120 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
timeout -k 10 400 python bench.py > "$OUT/bench_M.json" 2> "$OUT/bench_M.err" || { tail -20 "$OUT/bench_M.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_M.json')); print('bench M', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
echo "== done"
