#!/bin/bash
# Ghost-row shifts without the edge patch: GPU suite, deep tune, bench.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01j}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:62s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP_DEPTH=5;IBLB_SWEEP_DEPTH=4;IBLB_SWEEP_DEPTH=6;IBLB_SWEEP_DEPTH=5 IBLB_DEEP_W=128;IBLB_SWEEP_DEPTH=5 IBLB_DEEP_W=64"
echo "-- f64 4096^2"
timeout -k 10 500 python -u scripts/tune_fused.py --steps 120 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
echo "-- f32 4096^2"
timeout -k 10 400 python -u scripts/tune_fused.py --precision f32 --steps 120 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench_M.json" 2> "$OUT/bench_M.err" || { tail -20 "$OUT/bench_M.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_M.json')); print('bench M', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
echo "== done"
