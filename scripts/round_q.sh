#!/bin/bash
# Sweep wave mapping (4 sweeps per workgroup, XCD-contiguous) vs linear, sweep length.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01q}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread -k "sweep" > "$OUT/pytest_sweep.log" 2>&1 || { tail -30 "$OUT/pytest_sweep.log"; exit 1; }
tail -1 "$OUT/pytest_sweep.log"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:66s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
for nx in 4096 1024 512; do
  E="IBLB_SWEEP=0"
  for w in 2 4 6 8 12; do for m in 0 1; do
    E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=$m"
  done; done
  timeout -k 10 500 python -u scripts/tune_fused.py --nx $nx --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f64_$nx.log" 2>&1 \
    || { tail -20 "$OUT/tune_f64_$nx.log"; exit 1; }
  echo "-- f64 ${nx}x4096"; fmt "$OUT/tune_f64_$nx.log"
done
E="IBLB_SWEEP=0"
for w in 4 6 8 12; do for m in 0 1; do
  E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=$m"
done; done
timeout -k 10 500 python -u scripts/tune_fused.py --precision f32 --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
echo "-- f32 4096^2"; fmt "$OUT/tune_f32.log"
