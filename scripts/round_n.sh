#!/bin/bash
# Two-iteration sweep kernel: parity first (bit-identity vs one-step launches), then the GPU
# suite, then an interleaved A/B of the sweep widths / variants against the one-step kernel.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01n}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v -p no:cacheprovider --timeout 240 \
  --timeout-method thread -k "sweep" > "$OUT/pytest_sweep.log" 2>&1 || { tail -30 "$OUT/pytest_sweep.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest_sweep.log" | tail -3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
E="IBLB_SWEEP=0"
for vs in 1 2; do for w in 16 32 64; do for v in 1 3; do
  E="$E;IBLB_SWEEP_VS=$vs IBLB_SWEEP_W=$w IBLB_SWEEP_VARIANT=$v"
done; done; done
timeout -k 10 400 python -u scripts/tune_fused.py --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
grep config "$OUT/tune_f64.log" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:55s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS eq {d['tbps_equiv_one_step']:.2f} TB/s same={d['bitwise_equal_to_first']}\")"
E="IBLB_SWEEP=0"
for vs in 2 4; do for w in 32 64; do for v in 1 3; do
  E="$E;IBLB_SWEEP_VS=$vs IBLB_SWEEP_W=$w IBLB_SWEEP_VARIANT=$v"
done; done; done
timeout -k 10 400 python -u scripts/tune_fused.py --precision f32 --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
grep config "$OUT/tune_f32.log" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:55s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS eq {d['tbps_equiv_one_step']:.2f} TB/s same={d['bitwise_equal_to_first']}\")"
