#!/bin/bash
# Alternating walk direction (IBLB_SWEEP_ALT=1) with the XCD-contiguous order (map 2): sweep
# bit-identity test, tuning over sweep lengths, FETCH_SIZE of the sweep kernel.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01t}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 250 \
  --timeout-method thread -k "sweep" > "$OUT/pytest_sweep.log" 2>&1 || { tail -30 "$OUT/pytest_sweep.log"; exit 1; }
tail -1 "$OUT/pytest_sweep.log"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:55s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP_MAP=1"
for w in 4 6 8 12 16 32; do for al in 0 1; do E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=2 IBLB_SWEEP_ALT=$al"; done; done
echo "-- f64 4096^2"
timeout -k 10 400 python -u scripts/tune_fused.py --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
echo "-- f64 512x4096"
timeout -k 10 300 python -u scripts/tune_fused.py --nx 512 --steps 200 --rounds 3 --envs "$E" > "$OUT/tune_f64_512.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64_512.log"; exit 1; }
fmt "$OUT/tune_f64_512.log"
E="IBLB_SWEEP_MAP=1"
for w in 4 6 8 12 16; do for al in 0 1; do E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=2 IBLB_SWEEP_ALT=$al"; done; done
echo "-- f32 4096^2"
timeout -k 10 300 python -u scripts/tune_fused.py --precision f32 --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
for cfg in "2 4 1" "2 8 1" "2 16 1"; do
  set -- $cfg
  IBLB_SWEEP_MAP=$1 IBLB_SWEEP_W=$2 IBLB_SWEEP_ALT=$3 timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc_fetch_m$1_w$2_a$3" -o pmc \
    -- python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_m$1_w$2_a$3.err" \
    || { tail -20 "$OUT/pmc_fetch_m$1_w$2_a$3.err"; exit 1; }
done
echo "== done"
