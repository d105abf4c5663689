#!/bin/bash
# XCD-contiguous linear sweep order (IBLB_SWEEP_MAP=2) against the linear order, over sweep
# lengths; FETCH_SIZE of the sweep kernel under both orders.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01s}
OUT=gpurun_out/$T
mkdir -p "$OUT"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:55s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP_MAP=1"
for w in 4 6 8 12 16 24; do for m in 1 2; do E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=$m"; done; done
echo "-- f64 4096^2"
timeout -k 10 400 python -u scripts/tune_fused.py --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
echo "-- f64 512x4096"
timeout -k 10 300 python -u scripts/tune_fused.py --nx 512 --steps 200 --rounds 3 --envs "$E" > "$OUT/tune_f64_512.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64_512.log"; exit 1; }
fmt "$OUT/tune_f64_512.log"
E="IBLB_SWEEP_MAP=1"
for w in 4 6 8 12 16; do for m in 1 2; do E="$E;IBLB_SWEEP_W=$w IBLB_SWEEP_MAP=$m"; done; done
echo "-- f32 4096^2"
timeout -k 10 300 python -u scripts/tune_fused.py --precision f32 --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
for cfg in "1 4" "2 4" "2 8" "2 16"; do
  set -- $cfg
  IBLB_SWEEP_MAP=$1 IBLB_SWEEP_W=$2 timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_m$1_w$2" -o pmc \
    -- python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_m$1_w$2.err" \
    || { tail -20 "$OUT/pmc_fetch_m$1_w$2.err"; exit 1; }
done
echo "== done"
