#!/bin/bash
# Sweep tuning: cells per lane, prefetch, sweep length at 4096^2 and at the 8-rank slab width
# (512 x 4096); then the rocprofv3 kernel trace and HBM PMC counters of the default bench.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01p}
OUT=gpurun_out/$T
mkdir -p "$OUT"
fmt() { grep config "$1" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(f\"{d['config']:55s} {d['median_ms_per_iter']:.4f} ms/it {d['mlups']:9.0f} MLUPS same={d['bitwise_equal_to_first']}\")"; }
E="IBLB_SWEEP=0"
for vs in 1 2; do for w in 8 12 16 24; do for v in 1 9; do
  E="$E;IBLB_SWEEP_VS=$vs IBLB_SWEEP_W=$w IBLB_SWEEP_VARIANT=$v"
done; done; done
timeout -k 10 500 python -u scripts/tune_fused.py --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f64.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64.log"; exit 1; }
fmt "$OUT/tune_f64.log"
E="IBLB_SWEEP=0"
for vs in 1 2; do for w in 2 4 8 16; do for v in 1 9; do
  E="$E;IBLB_SWEEP_VS=$vs IBLB_SWEEP_W=$w IBLB_SWEEP_VARIANT=$v"
done; done; done
timeout -k 10 500 python -u scripts/tune_fused.py --nx 512 --steps 200 --rounds 3 --envs "$E" > "$OUT/tune_f64_512.log" 2>&1 \
  || { tail -20 "$OUT/tune_f64_512.log"; exit 1; }
fmt "$OUT/tune_f64_512.log"
E="IBLB_SWEEP=0"
for vs in 2 4; do for w in 8 16 32; do for v in 1 9; do
  E="$E;IBLB_SWEEP_VS=$vs IBLB_SWEEP_W=$w IBLB_SWEEP_VARIANT=$v"
done; done; done
timeout -k 10 500 python -u scripts/tune_fused.py --precision f32 --steps 100 --rounds 3 --envs "$E" > "$OUT/tune_f32.log" 2>&1 \
  || { tail -20 "$OUT/tune_f32.log"; exit 1; }
fmt "$OUT/tune_f32.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
for prec in f64 f32; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_$prec.err" \
    || { tail -20 "$OUT/pmc_fetch_$prec.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write_$prec.err" \
    || { tail -20 "$OUT/pmc_write_$prec.err"; exit 1; }
done
echo "== done"
