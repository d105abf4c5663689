#!/bin/bash
# rocprofv3 evidence of the headline kernel: kernel-trace stats of the driver's bench command, PMC
# HBM bytes (FETCH_SIZE / WRITE_SIZE in separate passes) and SQ VALU passes, f64 and f32.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02p}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- $B --steps 20 --warmup 5 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
for prec in f64 f32; do
  timeout -k 10 -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$prec" -o pmc \
    -- $B --precision $prec --steps 50 --warmup 5 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_$prec.err" \
    || { tail -20 "$OUT/pmc_fetch_$prec.err"; exit 1; }
  timeout -k 10 -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$prec" -o pmc \
    -- $B --precision $prec --steps 50 --warmup 5 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_write_$prec.err" \
    || { tail -20 "$OUT/pmc_write_$prec.err"; exit 1; }
done
timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_valu_f64" -o pmc \
  -- $B --steps 50 --warmup 5 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_valu_f64.err" \
  || { tail -20 "$OUT/pmc_valu_f64.err"; exit 1; }
timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_valu_f32" -o pmc \
  -- $B --precision f32 --steps 50 --warmup 5 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_valu_f32.err" \
  || { tail -20 "$OUT/pmc_valu_f32.err"; exit 1; }
find "$OUT" -name "*kernel_stats.csv" | head -3
echo done
