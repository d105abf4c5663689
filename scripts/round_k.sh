#!/bin/bash
# SQ counters of the deep kernel (VALU activity and stall split) and the counter list.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01k}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 -s KILL 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -o "SQ_[A-Z0-9_]*VALU[A-Z0-9_]*\|SQ_INSTS_[A-Z0-9_]*F64[A-Z0-9_]*\|SQ_[A-Z0-9_]*FLOPS[A-Z0-9_]*" "$OUT/counters.txt" | sort -u | head -40 || true
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_sq_f64" -o pmc \
  -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_sq_f64.err" \
  || { tail -20 "$OUT/pmc_sq_f64.err"; exit 1; }
echo "== done"
