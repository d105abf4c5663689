#!/bin/bash
# fp64 instruction mix and FLOPs of the deep kernel (f64) and f32 VALU of the f32 deep kernel.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01k}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_flops_f64" -o pmc \
  -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_flops_f64.err" \
  || { tail -20 "$OUT/pmc_flops_f64.err"; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_flops_f32" -o pmc \
  -- python bench.py --precision f32 --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_flops_f32.err" \
  || { tail -20 "$OUT/pmc_flops_f32.err"; exit 1; }
echo "== done"
