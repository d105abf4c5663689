#!/bin/bash
# Round-3 evidence of the current tree (run from the repo root through gpurun):
#   1. the whole -m gpu suite, smoke, the driver's default bench line (with the CPU baseline);
#   2. rocprofv3 kernel-trace stats of the same bench command (dominant kernel's mean duration);
#   3. HBM traffic (FETCH_SIZE and WRITE_SIZE in separate --pmc passes) and SQ VALU passes of the
#      headline f64 / f32 launches -> profiles/pmc_traffic.json / pmc_valu.json;
#   4. every BASELINE config at N = 1 (scripts/archive/r02_bench_all.sh), the strong-scaling slabs and the
#      K5-width slab on the RCCL self ring (scripts/archive/r03_scaling.sh).
# Each GPU step has its own time limit; a crash or time-out ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03z}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  rc=0; timeout -k 10 700 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
  tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
  cp gpurun_out/parity_f32.json "$OUT/" 2>/dev/null
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  grep smoke "$OUT/smoke.log"
}
[ -z "$SKIP_BENCH" ] && {
  timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
}
B="python3 bench.py --no-cpu-baseline"
[ -z "$SKIP_PMC" ] && {
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
    -- $B --steps 200 --warmup 20 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
  find "$OUT/trace" -name "*kernel_stats.csv" -exec head -4 {} \;
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
  echo "== pmc done"
}
[ -n "$SKIP_ALL" ] && exit 0
TAG=${TAG:-r03z} bash scripts/archive/r02_bench_all.sh || exit 1
TAG=${TAG:-r03z} bash scripts/archive/r03_scaling.sh || exit 1
echo "== done"
