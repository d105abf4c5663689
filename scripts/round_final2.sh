#!/bin/bash
# Round evidence for the deep-sweep default (K = 5): GPU suite, smoke, bench lines (M f64 / f32,
# K2..K5), rocprofv3 kernel stats of the headline command, HBM PMC passes of the deep kernel,
# self-ring slab probe.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01fin2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench_M.json" 2> "$OUT/bench_M.err" || { tail -20 "$OUT/bench_M.err"; exit 1; }
cat "$OUT/bench_M.json"
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > "$OUT/bench_M_f32.json" 2> "$OUT/bench_M_f32.err" \
  || { tail -20 "$OUT/bench_M_f32.err"; exit 1; }
for w in K2 K3 K4 K5; do
  timeout -k 10 400 python bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { tail -20 "$OUT/bench_$w.err"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
for prec in f64 f32; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_$prec.err" \
    || { tail -20 "$OUT/pmc_fetch_$prec.err"; exit 1; }
  timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write_$prec.err" \
    || { tail -20 "$OUT/pmc_write_$prec.err"; exit 1; }
done
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_valu_f64" -o pmc \
  -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_valu_f64.err" \
  || { tail -20 "$OUT/pmc_valu_f64.err"; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_valu_f32" -o pmc \
  -- python bench.py --precision f32 --steps 50 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_valu_f32.err" \
  || { tail -20 "$OUT/pmc_valu_f32.err"; exit 1; }
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 2048 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    --rccl-self > "$OUT/s_${nx}.json" 2> "$OUT/s_${nx}.err" || { tail -20 "$OUT/s_${nx}.err"; exit 1; }
  row "self-ring $nx" "$OUT/s_${nx}.json"
done
echo "== done"
