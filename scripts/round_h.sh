#!/bin/bash
# Full verification + measurement pass (tests, smoke, bench M f64/f32 with rocprof kernel stats and
# HBM PMC counters, the multi-slab rehearsal, every BASELINE config).
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01h}
OUT=gpurun_out/$T
mkdir -p "$OUT"
rc=0; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|^FAILED|^ERROR" "$OUT/pytest_gpu.log" | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
for prec in f64 f32; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_$prec.err" \
    || { tail -20 "$OUT/pmc_fetch_$prec.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write_$prec.err" \
    || { tail -20 "$OUT/pmc_write_$prec.err"; exit 1; }
  python scripts/pmc_summary.py ${prec}_4096x4096_n1 "$OUT/pmc_fetch_$prec" "$OUT/pmc_write_$prec" "$OUT/pmc_traffic.json"
done
cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err" \
  || { tail -20 "$OUT/bench_f32.err"; exit 1; }
cat "$OUT/bench_f32.json"
for w in K2 K3 K4 K5; do
  timeout -k 10 400 python bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cut -c1-200 "$OUT/bench_$w.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_k3" -o trace \
  -- python bench.py --workload K3 --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2> "$OUT/prof_k3.err" \
  || { tail -20 "$OUT/prof_k3.err"; exit 1; }
ROUND_TAG=$T bash scripts/gap_probe.sh
echo "== done"
