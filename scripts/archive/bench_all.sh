#!/bin/bash
# Every BASELINE.json config on one GPU (bench.py --workload), plus a kernel-trace profile of the
# IB workload K3.  Each GPU step has its own time limit; a crash or time-out ends the script.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}/bench_all
mkdir -p "$OUT"
rc=0; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|^FAILED" "$OUT/pytest_gpu.log" | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
for w in M K2 K3 K4 K5; do
  timeout -k 10 400 python bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_k3" -o trace \
  -- python bench.py --workload K3 --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2> "$OUT/prof_k3.err" \
  || { tail -20 "$OUT/prof_k3.err"; exit 1; }
cut -c1-150 "$OUT/prof_k3/trace_kernel_stats.csv" | head -12
echo "== done"
