#!/bin/bash
# IB configs' roofline as a measured number: K3 and K5 bench lines (deep launches timed
# by their own signals inside the timed region) and the same commands under rocprofv3 --kernel-trace --stats.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05ib}
mkdir -p "$OUT"
for w in K3 K5; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], r['launch_timing'])" "$OUT/bench_$w.json" $w
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$w" -o trace -- python3 bench.py --no-cpu-baseline --workload $w \
    > "$OUT/trace_bench_$w.json" 2> "$OUT/trace_$w.err" || { tail -20 "$OUT/trace_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'under rocprofv3', d['value'], d['ms_per_step'], r['launch_ms'])" "$OUT/trace_bench_$w.json" $w
  find "$OUT/trace_$w" -name "*kernel_stats.csv" -exec head -5 {} \;
done
echo "== done"
