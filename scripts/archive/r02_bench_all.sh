#!/bin/bash
# Every BASELINE config at N = 1 (bench.py JSON lines), the headline at the driver's flags too.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02f}
mkdir -p "$OUT"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail -5 "$OUT/bench_$name.err"; return 1; }; python3 -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], d.get('ib_band'))"; }
run M_20 --steps 20 --warmup 5 || exit 1
run M_500 --steps 500 --warmup 50 || exit 1
run M_f32 --steps 500 --warmup 50 --precision f32 || exit 1
run K2 --workload K2 --steps 500 --warmup 50 || exit 1
run K4 --workload K4 --steps 500 --warmup 50 || exit 1
run K3 --workload K3 --steps 500 --warmup 50 || exit 1
run K3_frozen --workload K3 --steps 500 --warmup 50 --frozen || exit 1
run K5 --workload K5 --steps 500 --warmup 50 || exit 1
run K5_frozen --workload K5 --steps 500 --warmup 50 --frozen || exit 1
