#!/bin/bash
# Host submission vs GPU on the K5-width slab's band cycle (1024 x 2048 f32, edge filaments): kernel and
# HIP runtime traces (scripts/submit_lag.py), ring and lone; the K5 N = 1 lattice for comparison.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05lag}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --steps 280 --warmup 28"
run() {  # name, extra bench args...
  local n=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/$n" -o trace -- $B "$@" \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' $OUT/$n.json)"
  python3 scripts/submit_lag.py "$OUT/$n" > "$OUT/${n}_lag.txt"; cat "$OUT/${n}_lag.txt"
}
run ring --nx 1024 --filament-offset 0 --rccl-self || exit 1
run lone --nx 1024 --filament-offset 0 || exit 1
run k5 || exit 1
echo "== done"
