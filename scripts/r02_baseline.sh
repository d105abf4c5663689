#!/bin/bash
# Round 2 baseline on a fresh box: host facts for the CPU baseline, the headline bench at the
# driver's flags and at a longer run (clock settled).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p "$OUT"
{ lscpu; echo; nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))';
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > "$OUT/host.txt" 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_20.json" 2> "$OUT/bench_20.err" || exit 1
timeout -k 10 200 python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline > "$OUT/bench_500.json" 2> "$OUT/bench_500.err" || exit 1
cat "$OUT"/bench_*.json | cut -c1-400
grep -E "Model name|^CPU\(s\)|Core|Socket|Thread|NUMA node\(s\)|affinity|max|OMP" "$OUT/host.txt"
