#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace): the 512 x 4096 strong-scaling slab on the RCCL self
# ring and alone (scripts/slab_timeline.py), and the K5-width slab (1024 x 2048 f32, 8 moving
# filaments) with the filaments mid-slab and on the slab edge (scripts/band_timeline.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03t}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events"
run() {  # name, timeline script, bench args...
  local n=$1 tl=$2; shift 2
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o trace -- $B "$@" \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n"; python3 scripts/$tl "$OUT/$n" | tee "$OUT/${n}_timeline.txt"
}
run ring512 slab_timeline.py --nx 512 --ny 4096 --steps 400 --warmup 40 --rccl-self || exit 1
run plain512 slab_timeline.py --nx 512 --ny 4096 --steps 400 --warmup 40 || exit 1
run k5slab_edge band_timeline.py --workload K5 --nx 1024 --steps 300 --warmup 30 --filament-offset 0 || exit 1
run k5slab_mid band_timeline.py --workload K5 --nx 1024 --steps 300 --warmup 30 --filament-offset 0.5 || exit 1
