#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace, scripts/slab_timeline.py) of the 512 x 4096 f64 slab on the
# RCCL self ring (edge flag on / off) and alone.  EXTRA: more bench.py arguments.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05tr}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o trace -- $B "$@" $EXTRA \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n"; python3 scripts/slab_timeline.py "$OUT/$n" | tee "$OUT/${n}_timeline.txt"
}
run ring512 --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
IBLB_EDGE_FLAG=0 run ring512_noflag --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
run plain512 --nx 512 --ny 4096 --steps 420 --warmup 42 || exit 1
