#!/bin/bash
# What sets the ~5 us between consecutive slab interiors (512-column f64 self ring): kernel + HIP traces
# with the interior's event on its completion signal (default), as a marker (IBLB_INT_EVENT=2), and
# none (0: timing probe, wrong results), and the lone slab.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05gap}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace $TR --output-format csv -d "$OUT/$n" -o trace -- $B "$@" \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n"; python3 scripts/slab_timeline.py "$OUT/$n" | tee "$OUT/${n}_timeline.txt"
}
TR=--hip-trace run ring512_hip --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
IBLB_INT_EVENT=2 run ring512_marker --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
IBLB_INT_EVENT=0 run ring512_noev --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
IBLB_RESERVE_CUS=0 IBLB_INT_EVENT=0 run ring512_noev_nomask --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
TR=--hip-trace run plain512_hip --nx 512 --ny 4096 --steps 420 --warmup 42 || exit 1
echo "== done"
