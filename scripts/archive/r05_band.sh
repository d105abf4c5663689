#!/bin/bash
# The K5-width slab's IB band cycle (1024 x 2048 f32, 8 filaments on the slab edges, merged chain): kernel
# timelines on the RCCL self ring and alone, and the timing probes IBLB_PROBE_LEVEL 1 (the merged launches'
# point groups skipped) / 2 (their entry waves skipped) — WRONG results, timing only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05band}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0"
run() {  # name, extra bench args...
  local n=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o trace -- $B "$@" \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"])' $OUT/$n.json)"
  python3 scripts/band_timeline.py "$OUT/$n" > "$OUT/${n}_timeline.txt"; head -2 "$OUT/${n}_timeline.txt"
}
run ring --rccl-self || exit 1
IBLB_PROBE_LEVEL=1 run ring_nopts --rccl-self || exit 1
IBLB_PROBE_LEVEL=2 run ring_noentries --rccl-self || exit 1
run lone || exit 1
echo "== done"
