#!/bin/bash
# Where the merged band launches' time goes on the K5-width slab (self ring): kernel timelines with the
# timing probes IBLB_PROBE_LEVEL 0 (none), 3 (point groups end after their region), 4 (before their
# spread), 1 (no point groups), 5 (spread with plain stores), 6 (spread without chunk flags) -- WRONG results, timing only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05probe}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0 --rccl-self"
for p in ${PROBES:-0 3 4 1}; do
  IBLB_PROBE_LEVEL=$p timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$p" -o trace -- $B \
    > "$OUT/p$p.json" 2> "$OUT/p$p.err" || { tail -20 "$OUT/p$p.err"; exit 1; }
  python3 scripts/band_timeline.py "$OUT/p$p" > "$OUT/p${p}_timeline.txt"; echo "== probe $p"; head -2 "$OUT/p${p}_timeline.txt"
done
echo "== done"
