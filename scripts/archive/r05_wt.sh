#!/bin/bash
# Write-through stores in a slab's interior sweep (IBLB_INTERIOR_VARIANT: f64 163 | 256 = 419, f32 107 | 256 = 363):
# kernel timelines of the 512-column f64 self ring with and without, then ring_reps A/B (two passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05wt}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-profile-events"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o trace -- $B "$@" \
    > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; return 1; }
  echo "== $n"; python3 scripts/slab_timeline.py "$OUT/$n" | tee "$OUT/${n}_timeline.txt"
}
run ring512 --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
IBLB_INTERIOR_VARIANT=419 run ring512_wt --nx 512 --ny 4096 --steps 420 --warmup 42 --rccl-self || exit 1
rr() {  # tag, variant env, ring_reps args
  local t=$1 v=$2; shift 2
  IBLB_INTERIOR_VARIANT=$v timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  rr def64 -1 512 4096 f64 --ring || exit 1
  rr wt64 419 512 4096 f64 --ring || exit 1
  rr def32 -1 1024 2048 f32 --ring || exit 1
  rr wt32 363 1024 2048 f32 --ring || exit 1
done
rr n1 -1 4096 4096 f64 || exit 1
echo "== done"
