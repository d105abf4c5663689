#!/bin/bash
# The persistent band chain (IBLB_BAND_PERSIST=1): its GPU tests, then the K5-width slab (1024 x 2048 f32,
# filaments on the slab edges) lone and on the RCCL self ring, default vs persistent, two passes
# (ring_reps: 7 regions, the same filament phase in each), then a kernel timeline of the persistent ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05persist}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    -k "persist or merged_equals_chained or band_par" > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "passed|failed" "$OUT/pytest.log" | tail -3; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
  [ $rc -eq 0 ] || exit 1
}
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  IBLB_BAND_PERSIST=0 rr ring 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_PERSIST=1 rr ring_p 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_PERSIST=0 rr lone 1024 2048 f32 --k5 0 --same-phase || exit 1
  IBLB_BAND_PERSIST=1 rr lone_p 1024 2048 f32 --k5 0 --same-phase || exit 1
done
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0 --rccl-self"
IBLB_BAND_PERSIST=1 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ring_p" -o trace -- $B \
  > "$OUT/ring_p.json" 2> "$OUT/ring_p.err" || { tail -20 "$OUT/ring_p.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/ring_p" > "$OUT/ring_p_timeline.txt"; head -3 "$OUT/ring_p_timeline.txt"
echo "== done"
