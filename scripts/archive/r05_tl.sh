#!/bin/bash
# Tests TESTK, then the K5-width slab's band cycle on the self ring: ring reps (same phase) alternated with
# AB_KNOB=0 (or the environment assignment AB_ENV, e.g. IBLB_LIB=<variant>), and a kernel timeline of the default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05tl}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "${TESTK:-band or rccl or full_size or across}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in $(seq ${REPS:-2}); do
  rr dev 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  [ -n "$AB_KNOB" ] && { ( export "IBLB_${AB_KNOB}=0"; rr ab 1024 2048 f32 --k5 0 --ring --same-phase ) || exit 1; }
  [ -n "$AB_ENV" ] && { ( export "$AB_ENV"; rr ab 1024 2048 f32 --k5 0 --ring --same-phase ) || exit 1; }
done
rr lone 1024 2048 f32 --k5 0 --same-phase || exit 1
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0 --rccl-self"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o trace -- $B \
  > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -20 "$OUT/tl.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/tl" > "$OUT/tl_timeline.txt"; head -2 "$OUT/tl_timeline.txt"
echo "== done"
