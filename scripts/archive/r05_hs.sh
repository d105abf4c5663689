#!/bin/bash
# The slab cycle's two-way device handshake: the slab-path GPU tests, a kernel timeline of the 512-column
# f64 self ring, then ring_reps with IBLB_EDGE_FLAG 0 / 1 and IBLB_EDGE_TRIM 0 / 1 / 2 (two passes) and N = 1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05hs}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    -k "${TESTK:-rccl or full_size_decomposed or app}" > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "passed|failed" "$OUT/pytest.log" | tail -3; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
  [ $rc -eq 0 ] || exit 1
}
B="python3 bench.py --no-cpu-baseline --no-profile-events"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ring512" -o trace -- $B --nx 512 --ny 4096 \
  --steps 420 --warmup 42 --rccl-self > "$OUT/ring512.json" 2> "$OUT/ring512.err" || { tail -20 "$OUT/ring512.err"; exit 1; }
python3 scripts/slab_timeline.py "$OUT/ring512" | tee "$OUT/ring512_timeline.txt"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  IBLB_EDGE_FLAG=2 rr oneway 512 4096 f64 --ring || exit 1
  IBLB_EDGE_FLAG=2 IBLB_EDGE_TRIM=1 rr oneway_t1 512 4096 f64 --ring || exit 1
  IBLB_EDGE_FLAG=1 IBLB_EDGE_TRIM=1 rr hs_t1 512 4096 f64 --ring || exit 1
  IBLB_EDGE_FLAG=1 IBLB_EDGE_TRIM=2 rr hs_t2 512 4096 f64 --ring || exit 1
  IBLB_EDGE_FLAG=2 rr oneway32 1024 2048 f32 --ring || exit 1
  IBLB_EDGE_FLAG=1 IBLB_EDGE_TRIM=1 rr hs32_t1 1024 2048 f32 --ring || exit 1
  IBLB_EDGE_FLAG=1 rr hs32 1024 2048 f32 --ring || exit 1
done
IBLB_EDGE_FLAG=2 rr oneway1024 1024 4096 f64 --ring || exit 1
IBLB_EDGE_FLAG=2 rr oneway2048 2048 4096 f64 --ring || exit 1
rr n1 4096 4096 f64 || exit 1
echo "== done"
