#!/bin/bash
# Lone-slab deep sweeps as ghost-column builds (IBLB_LONE_GHOST=1: no periodic wrap in the walk, the
# edge outputs stored again as the next launch's ghost columns): bit identity, then A/B on the N = 1 slabs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05lg}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "deep_bit_identical" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  IBLB_LONE_GHOST=0 rr g0 4096 4096 f64 || exit 1
  IBLB_LONE_GHOST=1 rr g1 4096 4096 f64 || exit 1
  IBLB_LONE_GHOST=0 rr g0 4096 4096 f32 || exit 1
  IBLB_LONE_GHOST=1 rr g1 4096 4096 f32 || exit 1
done
echo "== done"
