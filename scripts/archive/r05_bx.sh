#!/bin/bash
# The K5-width slab's band cycle with the boundary sweeps told by the level-0 IB (device word) vs after
# the exchange's event (IBLB_EDGE_FLAG=0; AB_KNOB=WRAP_SPLIT: the image groups, IBLB_WRAP_SPLIT=0), alternated in
# one call; the band / slab tests first (TESTK).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05bx}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "${TESTK:-band or rccl or full_size}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2 3; do
  rr dev 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  ( export "IBLB_${AB_KNOB:-EDGE_FLAG}=0"; rr ev 1024 2048 f32 --k5 0 --ring --same-phase ) || exit 1
done
rr mid 1024 2048 f32 --k5 0.5 --ring --same-phase || exit 1
echo "== done"
