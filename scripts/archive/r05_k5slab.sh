#!/bin/bash
# The K5-width slab (1024 x 2048 f32, filaments on the slab edges, same phase in every region) on the RCCL
# self ring: the band cycle's deep sweep variant (IBLB_BAND_DEEP_VARIANT: 1 = the default plain one-cell
# walk, 107 = the wall split + preshift of the no-IB slab sweeps) and the chain's CUs (IBLB_BAND_CUS 64 / 48 / 32).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05k5slab}
mkdir -p "$OUT"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  rr def 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_DEEP_VARIANT=107 rr v107 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_DEEP_VARIANT=75 rr v75 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_CUS=48 rr cus48 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  IBLB_BAND_CUS=32 IBLB_BAND_DEEP_VARIANT=107 rr cus32v107 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
done
echo "== done"
