# K5-width slab (1024 x 2048 f32, edge filaments, same phase) at depth 7: band chain knobs, lone and
# on the self ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04sk
mkdir -p $OUT
run() { local tag="$1"; shift; env "$@" timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 --k5 0 --same-phase --reps 3 $RING > "$OUT/r.json" 2>> "$OUT/err" || exit 1; echo "$tag $RING: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"], d["band_cycles"], d["band_merged_cycles"])')"; }
for RING in "" "--ring"; do
  run default IBLB_X=0
  run "chained" IBLB_BAND_MERGE=0
  run "cus64" IBLB_BAND_CUS=64
  run "cus-2" IBLB_BAND_CUS=-2
  run "par0" IBLB_BAND_PAR=0
  run "par2" IBLB_BAND_PAR=2
  run "depth6" IBLB_SWEEP_DEPTH=6
  run "depth5" IBLB_SWEEP_DEPTH=5
done
