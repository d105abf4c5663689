# band chain CUs on group slabs at depth 7 (self ring): 32 (auto here) / 64 / 96 on the K5-width slab
# (edge, same phase; mid-slab) and the 2048-column slab (N = 4 of config 5)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04sc
mkdir -p $OUT
for args in "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0.5" "2048 2048 f32 --k5 0 --same-phase" "4096 2048 f32 --k5 0 --same-phase"; do
  for cus in auto 32 64 96; do
    if [ $cus = auto ]; then unset IBLB_BAND_CUS; else export IBLB_BAND_CUS=$cus; fi
    timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 3 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
    echo "$args cus $cus: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"], d["band_cycles"], d["band_merged_cycles"])')"
  done
done
