# K5 / K3 at depth 7: the band chain on its own CUs (IBLB_BAND_CUS) beside the packed split deep sweep
# (f32, experiment switch IBLB_XP_BANDVAR=11); the K5-width slab lone and on the self ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k5v2
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --steps 420 --warmup 42"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for cus in 16 32 64; do
    IBLB_BAND_CUS=$cus IBLB_XP_BANDVAR=11 timeout -k 10 200 $B --workload K5 > "$OUT/a.json" 2> "$OUT/err" && one "K5 packed split, chain on $cus CUs" "$OUT/a.json" || exit 1
  done
  timeout -k 10 200 $B --workload K3 > "$OUT/a.json" 2> "$OUT/err" && one "K3 default" "$OUT/a.json" || exit 1
  IBLB_BAND_CUS=32 timeout -k 10 200 $B --workload K3 > "$OUT/a.json" 2> "$OUT/err" && one "K3 chain on 32 CUs" "$OUT/a.json" || exit 1
done
for args in "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0 --ring --same-phase" "1024 2048 f32 --k5 0.5 --ring" "2048 2048 f32 --k5 0 --ring --same-phase"; do
  for xp in 0 1; do
    if [ $xp = 1 ]; then export IBLB_XP_BANDVAR=11; else unset IBLB_XP_BANDVAR; fi
    timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
    echo "packed $xp $args: $(tail -1 $OUT/reps.json | cut -c1-170)"
  done
done
