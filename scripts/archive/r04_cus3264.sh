# band chain on 32 vs 64 CUs on group slabs (self ring, depth 7), five alternations per shape
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04c36
mkdir -p $OUT
for args in "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0.5" "2048 2048 f32 --k5 0 --same-phase"; do
  line32=""; line64=""
  for rep in 1 2 3 4 5; do
    for cus in 32 64; do
      IBLB_BAND_CUS=$cus timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 2 --steps 280 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
      v=$(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')
      if [ $cus = 32 ]; then line32="$line32 $v"; else line64="$line64 $v"; fi
    done
  done
  echo "$args | 32:$line32 | 64:$line64"
done
