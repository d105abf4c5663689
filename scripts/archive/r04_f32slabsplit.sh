# f32 group slabs (one cell per lane) at depth 7: the wall split at one cell per lane (variant bit 6:
# 75 = 11 | 64, 107 = 75 | 32 with the preshift) vs 11 (no split at one cell per lane)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04f32ss
mkdir -p $OUT
for rep in 1 2; do
  for args in "512 4096 f32" "1024 2048 f32" "2048 2048 f32"; do
    for v in 11 75 107; do
      IBLB_DEEP_VARIANT=$v timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 2 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
      echo "$args var $v: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')"
    done
  done
done
