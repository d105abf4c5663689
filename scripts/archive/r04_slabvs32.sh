# f32 group slabs at depth 7: one vs two cells per lane (IBLB_SLAB_VS)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04sv32
mkdir -p $OUT
for rep in 1 2; do
  for args in "1024 2048 f32" "512 4096 f32" "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0.5"; do
    for vs in 1 2; do
      IBLB_SLAB_VS=$vs timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 3 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
      echo "$args vs $vs: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"])')"
    done
  done
done
