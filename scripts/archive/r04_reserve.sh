# CUs reserved for the slab cycle's boundary sweeps (IBLB_RESERVE_CUS; default 32 at 4096 rows)
# on the self ring with the f64 two-cell split slabs; 3 regions of 300 iterations each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04res
mkdir -p $OUT
for rep in 1 2; do
  for args in "512 4096 f64" "512 4096 f32" "1024 4096 f64"; do
    for r in 8 16 24 32 48; do
      IBLB_RESERVE_CUS=$r timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
      echo "reserve $r: $(tail -1 $OUT/reps.json)"
    done
  done
done
