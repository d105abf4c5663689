# K5 (f32, IB band cycle): the packed split deep sweep (variant 11) beside a CU-masked chain instead of
# the two-wave scalar build beside an unmasked chain (IBLB_XP_FULL: experiment switch).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k5d
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'), d.get('ib_band'))" "$2" "$1"; }
for rep in 1 2; do
  timeout -k 10 200 $B --workload K5 --steps 500 > "$OUT/K5_def_$rep.json" 2> "$OUT/err" && one "K5 default" "$OUT/K5_def_$rep.json" || exit 1
  for cus in 32 64; do
    IBLB_BAND_CUS=$cus timeout -k 10 200 $B --workload K5 --steps 500 > "$OUT/K5_m${cus}_$rep.json" 2> "$OUT/err" && one "K5 chain on $cus CUs, scalar deep" "$OUT/K5_m${cus}_$rep.json" || exit 1
    IBLB_XP_FULL=1 IBLB_BAND_CUS=$cus timeout -k 10 200 $B --workload K5 --steps 500 > "$OUT/K5_x${cus}_$rep.json" 2> "$OUT/err" && one "K5 chain on $cus CUs, packed split deep" "$OUT/K5_x${cus}_$rep.json" || exit 1
  done
done
for args in "1024 2048 f32 --k5 0" "1024 2048 f32 --k5 0 --ring" "2048 2048 f32 --k5 0"; do
  for xp in 0 1; do
    if [ $xp = 1 ]; then export IBLB_XP_FULL=1; else unset IBLB_XP_FULL; fi
    timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 5 --same-phase > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
    echo "xp $xp $args: $(tail -1 $OUT/reps.json | cut -c1-200)"
  done
done
# f64 collide: one Newton step for 1/rho and rho (1 + base) as one FMA (variant library, sweep units only)
unset IBLB_XP_FULL
for rep in 1 2; do
  for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_rcp1.so; do
    IBLB_LIB=$lib timeout -k 10 200 $B --steps 500 > "$OUT/M_$rep.json" 2> "$OUT/err" && one "M f64 lib=${lib:-default}" "$OUT/M_$rep.json" || exit 1
  done
done
