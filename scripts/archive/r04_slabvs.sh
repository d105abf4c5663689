# group slabs' deep sweeps: one cell per lane (round-1 default) vs two with the f64 wall split +
# preshift (variant 35) and the f32 packed split (11); self-ring rehearsals alternated on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04svs
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for vs in 1 2; do
    IBLB_SLAB_VS=$vs timeout -k 10 200 $B --steps 500 --rccl-self > "$OUT/Mr_vs${vs}_$rep.json" 2> "$OUT/Mr_vs${vs}_$rep.err" && one "M f64 ring slab_vs $vs" "$OUT/Mr_vs${vs}_$rep.json" || exit 1
    IBLB_SLAB_VS=$vs timeout -k 10 200 $B --steps 500 --rccl-self --precision f32 > "$OUT/Mr32_vs${vs}_$rep.json" 2> "$OUT/Mr32_vs${vs}_$rep.err" && one "M f32 ring slab_vs $vs" "$OUT/Mr32_vs${vs}_$rep.json" || exit 1
    IBLB_SLAB_VS=$vs timeout -k 10 200 $B --workload K5 --steps 500 --rccl-self > "$OUT/K5r_vs${vs}_$rep.json" 2> "$OUT/K5r_vs${vs}_$rep.err" && one "K5 ring slab_vs $vs" "$OUT/K5r_vs${vs}_$rep.json" || exit 1
  done
done
for args in "512 4096 f64" "1024 4096 f64" "2048 4096 f64" "1024 2048 f32" "2048 2048 f32"; do
  for vs in 1 2; do
    IBLB_SLAB_VS=$vs timeout -k 10 150 python3 scripts/ring_reps.py $args --ring --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
    echo "slab_vs $vs: $(tail -1 $OUT/reps.json)"
  done
done
