set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04p2
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in 11 27; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --precision f32 --steps 500 > "$OUT/Mf32_v${v}_$rep.json" 2> "$OUT/Mf32_v${v}_$rep.err" && one "M f32 variant $v" "$OUT/Mf32_v${v}_$rep.json" || exit 1
  done
done
timeout -k 10 200 $B --steps 500 > "$OUT/M.json" 2> "$OUT/M.err" && one "M f64" "$OUT/M.json" || exit 1
for args in "1024 2048 f32" "1024 2048 f32 --ring" "512 4096 f64 --ring"; do
  timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || exit 1
  tail -1 "$OUT/reps.jsonl"
done
