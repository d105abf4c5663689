# f64 deep sweep depth K = 4 / 5 / 6 with the wall split (two cells per lane, variant 35; one cell per
# lane, variant 99) on M.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04dep
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'), (d['roofline'] or {}).get('frac'))" "$2" "$1"; }
for rep in 1 2; do
  for cfg in "5 2 35 f64" "6 2 35 f64" "6 1 99 f64" "4 2 35 f64" "4 1 99 f64" "5 2 11 f32" "5 1 99 f32" "6 2 11 f32" "6 1 99 f32"; do
    set -- $cfg
    IBLB_SWEEP_DEPTH=$1 IBLB_DEEP_VS=$2 IBLB_DEEP_VARIANT=$3 timeout -k 10 200 $B --precision $4 --steps 480 > "$OUT/M.json" 2> "$OUT/err" && one "M $4 K $1 vs $2 variant $3" "$OUT/M.json" || exit 1
  done
done
