# f64 at depth 7: one cell per lane with the wall split (variant 99, two waves per SIMD) vs two cells
# (variant 35, one wave): M, K2, and the 512-column self ring
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04v1k7
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for cfg in "2 35" "1 99"; do
    set -- $cfg
    IBLB_DEEP_VS=$1 IBLB_DEEP_VARIANT=$2 timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M vs $1 var $2" "$OUT/M.json" || exit 1
    IBLB_DEEP_VS=$1 IBLB_DEEP_VARIANT=$2 timeout -k 10 200 $B --workload K2 > "$OUT/M.json" 2> "$OUT/err" && one "K2 vs $1 var $2" "$OUT/M.json" || exit 1
    IBLB_SLAB_VS=$1 IBLB_DEEP_VARIANT=$2 timeout -k 10 150 python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 2 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
    echo "ring512 vs $1 var $2: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')"
  done
done
