# f64 deep variant 163 (the LDS window, default) vs 35 on one box, alternated three times: M, K4 and
# the 512-column self ring
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04lw2
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2 3; do
  for v in 35 163; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M f64 variant $v" "$OUT/M.json" || exit 1
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --workload K4 > "$OUT/M.json" 2> "$OUT/err" && one "K4 variant $v" "$OUT/M.json" || exit 1
    IBLB_DEEP_VARIANT=$v timeout -k 10 150 python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 3 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
    echo "ring 512 variant $v: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')"
  done
done
