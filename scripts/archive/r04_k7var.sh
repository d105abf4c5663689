# f64 deep variants at depth 7: 35 (default) vs 3 (split without the preshift) vs 1 (no split)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k7v
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in 35 3 1; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M f64 K7 variant $v" "$OUT/M.json" || exit 1
  done
done
