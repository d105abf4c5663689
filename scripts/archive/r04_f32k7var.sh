# f32 deep variants at depth 7 on M: 11 (packed split, default) / 9 (packed, no split) / 3 (scalar split, 3 waves) / 43 (packed split + preshift bit)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04f32v
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --precision f32"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in 11 9 3; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M f32 K7 variant $v" "$OUT/M.json" || exit 1
  done
done
