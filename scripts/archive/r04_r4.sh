# f64 wall split: wall sweeps per inner sweep 1 (default) vs 3/4 (IBLB_LIB variant), alternated
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04r4
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2 3; do
  for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_r4w3.so; do
    IBLB_LIB=$lib timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M f64 lib=${lib:-default}" "$OUT/M.json" || exit 1
  done
done
for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_r4w3.so; do
  IBLB_LIB=$lib timeout -k 10 200 $B --steps 20 --warmup 5 > "$OUT/M.json" 2> "$OUT/err" && one "M f64 20 steps lib=${lib:-default}" "$OUT/M.json" || exit 1
done
