# K5 (f32 IB band cycle, depth 7): the band cycle's deep sweep build (experiment switch IBLB_XP_BANDVAR)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k5v
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --workload K5 --steps 420 --warmup 42"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'), d.get('ib_band'))" "$2" "$1"; }
for rep in 1 2; do
  timeout -k 10 200 $B > "$OUT/a.json" 2> "$OUT/err" && one "default (scalar VS2)" "$OUT/a.json" || exit 1
  IBLB_XP_BANDVAR=11 timeout -k 10 200 $B > "$OUT/a.json" 2> "$OUT/err" && one "packed split" "$OUT/a.json" || exit 1
  IBLB_XP_BANDVAR=9 timeout -k 10 200 $B > "$OUT/a.json" 2> "$OUT/err" && one "packed no split" "$OUT/a.json" || exit 1
  IBLB_DEEP_VS=1 timeout -k 10 200 $B > "$OUT/a.json" 2> "$OUT/err" && one "scalar VS1" "$OUT/a.json" || exit 1
  IBLB_BAND_CUS=32 IBLB_XP_BANDVAR=11 timeout -k 10 200 $B > "$OUT/a.json" 2> "$OUT/err" && one "packed split, chain on 32 CUs" "$OUT/a.json" || exit 1
done
