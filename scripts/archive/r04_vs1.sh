# f64 deep sweep at one cell per lane (two waves per SIMD) vs two (one wave per SIMD); the VS 1 wall
# split (variant bit 6) with 1.5 wall sweeps per inner sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04vs1
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fused.py -m gpu \
  -k "sweep_deep_bit_identical" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for cfg in "2 35" "1 1" "1 33" "1 99" "1 97"; do
    set -- $cfg
    IBLB_DEEP_VS=$1 IBLB_DEEP_VARIANT=$2 timeout -k 10 200 $B --steps 500 > "$OUT/M.json" 2> "$OUT/err" && one "M f64 vs $1 variant $2" "$OUT/M.json" || exit 1
  done
done
for cfg in "2 35" "1 99"; do
  set -- $cfg
  IBLB_SLAB_VS=$1 IBLB_DEEP_VARIANT=$2 timeout -k 10 150 python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
  echo "ring 512 slab_vs $1 variant $2: $(tail -1 $OUT/reps.json | cut -c1-160)"
done
