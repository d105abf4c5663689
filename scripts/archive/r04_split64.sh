# f64 wall split (variant bit 1) and level-1 preshift (bit 5) vs the round-3 deep sweep (variant 1):
# bit identity, then M f64 per-launch time alternated on one box; K4 f64 (lone slab, deep sweep only).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04s64
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py -m gpu \
  -k "sweep_deep_bit_identical" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in 1 33 3 35; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --steps 500 > "$OUT/M_v${v}_$rep.json" 2> "$OUT/M_v${v}_$rep.err" && one "M f64 variant $v" "$OUT/M_v${v}_$rep.json" || exit 1
  done
done
for v in 1 3 35; do
  IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --workload K4 --steps 300 > "$OUT/K4_v${v}.json" 2> "$OUT/K4_v${v}.err" && one "K4 f64 variant $v" "$OUT/K4_v${v}.json" || exit 1
done
