# depth 8 vs 7 (448 = 64 x 7 = 56 x 8 iterations)
# depth: 420 = 70 x 6 = 60 x 7), the 512-column f64 self ring and the K5-width slab ring (same phase).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k8
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py -m gpu \
  -k "sweep_deep_bit_identical and 8" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'), r.get('frac'))" "$2" "$1"; }
for rep in 1 2; do
  for k in 7 8; do
    IBLB_SWEEP_DEPTH=$k timeout -k 10 200 $B --steps 448 --warmup 56 > "$OUT/M.json" 2> "$OUT/err" && one "M f64 K $k" "$OUT/M.json" || exit 1
    IBLB_SWEEP_DEPTH=$k timeout -k 10 200 $B --steps 448 --warmup 56 --precision f32 > "$OUT/M.json" 2> "$OUT/err" && one "M f32 K $k" "$OUT/M.json" || exit 1
    IBLB_SWEEP_DEPTH=$k timeout -k 10 200 $B --workload K3 --steps 448 --warmup 56 > "$OUT/M.json" 2> "$OUT/err" && one "K3 K $k" "$OUT/M.json" || exit 1
    IBLB_SWEEP_DEPTH=$k timeout -k 10 200 $B --workload K5 --steps 448 --warmup 56 > "$OUT/M.json" 2> "$OUT/err" && one "K5 K $k" "$OUT/M.json" || exit 1
  done
done
for args in "512 4096 f64 --ring" "1024 4096 f64 --ring" "1024 2048 f32 --k5 0 --ring --same-phase" "1024 2048 f32 --ring"; do
  for k in 7 8; do
    IBLB_SWEEP_DEPTH=$k timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 --steps 448 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
    echo "K $k $args: $(tail -1 $OUT/reps.json | cut -c1-150)"
  done
done
