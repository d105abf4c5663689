# f64 deep sweep: the moving populations of the level windows in LDS (IBLB_LDSWIN=1 build via
# IBLB_LIB: 260 instead of 398 VGPRs+AGPRs) vs the default, bit identity first, then alternated
# (historical: the IBLB_LDSWIN compile switch became variant bit 7; scripts/r04_ldswin2.sh reruns the A/B)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04lw
mkdir -p $OUT
V=cuda_iblb_11_amd/lib/variants/libiblb_ldsw.so
IBLB_LIB=$V timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "sweep_deep_bit_identical" > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
grep -q " passed" $OUT/pytest.log && ! grep -q "failed\|error" $OUT/pytest.log || exit 1
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for lib in "" $V; do
    IBLB_LIB=$lib timeout -k 10 200 $B > "$OUT/M.json" 2> "$OUT/err" && one "M f64 lib=${lib:-default}" "$OUT/M.json" || exit 1
    IBLB_LIB=$lib timeout -k 10 200 $B --workload K2 > "$OUT/M.json" 2> "$OUT/err" && one "K2 lib=${lib:-default}" "$OUT/M.json" || exit 1
    IBLB_LIB=$lib timeout -k 10 200 $B --workload K3 > "$OUT/M.json" 2> "$OUT/err" && one "K3 lib=${lib:-default}" "$OUT/M.json" || exit 1
    IBLB_LIB=$lib timeout -k 10 150 python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 3 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
    echo "ring 512 lib=${lib:-default}: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')"
  done
done
