# the merged chain's point groups at 16 lanes per point (IBLB_LIB variant nl16) vs 32: band tests with
# the variant, then the K5-width slab (lone / ring) and K5, alternated
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04nl
mkdir -p $OUT
V=cuda_iblb_11_amd/lib/variants/libiblb_nl16.so
IBLB_LIB=$V timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_fused.py tests/test_gpu_bulk.py \
  -k "ib_band or band_cycle or moving_points" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for args in "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0 --same-phase --ring" "1024 2048 f32 --k5 0.5 --ring"; do
    for lib in "" $V; do
      IBLB_LIB=$lib timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 2 --steps 280 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
      echo "$args ${lib:+nl16}: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"])')"
    done
  done
done
B="python3 bench.py --no-cpu-baseline --workload K5 --steps 420 --warmup 42"
for lib in "" $V; do
  IBLB_LIB=$lib timeout -k 10 200 $B > "$OUT/b.json" 2> "$OUT/err" && echo "K5 ${lib:+nl16} $(python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(d['value'])")" || exit 1
done
