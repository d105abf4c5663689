#!/bin/bash
# (IBLB_BND_VS and the two-wave f64 variant were temporary experiment hooks, removed after these runs: profiles/r03bv, r03w2)
# Group-slab boundary sweeps with two cells per lane (IBLB_BND_VS=2: 35 row chunks, one wave per
# SIMD -> 24 reserved CUs at 4096 rows instead of 32) vs one (default): slab tests, then the
# strong-scaling self rings 512 / 1024 / 2048 x 4096, alternated twice.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03bv}
mkdir -p "$OUT"
IBLB_BND_VS=2 timeout -k 10 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "rccl or slab or self_ring" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50"
for rep in 1 2; do
  for nx in 512 1024 2048; do
    for v in 1 2; do
      IBLB_BND_VS=$v timeout -k 10 200 $B --nx $nx --ny 4096 --rccl-self > "$OUT/ring_${nx}_v${v}_$rep.json" 2> "$OUT/ring_${nx}_v${v}_$rep.err" || { tail -5 "$OUT/ring_${nx}_v${v}_$rep.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), d['roofline']['launch_ms'])" "$OUT/ring_${nx}_v${v}_$rep.json" "ring $nx bnd_vs $v rep $rep"
    done
  done
done
echo "== done"
