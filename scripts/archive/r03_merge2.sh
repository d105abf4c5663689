#!/bin/bash
# Merged band chain, 32 lanes per point in the next-level IB: the merged / slab band tests, then the
# K5-width slab merged (2) vs chained (0), lone and self ring, filaments on the edge and mid-slab.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03mg2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "band or slab or cilia" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for rep in 1 2; do
for w in "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5" "K5 --nx 1024 --filament-offset 0 --rccl-self" "K5 --nx 1024 --filament-offset 0.5 --rccl-self"; do
  tag=$(echo "$w" | tr -d ' -')
  for m in 2 0; do
    IBLB_BAND_MERGE=$m timeout -k 10 120 $B --workload $w > "$OUT/${tag}_m${m}_$rep.json" 2> "$OUT/${tag}_m${m}_$rep.err" || { tail -5 "$OUT/${tag}_m${m}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band']['one_step_ms_per_cycle'])" "$OUT/${tag}_m${m}_$rep.json" "merge=$m $w"
  done
done
done
echo "== done"
