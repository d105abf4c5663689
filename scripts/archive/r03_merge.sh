#!/bin/bash
# Merged band chain (IBLB_BAND_MERGE=1: each level's launch also evaluates the next level's force):
# the band / slab / bulk GPU tests, then the band workloads merged vs chained (K5-width slab lone
# and self ring with filaments on the edge and mid-slab, K3, K5).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03mg}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "band or slab or rccl or cilia or bulk" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for w in "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5" "K5 --nx 1024 --filament-offset 0 --rccl-self" "K5 --nx 1024 --filament-offset 0.5 --rccl-self" "K3" "K5"; do
  tag=$(echo "$w" | tr -d ' -')
  for m in 1 2 0; do
    IBLB_BAND_MERGE=$m timeout -k 10 120 $B --workload $w > "$OUT/${tag}_m$m.json" 2> "$OUT/${tag}_m$m.err" || { tail -5 "$OUT/${tag}_m$m.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/${tag}_m$m.json" "merge=$m $w"
  done
done
echo "== done"
