#!/bin/bash
# Run-length band planning (plan_bands_t accumulates a column's points in registers): the band GPU
# tests, then the band workloads at the default merge setting.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03pl}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "band or cilia" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for w in "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5" "K5 --nx 1024 --filament-offset 0.5 --rccl-self" "K3" "K5"; do
  tag=$(echo "$w" | tr -d ' -')
  timeout -k 10 120 $B --workload $w > "$OUT/${tag}.json" 2> "$OUT/${tag}.err" || { tail -5 "$OUT/${tag}.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/${tag}.json" "$w"
done
echo "== done"
