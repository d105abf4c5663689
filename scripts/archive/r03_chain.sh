#!/bin/bash
# Band cycles chained on their streams: band tests, then K3 / K5 / K5-width slab benches with the
# default band streams and IBLB_BAND_CUS=-2 / 0, then the K3 timeline (default streams).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ch}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider \
  -m gpu ${TESTS:-tests/test_gpu_fused.py tests/test_gpu_bulk.py tests/test_bench_dist.py} > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for cus in ${CUS:-default -2 0}; do
  env=""; [ "$cus" != default ] && env="IBLB_BAND_CUS=$cus"
  for w in "K3" "K5" "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5"; do
    tag=$(echo "$w" | tr -d ' -')
    env $env timeout -k 10 120 $B --workload $w > "$OUT/${tag}_$cus.json" 2> "$OUT/${tag}_$cus.err" || { tail -5 "$OUT/${tag}_$cus.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/${tag}_$cus.json" "cus=$cus $w"
  done
done
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/k3" -o trace -- \
  python3 bench.py --no-cpu-baseline --no-profile-events --workload K3 --steps 300 --warmup 30 > "$OUT/k3.json" 2> "$OUT/k3.err" \
  || { tail -20 "$OUT/k3.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/k3" > "$OUT/k3_timeline.txt" && head -30 "$OUT/k3_timeline.txt"
