#!/bin/bash
# Kernel timeline of the K3 band cycle (2048^2 f64 + 256 moving points) with the default band
# streams and with IBLB_BAND_CUS=-2 / 0 (scripts/band_timeline.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03k}
mkdir -p "$OUT"
for cus in default -2 0; do
  env=""; [ "$cus" != default ] && env="IBLB_BAND_CUS=$cus"
  env $env timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/k3_$cus" -o trace -- \
    python3 bench.py --no-cpu-baseline --no-profile-events --workload K3 --steps 300 --warmup 30 > "$OUT/k3_$cus.json" 2> "$OUT/k3_$cus.err" \
    || { tail -20 "$OUT/k3_$cus.err"; exit 1; }
  echo "== K3 band cus=$cus"; python3 scripts/band_timeline.py "$OUT/k3_$cus" | head -40 | tee "$OUT/k3_${cus}_timeline.txt"
done
