#!/bin/bash
# Timeline of the default deep slab cycle (self ring 512 x 4096) and the plain slab.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01i2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tlplain" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events \
  > /dev/null 2> "$OUT/tlplain.err" || { tail -20 "$OUT/tlplain.err"; exit 1; }
echo "== done"
