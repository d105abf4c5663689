#!/bin/bash
# Kernel timeline of the deep slab cycle on the self ring (512 x 4096, K = 5).
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for vs in 2 1; do
  IBLB_DEEP_VS=$vs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl512_vs$vs" -o trace \
    -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
    > /dev/null 2> "$OUT/tl512_vs$vs.err" || { tail -20 "$OUT/tl512_vs$vs.err"; exit 1; }
done
echo "== done"
