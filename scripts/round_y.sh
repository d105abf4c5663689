#!/bin/bash
# HIP runtime dispatch settings on the self-ring slab schedule (512 and 1024 columns).
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01y}
OUT=gpurun_out/$T
mkdir -p "$OUT"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 512 1024; do
  for cfg in "IBLB_OVERLAP=1" "AMD_DIRECT_DISPATCH=0" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "IBLB_RESERVE_CUS=12"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
AMD_DIRECT_DISPATCH=0 timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
  -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
echo "== done"
