#!/bin/bash
# Deep slab cycle submitted interior first (IBLB_DEEP_ORDER=1): self-ring parity and step time.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01l}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 350 \
  --timeout-method thread -k "self_ring or rccl" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 512 1024 2048; do
  for cfg in "IBLB_DEEP_ORDER=0" "IBLB_DEEP_ORDER=1"; do
    for rep in 1 2; do
      tag=$(echo "$cfg" | tr '= ' '_-')_$rep
      env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 600 --warmup 40 --no-cpu-baseline \
        --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
        || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
      row "self-ring $nx $cfg #$rep" "$OUT/s_${nx}_${tag}.json"
    done
  done
done
IBLB_DEEP_ORDER=1 timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
echo "== done"
