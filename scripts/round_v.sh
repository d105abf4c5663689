#!/bin/bash
# Interior-first submission of the slab sweep schedule (IBLB_SWEEP_ORDER=1): self-ring parity,
# step time against the current order, and a host/kernel timeline.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01v}
OUT=gpurun_out/$T
mkdir -p "$OUT"
IBLB_SWEEP_ORDER=1 IBLB_EVENT_FENCE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q \
  -p no:cacheprovider --timeout 250 --timeout-method thread -k "self_ring or rccl" > "$OUT/pytest_ring.log" 2>&1 \
  || { tail -30 "$OUT/pytest_ring.log"; exit 1; }
echo "order 1: $(tail -1 $OUT/pytest_ring.log)"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
timeout -k 10 200 python bench.py --nx 512 --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
  > "$OUT/b_512.json" 2> "$OUT/b_512.err" || { tail -20 "$OUT/b_512.err"; exit 1; }
row "plain 512" "$OUT/b_512.json"
for nx in 1024 512; do
  for cfg in "IBLB_EVENT_FENCE=1" "IBLB_EVENT_FENCE=1 IBLB_SWEEP_ORDER=1" "IBLB_EVENT_FENCE=0 IBLB_SWEEP_ORDER=1" \
             "IBLB_EVENT_FENCE=1 IBLB_SWEEP_ORDER=1 IBLB_RESERVE_CUS=4" "IBLB_EVENT_FENCE=1 IBLB_SWEEP_ORDER=1 GPU_MAX_HW_QUEUES=8"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
IBLB_EVENT_FENCE=1 IBLB_SWEEP_ORDER=1 timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
  -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
echo "== done"
