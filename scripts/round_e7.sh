#!/bin/bash
# Deep slab interior under a whole-XCD reservation: workgroup dealing over 7 XCDs vs 8, linear.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e7}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 350 \
  --timeout-method thread -k "self_ring or deep" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 512 1024 2048; do
  for cfg in "IBLB_DEEP_XCD_DEAL=1" "IBLB_DEEP_XCD_DEAL=0" "IBLB_SWEEP_MAP=1" "IBLB_SWEEP_DEPTH=4" "IBLB_DEEP_VS=1"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
echo "== done"
