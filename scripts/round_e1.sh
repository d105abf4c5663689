#!/bin/bash
# Deep sweeps as the default (K = 5): the whole GPU suite (deep slab path on mock ranks and the
# self ring included), then the self-ring slab probe over depth and reserved CUs.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e1}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 4096 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
done
for nx in 1024 512; do
  for cfg in "IBLB_SWEEP_DEPTH=2" "IBLB_SWEEP_DEPTH=5" "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=16" "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=24" \
             "IBLB_SWEEP_DEPTH=4 IBLB_RESERVE_CUS=16" "IBLB_SWEEP_DEPTH=3 IBLB_RESERVE_CUS=16" "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=16 IBLB_DEEP_VS=1"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
echo "== done"
