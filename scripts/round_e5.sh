#!/bin/bash
# Reserved CUs: top bits in multiples of 8 (one per XCD per 8), depth 5 vs 2.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e5}
OUT=gpurun_out/$T
mkdir -p "$OUT"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 512 1024 2048; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
  for cfg in "IBLB_SWEEP_DEPTH=5" "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=32" "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=40" \
             "IBLB_SWEEP_DEPTH=5 IBLB_RESERVE_CUS=16" "IBLB_SWEEP_DEPTH=5 IBLB_DEEP_BND_VS=1" "IBLB_SWEEP_DEPTH=5 IBLB_DEEP_VS=1" \
             "IBLB_SWEEP_DEPTH=4 IBLB_RESERVE_CUS=32" "IBLB_SWEEP_DEPTH=3 IBLB_RESERVE_CUS=32" "IBLB_SWEEP_DEPTH=2" "IBLB_SWEEP_DEPTH=2 IBLB_RESERVE_CUS=16"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
echo "== done"
