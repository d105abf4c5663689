#!/bin/bash
# Step time of the per-rank slab sizes of the strong-scaling runs (4096 x 4096 over 1/2/4/8
# ranks): the plain single slab, and the RCCL multi-slab schedule rehearsed on one GPU (the slab
# is its own neighbour, IBLB_RCCL_SELF) under the comm-stream knobs.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}/gap
mkdir -p "$OUT"
row() {  # name json
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['launch_ms'])" "$2" "$1"
}
for nx in 4096 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
done
for nx in 1024 512; do
  for cfg in "IBLB_RESERVE_CUS=8" "IBLB_RESERVE_CUS=4" "IBLB_RESERVE_CUS=16" "IBLB_RESERVE_CUS=0" "IBLB_OVERLAP=0"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof512s" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/prof512s.err" || { tail -20 "$OUT/prof512s.err"; exit 1; }
echo "== done"
