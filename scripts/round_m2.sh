#!/bin/bash
# Interior-first deep cycle as default: GPU suite and the strong-scaling slab probe.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01m2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
timeout -k 10 200 python bench.py --steps 600 --warmup 40 --no-cpu-baseline --no-profile-events > "$OUT/b_4096.json" 2> "$OUT/b_4096.err" \
  || { tail -20 "$OUT/b_4096.err"; exit 1; }
row "plain 4096" "$OUT/b_4096.json"
for nx in 2048 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 600 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 600 --warmup 40 --no-cpu-baseline --no-profile-events \
    --rccl-self > "$OUT/s_${nx}.json" 2> "$OUT/s_${nx}.err" || { tail -20 "$OUT/s_${nx}.err"; exit 1; }
  row "self-ring $nx" "$OUT/s_${nx}.json"
  IBLB_SWEEP_DEPTH=2 timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 600 --warmup 40 --no-cpu-baseline --no-profile-events \
    --rccl-self > "$OUT/s2_${nx}.json" 2> "$OUT/s2_${nx}.err" || { tail -20 "$OUT/s2_${nx}.err"; exit 1; }
  row "self-ring depth-2 $nx" "$OUT/s2_${nx}.json"
done
echo "== done"
