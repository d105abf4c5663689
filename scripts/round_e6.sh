#!/bin/bash
# Deep slab cycle (K = 5, whole-XCD reservation): host + kernel timeline on the self ring.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e6}
OUT=gpurun_out/$T
mkdir -p "$OUT"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
timeout -k 10 200 python bench.py --nx 512 --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events --rccl-self \
  > "$OUT/s_512.json" 2> "$OUT/s_512.err" || { tail -20 "$OUT/s_512.err"; exit 1; }
row "self-ring 512 default" "$OUT/s_512.json"
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
echo "== done"
