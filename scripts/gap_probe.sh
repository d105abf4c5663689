#!/bin/bash
# Launch-gap probe: step time vs fused-kernel time at the per-rank slab sizes of the
# strong-scaling runs (4096x4096 over 1/2/4/8 ranks), with and without per-launch events.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}/gap
mkdir -p "$OUT"
for nx in 4096 1024 512; do
  for ev in "" "--no-profile-events"; do
    timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline $ev \
      > "$OUT/b_${nx}${ev}.json" 2> "$OUT/b_${nx}${ev}.err" || { tail -20 "$OUT/b_${nx}${ev}.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['launch_ms'])" \
      "$OUT/b_${nx}${ev}.json" $nx "x$ev"
  done
done
for nx in 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --rccl-self \
    > "$OUT/s_${nx}.json" 2> "$OUT/s_${nx}.err" || { tail -20 "$OUT/s_${nx}.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('self-ring', sys.argv[2], d['ms_per_step'], d['roofline']['launch_ms'])" "$OUT/s_${nx}.json" $nx
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof512s" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self > /dev/null 2> "$OUT/prof512s.err" \
  || { tail -20 "$OUT/prof512s.err"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/prof512.err" \
  || { tail -20 "$OUT/prof512.err"; exit 1; }
echo "== done"
