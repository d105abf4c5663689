#!/bin/bash
# Kernel timeline of the 512 x 4096 self-ring slab (the per-rank slab of the 8-GPU 4096^2 run):
# interior sweep, boundary sweeps, pack and RCCL kernels per cycle (rocprofv3 kernel trace).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02q}
RING=${RING---rccl-self}
mkdir -p "$OUT"
for cfg in ${CFGS:-"base:"}; do
  lab=${cfg%%:*}; ev=${cfg#*:}
  env $ev timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace ${HIPTRACE:+--hip-trace} --stats --output-format csv -d "$OUT/$lab" -o trace \
    -- python3 bench.py --nx ${NX:-512} --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events $RING \
    > "$OUT/$lab.json" 2> "$OUT/$lab.err" || { tail -20 "$OUT/$lab.err"; exit 1; }
  python3 scripts/slab_timeline.py "$OUT/$lab" | tee "$OUT/${lab}_timeline.txt"
done
