#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02m}
mkdir -p "$OUT"
timeout -k 10 400 python -u scripts/tune_fused.py --precision f32 --rounds 3 --steps 100 --envs "$ENVS" > "$OUT/tune_f32.log" 2>&1 || exit 1
grep config "$OUT/tune_f32.log" | python3 -c 'import sys,json; [print(round(d["median_ms_per_iter"],5), round(d["mlups"]), d["bitwise_equal_to_first"], d["config"]) for d in map(json.loads, sys.stdin)]'
