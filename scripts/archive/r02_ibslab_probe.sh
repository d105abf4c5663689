#!/bin/bash
# K5 slab of an 8-GPU run (1024 x 2048 f32, 8 filaments that move every iteration) rehearsed on one
# GPU: lone slab, RCCL self ring without IB, self ring with IB (overlapped IB step vs sequential).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02j}
mkdir -p "$OUT"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']))" "$2" "$1"; }
B="python3 bench.py --nx 1024 --ny 2048 --precision f32 --steps 300 --warmup 30 --no-cpu-baseline --no-profile-events"
timeout -k 10 120 $B > "$OUT/plain_noib.json" 2>/dev/null && one "plain no-IB" "$OUT/plain_noib.json"
timeout -k 10 120 $B --workload K5 > "$OUT/plain_ib.json" 2>/dev/null && one "plain IB (band cycle)" "$OUT/plain_ib.json"
timeout -k 10 120 $B --rccl-self > "$OUT/ring_noib.json" 2>/dev/null && one "ring no-IB" "$OUT/ring_noib.json"
timeout -k 10 120 $B --rccl-self --workload K5 > "$OUT/ring_ib.json" 2>"$OUT/ring_ib.err" && one "ring IB overlapped" "$OUT/ring_ib.json"
IBLB_IB_OVERLAP=0 timeout -k 10 120 $B --rccl-self --workload K5 > "$OUT/ring_ib_seq.json" 2>"$OUT/ring_ib_seq.err" && one "ring IB sequential" "$OUT/ring_ib_seq.json"
