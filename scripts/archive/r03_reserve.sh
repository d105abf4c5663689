#!/bin/bash
# Self-ring 512 x 4096 (the N = 8 strong-scaling slab) vs the CUs reserved for the comm stream
# (IBLB_RESERVE_CUS: exchange + boundary sweeps), and the lone slab for reference.
set -o pipefail
OUT=gpurun_out/${TAG:-r03r}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --nx 512 --ny 4096 --steps 500 --warmup 50"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
timeout -k 10 200 $B > "$OUT/plain_512.json" 2> "$OUT/plain_512.err" && one "plain 512" "$OUT/plain_512.json" || exit 1
for r in ${RESERVE:-8 16 24 32 48}; do
  IBLB_RESERVE_CUS=$r timeout -k 10 200 $B --rccl-self > "$OUT/ring_512_r$r.json" 2> "$OUT/ring_512_r$r.err" \
    && one "ring 512 reserve $r" "$OUT/ring_512_r$r.json" || exit 1
done
