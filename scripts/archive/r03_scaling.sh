#!/bin/bash
# Multi-GPU rehearsal on one MI355X (RCCL self ring = a slab that is its own neighbour, the
# complete per-rank schedule of an N-GPU run with real RCCL): the strong-scaling slabs of the
# 4096^2 M lattice (N = 2, 4, 8 -> 2048 / 1024 / 512 columns), plain (lone slab) and self ring,
# and the K5-width slab (1024 x 2048 f32 + 8 moving filaments) with the filaments mid-slab
# (offset 0.5) and on the slab edge (offset 0, BASELINE config 5).
set -o pipefail
OUT=gpurun_out/${TAG:-r03s}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'), d.get('ib_band'))" "$2" "$1"; }
timeout -k 10 200 $B --steps 500 --warmup 50 > "$OUT/M.json" 2> "$OUT/M.err" && one "M 4096 N=1" "$OUT/M.json" || exit 1
for nx in ${WIDTHS:-2048 1024 512}; do
  timeout -k 10 200 $B --nx $nx --ny 4096 --steps 500 --warmup 50 > "$OUT/plain_$nx.json" 2> "$OUT/plain_$nx.err" \
    && one "plain $nx x 4096" "$OUT/plain_$nx.json" || exit 1
  timeout -k 10 200 $B --nx $nx --ny 4096 --steps 500 --warmup 50 --rccl-self > "$OUT/ring_$nx.json" 2> "$OUT/ring_$nx.err" \
    && one "self ring $nx x 4096" "$OUT/ring_$nx.json" || exit 1
done
for off in 0.5 0; do
  timeout -k 10 200 $B --workload K5 --nx 1024 --steps 300 --warmup 30 --filament-offset $off > "$OUT/k5slab_lone_$off.json" 2> "$OUT/k5slab_lone_$off.err" \
    && one "K5 slab lone offset $off" "$OUT/k5slab_lone_$off.json" || exit 1
  timeout -k 10 200 $B --workload K5 --nx 1024 --steps 300 --warmup 30 --filament-offset $off --rccl-self > "$OUT/k5slab_ring_$off.json" 2> "$OUT/k5slab_ring_$off.err" \
    && one "K5 slab self ring offset $off" "$OUT/k5slab_ring_$off.json" || exit 1
done
echo "== done"
