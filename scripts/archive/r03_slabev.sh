#!/bin/bash
# Deep slab cycle with completion-signal events (no marker packets on the compute stream): the slab
# and RCCL tests, then the strong-scaling slabs of the 4096^2 lattice on the RCCL self ring (and
# alone), and the 512-column ring at depth 4.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ev}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "rccl or slab or self_ring" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for nx in 512 1024 2048; do
  timeout -k 10 200 $B --nx $nx --ny 4096 --rccl-self > "$OUT/ring_$nx.json" 2> "$OUT/ring_$nx.err" \
    && one "self ring $nx x 4096" "$OUT/ring_$nx.json" || exit 1
  timeout -k 10 200 $B --nx $nx --ny 4096 > "$OUT/plain_$nx.json" 2> "$OUT/plain_$nx.err" \
    && one "plain $nx x 4096" "$OUT/plain_$nx.json" || exit 1
done
IBLB_SWEEP_DEPTH=4 timeout -k 10 200 $B --nx 512 --ny 4096 --rccl-self > "$OUT/ring_512_k4.json" 2> "$OUT/ring_512_k4.err" \
  && one "self ring 512 x 4096 K=4" "$OUT/ring_512_k4.json" || exit 1
echo "== done"
