#!/bin/bash
# The fused band kernel (one launch per band cycle): band / slab / moving-point tests, then K3 / K5
# benches fused vs the 2K-launch chain, then the K5-width slab (1024 x 2048 f32) lone and on the
# RCCL self ring, with and without IB.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ac}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "${KEXPR:-band or moving or schedule or k3 or k5 or self_ring or rccl}" \
  > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
[ $rc -eq 0 ] || exit $rc
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('ib_band'))" "$2" "$1"; }
for w in K3 K5; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w --steps 500 --warmup 50 > "$OUT/$w.json" 2> "$OUT/$w.err" && one "$w fused" "$OUT/$w.json" || exit 1
  IBLB_BAND_FUSED=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w --steps 500 --warmup 50 > "$OUT/${w}_chain.json" 2> "$OUT/${w}_chain.err" && one "$w chain" "$OUT/${w}_chain.json" || exit 1
done
B="python3 bench.py --nx 1024 --ny 2048 --precision f32 --steps 300 --warmup 30 --no-cpu-baseline"
timeout -k 10 120 $B > "$OUT/plain_noib.json" 2>"$OUT/plain_noib.err" && one "plain no-IB" "$OUT/plain_noib.json" || exit 1
timeout -k 10 120 $B --workload K5 > "$OUT/plain_ib.json" 2>"$OUT/plain_ib.err" && one "plain IB" "$OUT/plain_ib.json" || exit 1
timeout -k 10 120 $B --rccl-self > "$OUT/ring_noib.json" 2>"$OUT/ring_noib.err" && one "ring no-IB" "$OUT/ring_noib.json" || exit 1
timeout -k 10 120 $B --rccl-self --workload K5 > "$OUT/ring_ib.json" 2>"$OUT/ring_ib.err" && one "ring IB" "$OUT/ring_ib.json" || exit 1
IBLB_BAND_FUSED=0 timeout -k 10 120 $B --rccl-self --workload K5 > "$OUT/ring_ib_chain.json" 2>"$OUT/ring_ib_chain.err" && one "ring IB chain" "$OUT/ring_ib_chain.json" || exit 1
