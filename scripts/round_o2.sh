#!/bin/bash
# IB band cycle overlapped (band chain on reserved XCDs beside the deep sweep): tests, then K3 / K5
# at IBLB_BAND_RESERVE_CUS = 0 (sequential), 32, 64, 96.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01o3}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py -k "band or ib_ or k3_full or checkpoint" > "$OUT/pytest_band.log" 2>&1 \
  || { tail -60 "$OUT/pytest_band.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest_band.log" | tail -3
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['launch_ms'], d.get('ib_band'))" "$2" "$1"; }
for w in K3 K5; do
  for r in 0 32 64; do
    IBLB_BAND_RESERVE_CUS=$r timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/${w}_r$r.json" 2> "$OUT/${w}_r$r.err" \
      || { tail -20 "$OUT/${w}_r$r.err"; exit 1; }
    row "$w reserve=$r" "$OUT/${w}_r$r.json"
  done
done
echo "== done"
