#!/bin/bash
# IB band cycle: its GPU tests, the IB tests around it, then K3 / K5 benches (band on / off).
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01o1}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py -k "band or ib_ or k3_full" > "$OUT/pytest_band.log" 2>&1 \
  || { tail -60 "$OUT/pytest_band.log"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$OUT/pytest_band.log" | tail -20
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['ib_ms_per_step'], d['roofline']['launch_ms'], d.get('ib_band'))" "$2" "$1"; }
for w in K3 K5; do
  timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/${w}.json" 2> "$OUT/${w}.err" \
    || { tail -20 "$OUT/${w}.err"; exit 1; }
  row "band $w" "$OUT/${w}.json"
  IBLB_IB_BAND=0 timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/${w}_noband.json" 2> "$OUT/${w}_noband.err" \
    || { tail -20 "$OUT/${w}_noband.err"; exit 1; }
  row "one-step $w" "$OUT/${w}_noband.json"
done
echo "== done"
