#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02g}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bulk.py tests/test_gpu_fused.py -k "moving or schedule or k3 or k5 or band or stream or checkpoint" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for w in K3 K5; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --workload $w --steps 500 --warmup 50 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d.get('ib_band'))"
done
