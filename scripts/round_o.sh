#!/bin/bash
# Slab sweeps: RCCL-group parity (mock ranks, self ring), the whole GPU suite, the per-rank slab
# probe (plain vs self ring), and the default bench line.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01o}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "rccl or sweep" > "$OUT/pytest_slab.log" 2>&1 || { tail -40 "$OUT/pytest_slab.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest_slab.log" | tail -3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
ROUND_TAG=$T bash scripts/gap_probe.sh
