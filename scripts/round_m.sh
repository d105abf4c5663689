#!/bin/bash
# Re-entry check: the whole GPU suite (pipelined RCCL schedule included), smoke, the default
# bench line, then the per-rank slab probe (plain vs RCCL self ring).
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01m}
OUT=gpurun_out/$T
mkdir -p "$OUT"
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|^FAILED|^ERROR" "$OUT/pytest_gpu.log" | tail -30
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
ROUND_TAG=$T bash scripts/gap_probe.sh
