#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01j}
OUT=gpurun_out/$T
mkdir -p "$OUT"
rc=0; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "rccl or self_ring or app or checkpoint or local" > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|^FAILED|^ERROR" "$OUT/pytest_gpu.log" | tail -30
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
ROUND_TAG=$T bash scripts/gap_probe.sh
