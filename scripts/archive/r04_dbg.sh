#!/bin/bash
# debug: the mock-RCCL slab band cycle (mode 3) that stopped answering in r04par, with progress
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04dbg
mkdir -p $OUT
for par in 0 1; do
  echo "== PAR=$par"
  IBLB_BAND_PAR=$par IBLB_OVERLAP=1 IBLB_SWEEP_DEPTH=5 RUN_GROUP_TRACE=1 timeout -k 5 90 python3 -u tests/mock_rccl/run_group.py 2 96 130 25 3 f64 1 2>&1 | tail -5
  echo "rc=$?"
done
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests -k "par_equals_serial" 2>&1 | tail -15
