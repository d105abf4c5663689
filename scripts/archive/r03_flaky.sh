#!/bin/bash
# The whole -m gpu suite twice and smoke (flakiness check of the final tree).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03fl}
mkdir -p "$OUT"
for rep in 1 2; do
  timeout -k 10 600 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > "$OUT/pytest_$rep.log" 2>&1; rc=$?
  tail -2 "$OUT/pytest_$rep.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_$rep.log" | head -20
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "pytest rc=$rc"; exit 1; }
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
