#!/bin/bash
# GPU test files given in $TESTS (default: the whole -m gpu suite), one pytest process.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02e}
mkdir -p "$OUT"
timeout -k 10 ${TLIM:-900} python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  ${TESTS:-tests} ${KEXPR:+-k "$KEXPR"} > "$OUT/pytest.log" 2>&1; rc=$?
tail -5 "$OUT/pytest.log"
grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head -20
exit $rc
