#!/bin/bash
# The whole -m gpu suite and smoke on the current tree (round 5).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05suite}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
echo "== done"
