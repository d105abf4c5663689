#!/bin/bash
# Verification pass of the current tree: the -m gpu suite, smoke, the driver's default bench line
# (with the CPU baseline), then every BASELINE config at N = 1 (scripts/archive/r02_bench_all.sh).
# Every GPU step has its own time limit; a crash or time-out ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02v}
mkdir -p "$OUT"
rc=0; timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
[ -n "$SKIP_ALL" ] && exit $rc
TAG=${TAG:-r02v} bash scripts/archive/r02_bench_all.sh || exit 1
exit $rc
