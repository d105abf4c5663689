#!/bin/bash
# Round-3 verification of the current tree on one MI355X (run from the repo root through gpurun):
#   TESTS   pytest selection (default: the whole -m gpu suite)
#   BENCH   space-separated bench workloads to run after the tests (default: M; "" = none)
#   SMOKE   1 = run __graft_entry__.smoke() too
# Every GPU step has its own time limit; a crash or time-out ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03v}
mkdir -p "$OUT"
rc=0
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -q ${PYTEST_X--x} --timeout 240 --timeout-method thread -p no:cacheprovider \
  -m gpu ${TESTS:-tests} > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR|Error" "$OUT/pytest_gpu.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  grep smoke "$OUT/smoke.log"
fi
for w in ${BENCH-M}; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d.get('ib_band'))" "$OUT/bench_$w.json" $w
done
exit $rc
