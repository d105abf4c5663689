#!/bin/bash
# Round-end evidence for the default (sweep) path: whole GPU suite, smoke, bench lines (f64
# headline, f32), rocprofv3 kernel trace + stats of the headline command, HBM PMC passes of
# the sweep kernel (f64, f32), and the strong-scaling slab probe.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01r}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err" \
  || { tail -20 "$OUT/bench_f32.err"; exit 1; }
cat "$OUT/bench_f32.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
for prec in f64 f32; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch_$prec.err" \
    || { tail -20 "$OUT/pmc_fetch_$prec.err"; exit 1; }
  timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$prec" -o pmc \
    -- python bench.py --precision $prec --steps 20 --warmup 4 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write_$prec.err" \
    || { tail -20 "$OUT/pmc_write_$prec.err"; exit 1; }
done
ROUND_TAG=$T bash scripts/gap_probe.sh
echo "== done"
