#!/bin/bash
# Verification + measurement pass: GPU tests, smoke, bench M (+ rocprof kernel stats and HBM PMC
# counters), bench f32, the multi-slab schedule rehearsal and an f32 layout/variant sweep.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01e}
OUT=gpurun_out/$T
mkdir -p "$OUT"
rc=0; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|^FAILED|^ERROR" "$OUT/pytest_gpu.log" | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch.err" \
  || { tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write.err" \
  || { tail -20 "$OUT/pmc_write.err"; exit 1; }
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
python scripts/pmc_summary.py f64_4096x4096_n1 "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json"
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err" \
  || { tail -20 "$OUT/bench_f32.err"; exit 1; }
cat "$OUT/bench_f32.json"
ROUND_TAG=$T bash scripts/gap_probe.sh
E32="IBLB_FUSED_VARIANT=2"
for v in 0 1 2 3 4 5; do E32="$E32;IBLB_FUSED_VARIANT=$v IBLB_LAYOUT=1 IBLB_COL_PAD=0 IBLB_PLANE_PAD=0"; done
timeout -k 10 600 python scripts/tune_fused.py --precision f32 --envs "$E32" --rounds 4 > "$OUT/tune_f32.log" 2>&1
grep median "$OUT/tune_f32.log"
echo "== done"
