#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root):
#   parity tests, smoke, the default bench line, a rocprofv3 kernel-trace summary, HBM PMC
#   counters, an f32 bench line, and a 2-rank RCCL slab probe on the one GPU (last).
# Every GPU step has its own time limit; a crash or time-out ends the script.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}
mkdir -p "$OUT"
# pytest exit 1 = assertion failures (keep going to collect the bench); anything else
# (abort, segfault, time limit) ends the script before more GPU work.
rc=0; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "passed|failed|Error" "$OUT/pytest_gpu.log" | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
cat "$OUT/prof_bench.json"
# HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot limits), short runs
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_fetch.err" \
  || { tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile-events > /dev/null 2> "$OUT/pmc_write.err" \
  || { tail -20 "$OUT/pmc_write.err"; exit 1; }
python scripts/pmc_summary.py f64_4096x4096_n1 "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json"
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err" \
  || { tail -20 "$OUT/bench_f32.err"; exit 1; }
cat "$OUT/bench_f32.json"
# RCCL slab path with 2 ranks sharing the one GPU (may be refused by RCCL: informational)
rc=0; timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --same-device > "$OUT/rccl2.json" 2> "$OUT/rccl2.err" || rc=$?
echo "rccl2 rc=$rc"; cat "$OUT/rccl2.json"; tail -5 "$OUT/rccl2.err"
echo "== done"
