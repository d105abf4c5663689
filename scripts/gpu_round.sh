#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root):
#   parity tests, smoke, the default bench line, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ROUND_TAG:-r01}
mkdir -p "$OUT"
echo "== host: $(nproc) cpus; $(rocm-smi --showproductname 2>/dev/null | grep -m1 -i 'card series' || true)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*stats*' | head
echo "== done"
