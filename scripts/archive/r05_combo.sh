#!/bin/bash
# One call: the IB / band / slab tests, the K5-width ring (same phase) and its timeline, and K5 / K3 at N = 1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05combo}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  -k "${TESTK:-band or rccl or full_size or across or ib or ghost or point}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 --k5 0 --ring --same-phase >> "$OUT/reps_ring.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
  tail -1 "$OUT/reps_ring.jsonl"
done
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0 --rccl-self"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o trace -- $B \
  > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -20 "$OUT/tl.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/tl" > "$OUT/tl_timeline.txt"; head -30 "$OUT/tl_timeline.txt"
for w in K5 K3; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], (d.get("ib_band") or {}).get("cycle_ms"))' "$OUT/bench_$w.json" $w
done
echo "== done"
