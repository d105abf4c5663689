#!/bin/bash
# The band cycle's deep sweep submitted first (ctx_band.hip:band_step): the band / slab / cilia tests,
# the K5-width slab on the self ring and alone (ring_reps, same phase), kernel timeline and host lag,
# and the K3 / K5 N = 1 bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05df}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "band or rccl or full_size or cilia" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
rr() {  # tag, ring_reps args (env from the caller)
  local t=$1; shift
  timeout -k 10 150 python3 scripts/ring_reps.py "$@" >> "$OUT/reps_$t.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; return 1; }
  echo "$t $(tail -1 $OUT/reps_$t.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["median"], d["spread"])')"
}
for rep in 1 2; do
  rr ring 1024 2048 f32 --k5 0 --ring --same-phase || exit 1
  rr lone 1024 2048 f32 --k5 0 --same-phase || exit 1
done
B="python3 bench.py --no-cpu-baseline --no-profile-events --workload K5 --nx 1024 --steps 280 --warmup 28 --filament-offset 0"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o trace -- $B --rccl-self \
  > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -20 "$OUT/tl.err"; exit 1; }
python3 scripts/band_timeline.py "$OUT/tl" > "$OUT/tl_timeline.txt"; head -2 "$OUT/tl_timeline.txt"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/lag" -o trace -- $B --rccl-self \
  > "$OUT/lag.json" 2> "$OUT/lag.err" || { tail -20 "$OUT/lag.err"; exit 1; }
python3 scripts/submit_lag.py "$OUT/lag" --kernel "sweepk_kernel<float, 1, 129, 7, false" --kernel band_level > "$OUT/lag.txt"; head -6 "$OUT/lag.txt"
for w in K3 K5; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"])' "$OUT/bench_$w.json" $w
done
echo "== done"
