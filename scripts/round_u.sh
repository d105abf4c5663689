#!/bin/bash
# Cross-stream event fences on the self-ring slab schedule (correctness + step time), a host/
# kernel timeline of the self ring, and the headline bench + profiles under the new sweep order.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01u}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for ef in 1 2; do
  IBLB_EVENT_FENCE=$ef timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider \
    --timeout 250 --timeout-method thread -k "self_ring" > "$OUT/pytest_ring_ef$ef.log" 2>&1 \
    || { tail -30 "$OUT/pytest_ring_ef$ef.log"; exit 1; }
  echo "event fence $ef: $(tail -1 $OUT/pytest_ring_ef$ef.log)"
done
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$2" "$1"; }
for nx in 4096 1024 512; do
  timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events \
    > "$OUT/b_${nx}.json" 2> "$OUT/b_${nx}.err" || { tail -20 "$OUT/b_${nx}.err"; exit 1; }
  row "plain $nx" "$OUT/b_${nx}.json"
done
for nx in 1024 512; do
  for cfg in "IBLB_EVENT_FENCE=0" "IBLB_EVENT_FENCE=1" "IBLB_EVENT_FENCE=2" "IBLB_EVENT_FENCE=1 IBLB_RESERVE_CUS=16" "IBLB_EVENT_FENCE=2 IBLB_RESERVE_CUS=16"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline \
      --no-profile-events --rccl-self > "$OUT/s_${nx}_${tag}.json" 2> "$OUT/s_${nx}_${tag}.err" \
      || { tail -20 "$OUT/s_${nx}_${tag}.err"; exit 1; }
    row "self-ring $nx $cfg" "$OUT/s_${nx}_${tag}.json"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/tl512" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 200 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/tl512.err" || { tail -20 "$OUT/tl512.err"; exit 1; }
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
echo "== done"
