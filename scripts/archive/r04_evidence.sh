#!/bin/bash
# Round-4 evidence:
#   1. repeatability of the slab cycles inside one process (scripts/ring_reps.py, 7 timed regions each):
#      the 512-column strong-scaling slab of M lone / RCCL self ring, the K5-width slab (1024 x 2048 f32,
#      8 filaments) on the slab edge and mid-slab, lone / self ring;
#   2. the one-step fused_kernel on the current tree (IBLB_SWEEP=0): M f64 / f32 bench lines, rocprofv3
#      kernel stats, FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc_traffic.json keys f64/f32_4096x4096_n1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04e}
mkdir -p "$OUT"
[ -z "$SKIP_REPS" ] && {
  for args in "512 4096 f64" "512 4096 f64 --ring" "1024 2048 f32 --k5 0" "1024 2048 f32 --k5 0 --ring" \
              "1024 2048 f32 --k5 0.5" "1024 2048 f32 --k5 0.5 --ring" "1024 2048 f32" "1024 2048 f32 --ring"; do
    timeout -k 10 150 python3 scripts/ring_reps.py $args >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
    tail -1 "$OUT/reps.jsonl"
  done
}
[ -z "$SKIP_FUSED" ] && {
  B="python3 bench.py --no-cpu-baseline"
  for prec in f64 f32; do
    IBLB_SWEEP=0 timeout -k 10 200 $B --precision $prec --steps 300 > "$OUT/fused_$prec.json" 2> "$OUT/fused_$prec.err" || { tail -5 "$OUT/fused_$prec.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['launch_ms'], r['achieved'], r['frac'], r['kernel'][:40])" "$OUT/fused_$prec.json" "fused $prec"
  done
  IBLB_SWEEP=0 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_fused" -o trace \
    -- $B --steps 200 --warmup 20 --no-profile-events > /dev/null 2> "$OUT/trace_fused.err" || { tail -5 "$OUT/trace_fused.err"; exit 1; }
  find "$OUT/trace_fused" -name "*kernel_stats.csv" -exec head -3 {} \;
  for prec in f64 f32; do
    for c in FETCH_SIZE WRITE_SIZE; do
      IBLB_SWEEP=0 timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${c}_$prec" -o pmc \
        -- $B --precision $prec --steps 30 --warmup 5 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_${c}_$prec.err" \
        || { tail -5 "$OUT/pmc_${c}_$prec.err"; exit 1; }
    done
    python3 scripts/pmc_summary.py ${prec}_4096x4096_n1 "$OUT/pmc_FETCH_SIZE_$prec" "$OUT/pmc_WRITE_SIZE_$prec" "$OUT/pmc_traffic.json" --kernel fused_kernel
  done
  cat "$OUT/pmc_traffic.json"
}
echo "== done"
