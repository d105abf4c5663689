#!/bin/bash
# Evidence of the current tree (run from the repo root through gpurun; TAG names the run):
#   1. the whole -m gpu suite, smoke, the driver's default bench line (with the CPU baseline);
#   2. rocprofv3 kernel-trace stats of the default bench command (the dominant kernel's mean duration);
#   3. HBM traffic (FETCH_SIZE and WRITE_SIZE in separate --pmc passes) and SQ VALU passes of the
#      deep f64 / f32 launches -> profiles/pmc_traffic.json / pmc_valu.json (scripts/pmc_*.py);
#   4. every BASELINE config at N = 1 (M at the driver's 20 steps and at 420, M f32, K2, K3, K4, K5);
#   5. the multi-GPU rehearsal: the per-rank slabs of the 4096^2 strong-scaling runs (2048 / 1024 / 512
#      columns) and the K5-width slab (1024 x 2048 f32, filaments on the slab edge / mid-slab), lone
#      and on the RCCL self ring, 7 timed regions each inside one process (scripts/ring_reps.py).
# Each GPU step has its own time limit; a crash or time-out ends the script.  SKIP_TESTS, SKIP_BENCH,
# SKIP_PMC, SKIP_CONFIGS, SKIP_REPS skip a part.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  rc=0; timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
  tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
  cp gpurun_out/parity_f32.json "$OUT/" 2>/dev/null
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  grep smoke "$OUT/smoke.log"
}
[ -z "$SKIP_BENCH" ] && {
  timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
}
B="python3 bench.py --no-cpu-baseline"
[ -z "$SKIP_PMC" ] && {
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
    -- $B > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 1; }
  find "$OUT/trace" -name "*kernel_stats.csv" -exec head -4 {} \;
  # the depth-7 launches only (the default; a call's K-1 launches carry the same bytes): 70 steps =
  # ten of them, the kernel named with its template arguments (f64 variant 163 -> mode 785, f32 235 -> 593)
  for prec in f64 f32; do
    if [ $prec = f64 ]; then kn="sweepk_kernel<double, 2, 785, 7,"; else kn="sweepk_kernel<float, 2, 593, 7,"; fi
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${c}_$prec" -o pmc \
        -- $B --precision $prec --steps 70 --warmup 7 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_${c}_$prec.err" \
        || { tail -20 "$OUT/pmc_${c}_$prec.err"; exit 1; }
    done
    python3 scripts/pmc_summary.py ${prec}_4096x4096_n1_sweep7 "$OUT/pmc_FETCH_SIZE_$prec" "$OUT/pmc_WRITE_SIZE_$prec" \
      "$OUT/pmc_traffic.json" --kernel "$kn"
    fl=FP64; [ $prec = f32 ] && fl=FP32
    timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_$fl SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
      --output-format csv -d "$OUT/pmc_valu_$prec" -o pmc \
      -- $B --precision $prec --steps 70 --warmup 7 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_valu_$prec.err" \
      || { tail -20 "$OUT/pmc_valu_$prec.err"; exit 1; }
  done
  # the IB configs' deep sweeps inside the band cycle (K3 f64 variant 163 without the window -> mode 273,
  # K5 f32 235 -> 593)
  for wl in K3 K5; do
    if [ $wl = K3 ]; then kn="sweepk_kernel<double, 2, 273, 7,"; key=f64_2048x2048_n1_ib256_sweep7;
    else kn="sweepk_kernel<float, 2, 593, 7,"; key=f32_8192x2048_n1_ib6144_sweep7; fi
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${c}_$wl" -o pmc \
        -- $B --workload $wl --steps 70 --warmup 7 --prime-seconds 0.3 --no-profile-events > /dev/null 2> "$OUT/pmc_${c}_$wl.err" \
        || { tail -20 "$OUT/pmc_${c}_$wl.err"; exit 1; }
    done
    python3 scripts/pmc_summary.py $key "$OUT/pmc_FETCH_SIZE_$wl" "$OUT/pmc_WRITE_SIZE_$wl" "$OUT/pmc_traffic.json" --kernel "$kn"
  done
  cat "$OUT/pmc_traffic.json"
  echo "== pmc done"
}
[ -z "$SKIP_CONFIGS" ] && {
  run() { local name=$1; shift; timeout -k 10 300 $B "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail -5 "$OUT/bench_$name.err"; return 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], d.get('ib_band'))" "$OUT/bench_$name.json" "$name"; }
  run M_20 --steps 20 --warmup 5 || exit 1
  run M_420 --steps 420 --warmup 42 || exit 1
  run M_f32 --steps 420 --warmup 42 --precision f32 || exit 1
  run K2 --workload K2 --steps 420 --warmup 42 || exit 1
  run K4 --workload K4 --steps 420 --warmup 42 || exit 1
  run K3 --workload K3 --steps 420 --warmup 42 || exit 1
  run K5 --workload K5 --steps 420 --warmup 42 || exit 1
}
[ -z "$SKIP_REPS" ] && {
  for args in "2048 4096 f64" "2048 4096 f64 --ring" "1024 4096 f64" "1024 4096 f64 --ring" "512 4096 f64" "512 4096 f64 --ring" \
              "1024 2048 f32 --k5 0" "1024 2048 f32 --k5 0 --ring" "1024 2048 f32 --k5 0.5" "1024 2048 f32 --k5 0.5 --ring" \
              "1024 2048 f32" "1024 2048 f32 --ring"; do
    timeout -k 10 150 python3 scripts/ring_reps.py $args >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
    tail -1 "$OUT/reps.jsonl"
  done
}
echo "== done"
