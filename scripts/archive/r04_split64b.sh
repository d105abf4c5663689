# after the f64 default moved to variant 35: the whole -m gpu suite, then K5 / M f64 and the ring
# rehearsals with 35 vs 1 alternated on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04s64b
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $OUT/pytest.log 2>&1 || { grep -E "FAILED|ERROR|Error|passed|failed" $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for v in 1 35; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --workload K5 --steps 500 > "$OUT/K5_v${v}_$rep.json" 2> "$OUT/K5_v${v}_$rep.err" && one "K5 f64 variant $v" "$OUT/K5_v${v}_$rep.json" || exit 1
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --workload K5 --steps 500 --rccl-self > "$OUT/K5r_v${v}_$rep.json" 2> "$OUT/K5r_v${v}_$rep.err" && one "K5 f64 ring variant $v" "$OUT/K5r_v${v}_$rep.json" || exit 1
    IBLB_DEEP_VARIANT=$v timeout -k 10 200 $B --steps 500 --rccl-self > "$OUT/Mr_v${v}_$rep.json" 2> "$OUT/Mr_v${v}_$rep.err" && one "M f64 ring variant $v" "$OUT/Mr_v${v}_$rep.json" || exit 1
  done
done
for args in "512 4096 f64 --ring" "1024 4096 f64 --ring"; do
  for v in 1 35; do
    IBLB_DEEP_VARIANT=$v timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 > "$OUT/reps_$v.json" 2>> "$OUT/reps.err" || exit 1
    echo "variant $v: $(tail -1 $OUT/reps_$v.json)"
  done
done
