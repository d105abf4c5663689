#!/bin/bash
# PAR on group slabs (round 4): band / slab / full-size GPU tests, then the K5-width slab (1024 x 2048
# f32, filaments on the slab edge and mid-slab, same-phase regions) on the RCCL self ring and lone, with
# IBLB_BAND_PAR=1 (auto: on for these narrow slabs) vs 0, alternated; K3 / K5 at N = 1 (auto: off).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04par2}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests \
    -k "${TESTK:-band or slab or full_size or rccl or moving or k5 or k3}" > "$OUT/pytest.log" 2>&1; rc=$?
  grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -E "^FAILED|Timeout" "$OUT/pytest.log" | head
  [ $rc -ne 0 ] && exit 1
fi
for rep in 1 2; do
  for case in "--k5 0 --ring" "--k5 0.5 --ring" "--k5 0"; do
    for par in 1 0; do
      IBLB_BAND_PAR=$par timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 $case --same-phase --reps 5 > "$OUT/tmp.json" 2>> "$OUT/reps.err" || exit 1
      echo "slab $case PAR=$par $(tail -1 $OUT/tmp.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"], d["band_cycles"])')" | tee -a "$OUT/summary.txt"
      tail -1 "$OUT/tmp.json" >> "$OUT/reps.jsonl"
    done
  done
done
B="python3 bench.py --no-cpu-baseline"
for w in K3 K5; do
  timeout -k 10 200 $B --workload $w --steps 300 --warmup 30 > "$OUT/$w.json" 2> "$OUT/$w.err" || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config'].get('band_par_cycles'))" "$OUT/$w.json" $w
done
echo "== done"
