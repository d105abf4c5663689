#!/bin/bash
# M (4096^2) with the round-2 tree (exp/r02, built from commit 6ecc08a) and the current tree,
# alternating on one box (f64 and f32): deep-kernel launch time, current vs round 2.
set -o pipefail
OUT=gpurun_out/${TAG:-r03ab}
mkdir -p "$OUT"
for i in 1 2; do
  for p in f64 f32; do
    (cd exp/r02 && timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 500 --warmup 50 --precision $p) > "$OUT/r02_${p}_$i.json" 2> "$OUT/r02_${p}_$i.err" || { tail -5 "$OUT/r02_${p}_$i.err"; exit 1; }
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 500 --warmup 50 --precision $p > "$OUT/r03_${p}_$i.json" 2> "$OUT/r03_${p}_$i.err" || { tail -5 "$OUT/r03_${p}_$i.err"; exit 1; }
    for t in r02 r03; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" "$OUT/${t}_${p}_$i.json" "$t $p #$i"; done
  done
done
[ -n "$TESTS" ] && { timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu $TESTS > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }; tail -2 "$OUT/pytest.log"; }
exit 0
