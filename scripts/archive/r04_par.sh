#!/bin/bash
# The IB band cycle's last level beside the deep sweep (PAR, lone slab; round 4): the GPU suite,
# then K3, K5 and the K5-width lone slab with IBLB_BAND_PAR=1 (default) vs 0, alternated.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04par}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests \
    ${TESTK:+-k "$TESTK"} > "$OUT/pytest.log" 2>&1; rc=$?
  grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -E "^FAILED|Timeout" "$OUT/pytest.log" | head
  [ $rc -ne 0 ] && exit 1
fi
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d.get('ib_band') or {}).get('deep_ms_per_cycle'), d['config'].get('band_par_cycles'))" "$2" "$1"; }
for rep in 1 2; do
  for par in 1 0; do
    IBLB_BAND_PAR=$par timeout -k 10 200 $B --workload K3 --steps 500 > "$OUT/K3_p${par}_$rep.json" 2> "$OUT/K3_p${par}_$rep.err" && one "K3 PAR=$par" "$OUT/K3_p${par}_$rep.json" || exit 1
    IBLB_BAND_PAR=$par timeout -k 10 200 $B --workload K5 --steps 300 --warmup 30 > "$OUT/K5_p${par}_$rep.json" 2> "$OUT/K5_p${par}_$rep.err" && one "K5 PAR=$par" "$OUT/K5_p${par}_$rep.json" || exit 1
    IBLB_BAND_PAR=$par timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 --k5 0 --same-phase --reps 5 > "$OUT/slab_p$par.json" 2>> "$OUT/reps.err" || exit 1
    echo "K5 slab lone edge PAR=$par $(tail -1 $OUT/slab_p$par.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"])')"
  done
done
echo "== done"
