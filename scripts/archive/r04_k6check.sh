# depth 6 default with the K / K-1 mix: the whole -m gpu suite, then M at 20 / 480 / 500 steps and
# the 512-column self ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k6c
mkdir -p $OUT
rc=0; timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['ms_per_step'], round(d['value']), r.get('launch_ms'), r.get('frac'), r.get('kernel','')[:24])" "$2" "$1"; }
for s in 20 480 500; do
  timeout -k 10 200 $B --steps $s > "$OUT/M_$s.json" 2> "$OUT/err" && one "M f64 $s steps" "$OUT/M_$s.json" || exit 1
done
timeout -k 10 200 $B --steps 20 --precision f32 > "$OUT/Mf32_20.json" 2> "$OUT/err" && one "M f32 20 steps" "$OUT/Mf32_20.json" || exit 1
timeout -k 10 150 python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" && tail -1 "$OUT/reps.json" | cut -c1-200
