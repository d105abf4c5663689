#!/bin/bash
# (IBLB_DEEP_WALLX4, IBLB_SLAB_VS and the spare-slot sizing were temporary experiment hooks, removed after these runs)
# f32 deep sweep, wall split (IBLB_DEEP_VARIANT bit 1: the three-wave build, the wall-row chunks as
# their own sweep family): bit-identity tests, then M f32 / K5 benches alternating the default
# variant (1) and the split (3) with wall sweeps per inner sweep IBLB_DEEP_WALLX4 / 4.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03sp}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py -k "sweep_deep_bit_identical" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50 --precision f32"
for rep in 1 2; do
  for cfg in "1 8" "3 4" "3 6" "3 8" "3 12"; do
    set -- $cfg
    IBLB_DEEP_VARIANT=$1 IBLB_DEEP_WALLX4=$2 timeout -k 10 120 $B > "$OUT/M_v$1_w$2_$rep.json" 2> "$OUT/M_v$1_w$2_$rep.err" \
      || { tail -5 "$OUT/M_v$1_w$2_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" \
      "$OUT/M_v$1_w$2_$rep.json" "M f32 variant $1 wallx4 $2 rep $rep"
  done
done
for v in 1 3; do
  IBLB_DEEP_VARIANT=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --workload K5 --steps 300 --warmup 30 > "$OUT/K5_v$v.json" 2> "$OUT/K5_v$v.err" \
    || { tail -5 "$OUT/K5_v$v.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d.get('ib_band'))" "$OUT/K5_v$v.json" "K5 variant $v"
done
echo "== done"
