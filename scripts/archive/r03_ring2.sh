#!/bin/bash
# (IBLB_DEEP_WALLX4, IBLB_SLAB_VS and the spare-slot sizing were temporary experiment hooks, removed after these runs)
# (1) f32 wall split: wall sweeps per inner sweep (IBLB_DEEP_WALLX4 / 4) around the optimum;
# (2) strong-scaling slabs on the RCCL self ring: reserved CUs (default) vs none with spare wave
#     slots (IBLB_RESERVE_CUS=0), one vs two cells per lane in the slab sweeps (IBLB_SLAB_VS).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03r2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "rccl or slab or self_ring or sweep_deep" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'))" "$2" "$1"; }
for rep in 1 2; do
  for w in 8 9 10; do
    IBLB_DEEP_WALLX4=$w timeout -k 10 120 $B --precision f32 > "$OUT/M_f32_w${w}_$rep.json" 2> "$OUT/M_f32_w${w}_$rep.err" \
      && one "M f32 wallx4 $w rep $rep" "$OUT/M_f32_w${w}_$rep.json" || exit 1
  done
done
for nx in 512 1024 2048; do
  for cfg in "32 1" "0 1" "32 2" "0 2"; do
    set -- $cfg
    [ "$nx" != 512 ] && [ "$2" = 2 ] && continue
    IBLB_RESERVE_CUS=$1 IBLB_SLAB_VS=$2 timeout -k 10 200 $B --nx $nx --ny 4096 --rccl-self > "$OUT/ring_${nx}_r$1_vs$2.json" 2> "$OUT/ring_${nx}_r$1_vs$2.err" \
      && one "self ring $nx x 4096 reserve $1 slab_vs $2" "$OUT/ring_${nx}_r$1_vs$2.json" || exit 1
  done
done
echo "== done"
