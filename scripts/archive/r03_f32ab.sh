#!/bin/bash
# f32 deep sweep A/B: M f32 with the product library and kernel-build variants (lib/variants).
set -o pipefail
OUT=gpurun_out/${TAG:-r03f32}
mkdir -p "$OUT"
for v in ${VARIANTS:-base w3 nw3}; do
  lib=""; [ "$v" != base ] && lib="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_$v.so"
  for e in ${ENVS:-none}; do
    ev=""; [ "$e" != none ] && ev="$e"
    env $lib $ev timeout -k 10 120 python3 bench.py --no-cpu-baseline --precision f32 ${BENCH_ARGS} > "$OUT/M_${v}_$e.json" 2> "$OUT/M_${v}_$e.err" || { tail -5 "$OUT/M_${v}_$e.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])" "$OUT/M_${v}_$e.json" "$v $e"
  done
done
