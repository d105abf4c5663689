#!/bin/bash
# Timing probe of the IB band chain (wrong results, timing only): the chain without its IB launches
# (variant build scripts/variants/noib, IBLB_T_NOIB=1) vs the default, on the K5-width slab (lone,
# filaments on the slab edge and mid-slab; self ring on the edge), K3 and K5; then the kernel
# timelines of scripts/r03_trace.sh.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03nb}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for w in "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5" "K5 --nx 1024 --filament-offset 0 --rccl-self" "K3" "K5"; do
  tag=$(echo "$w" | tr -d ' -')
  for v in default noib; do
    if [ $v = noib ]; then env="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_noib.so IBLB_T_NOIB=1"; else env=""; fi
    env $env timeout -k 10 120 $B --workload $w > "$OUT/${tag}_$v.json" 2> "$OUT/${tag}_$v.err" || { tail -5 "$OUT/${tag}_$v.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['ib_band'])" "$OUT/${tag}_$v.json" "$v $w"
  done
done
TAG=${TAG:-r03nb} bash scripts/r03_trace.sh
