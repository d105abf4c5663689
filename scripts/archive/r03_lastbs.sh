#!/bin/bash
# Timing probe (wrong results): the band cycle's last level on the chain's stream right after the
# chain, beside the deep sweep, instead of behind it (variant build: scripts/variants/lastbs.patch,
# IBLB_T_LASTBS=1), vs the default, on K3, K5 and the K5-width slab.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03lb}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --steps 300 --warmup 30"
for rep in 1 2; do
  for w in "K3" "K5" "K5 --nx 1024 --filament-offset 0.5"; do
    tag=$(echo "$w" | tr -d ' -')
    for v in default lastbs; do
      env=""; [ $v = lastbs ] && env="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_lastbs.so IBLB_T_LASTBS=1"
      env $env timeout -k 10 120 $B --workload $w > "$OUT/${tag}_${v}_$rep.json" 2> "$OUT/${tag}_${v}_$rep.err" || { tail -5 "$OUT/${tag}_${v}_$rep.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'])" "$OUT/${tag}_${v}_$rep.json" "$v $w rep $rep"
    done
  done
done
echo "== done"
