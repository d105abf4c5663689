#!/bin/bash
# Deep sweep units built with other AMDGPU machine-scheduler strategies (scripts/build_variant.sh
# s_<strategy> with -mllvm --amdgpu-sched-strategy=<strategy>) vs the default build: M f64 / f32.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03sc}
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --steps 500 --warmup 50"
for rep in 1 2; do
  for v in default max-ilp max-memory-clause iterative-ilp; do
    env=""; [ $v != default ] && env="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_s_$v.so"
    for p in f64 f32; do
      env $env timeout -k 10 120 $B --precision $p > "$OUT/M_${p}_${v}_$rep.json" 2> "$OUT/M_${p}_${v}_$rep.err" || { tail -5 "$OUT/M_${p}_${v}_$rep.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" "$OUT/M_${p}_${v}_$rep.json" "$p $v rep $rep"
    done
  done
done
echo "== done"
