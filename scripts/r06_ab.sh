#!/bin/bash
# Kernel-build A/B on one box (round 6): bench lines of WORKLOADS (e.g. "M M32 K5"; M32 = M in f32)
# with the in-tree libiblb.so ("def") alternated with the IBLB_LIB variants named in VARIANTS
# (cuda_iblb_11_amd/lib/variants/libiblb_<name>.so, built here by scripts/build_variant.sh) or
# NAME=VALUE environment settings (the in-tree library under them), REPS times.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ab}
mkdir -p "$OUT"
for rep in $(seq ${REPS:-3}); do
  for w in ${WORKLOADS:-M}; do
    args="--workload $w"
    [ "$w" = M32 ] && args="--workload M --precision f32"
    for v in def ${VARIANTS:-base}; do
      # a variant NAME=VALUE is the in-tree library under that environment setting
      case $v in
        def) lib="" ;;
        *=*) lib="$v" ;;
        *) lib="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_$v.so" ;;
      esac
      f="$OUT/${w}_${v//=/-}_$rep"
      env $lib $AB_ENV timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$f.json" 2> "$f.err" || { tail -5 "$f.err"; exit 1; }
      python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], (d.get("ib_band") or {}).get("cycle_ms"))' "$f.json" "$w $v"
    done
  done
done
echo "== done"
