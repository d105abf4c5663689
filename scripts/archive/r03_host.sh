#!/bin/bash
# Host-side cost of the band cycle: HIP call costs (scripts/bin/api_probe), and the host time in
# planning and band_step per cycle (variant build scripts/variants/hostprof) next to the GPU time,
# on the K5-width slab (filaments on the edge / mid-slab, self ring) and K5.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03h}
mkdir -p "$OUT"
timeout -k 10 60 scripts/bin/api_probe | tee "$OUT/api_probe.txt" || exit 1
B="python3 bench.py --no-cpu-baseline --no-profile-events --steps 300 --warmup 30"
for w in "K5 --nx 1024 --filament-offset 0" "K5 --nx 1024 --filament-offset 0.5" "K5 --nx 1024 --filament-offset 0 --rccl-self" "K5" "K5 --nx 1024 --filament-offset 0 --frozen"; do
  tag=$(echo "$w" | tr -d ' -')
  IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_hostprof.so timeout -k 10 120 $B --workload $w > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'])" "$OUT/$tag.json" "$w"
  grep hostprof "$OUT/$tag.err"
done
timeout -k 10 100 python3 scripts/host_probe.py 1024 2048 f32 K5 | tee "$OUT/host_probe.txt" || exit 1
