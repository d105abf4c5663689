#!/bin/bash
# Per-rank slab of the 4096^2 strong-scaling runs (N = 1/2/4/8 -> 4096/2048/1024/512 columns):
# plain lone slab and the RCCL self-ring rehearsal, per sweep depth and cells per lane.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02i}
mkdir -p "$OUT"
one() {  # label json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']))" "$2" "$1"
}
timeout -k 10 120 python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events > "$OUT/plain_4096.json" 2>/dev/null && one "plain 4096 default" "$OUT/plain_4096.json"
for nx in ${WIDTHS:-2048 1024 512}; do
  for cfg in ${CFGS:-"D5V1" "D5V2" "D4V1" "D4V2" "D3V2"}; do
    d=${cfg:1:1}; v=${cfg:3:1}
    IBLB_SWEEP_DEPTH=$d IBLB_DEEP_SLAB_VS=$v IBLB_DEEP_VS=$v timeout -k 10 120 python3 bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 \
      --no-cpu-baseline --no-profile-events --rccl-self > "$OUT/s_${nx}_$cfg.json" 2> "$OUT/s_${nx}_$cfg.err" || { tail -5 "$OUT/s_${nx}_$cfg.err"; exit 1; }
    one "self-ring $nx $cfg" "$OUT/s_${nx}_$cfg.json"
  done
done
