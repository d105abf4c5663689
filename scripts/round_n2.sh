#!/bin/bash
# IB workloads on the RCCL slab path (self ring): K5 (f32, 6144 points) and K3 at full width and
# at the 8-rank slab width.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01n2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['ib_ms_per_step'], d['roofline']['launch_ms'])" "$2" "$1"; }
for w in K5 K3; do
  timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/${w}.json" 2> "$OUT/${w}.err" \
    || { tail -20 "$OUT/${w}.err"; exit 1; }
  row "plain $w" "$OUT/${w}.json"
  timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 30 --no-cpu-baseline --rccl-self > "$OUT/${w}_ring.json" 2> "$OUT/${w}_ring.err" \
    || { tail -20 "$OUT/${w}_ring.err"; exit 1; }
  row "self-ring $w" "$OUT/${w}_ring.json"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tlk5" -o trace \
  -- python bench.py --workload K5 --steps 100 --warmup 10 --no-cpu-baseline --rccl-self --no-profile-events \
  > /dev/null 2> "$OUT/tlk5.err" || { tail -20 "$OUT/tlk5.err"; exit 1; }
echo "== done"
