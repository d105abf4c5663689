#!/bin/bash
# Timing events of the IB workloads: system-scope fence vs device scope vs no events.
set -eo pipefail
export TMPDIR=/tmp
T=${ROUND_TAG:-r01x}
OUT=gpurun_out/$T
mkdir -p "$OUT"
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['launch_ms'], d['ib_ms_per_step'])" "$2" "$1"; }
for w in K3 K5 M; do
  for cfg in "IBLB_PROF_EVENT_FENCE=1" "IBLB_PROF_EVENT_FENCE=0"; do
    tag=$(echo "$cfg" | tr '= ' '_-')
    env $cfg timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > "$OUT/${w}_${tag}.json" 2> "$OUT/${w}_${tag}.err" \
      || { tail -20 "$OUT/${w}_${tag}.err"; exit 1; }
    row "$w $cfg" "$OUT/${w}_${tag}.json"
  done
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-profile-events > "$OUT/${w}_noev.json" 2> "$OUT/${w}_noev.err" \
    || { tail -20 "$OUT/${w}_noev.err"; exit 1; }
  row "$w no events" "$OUT/${w}_noev.json"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -p no:cacheprovider --timeout 250 \
  --timeout-method thread -k "k3 or filament or timing or profil" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
echo "== done"
