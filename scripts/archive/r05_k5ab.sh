#!/bin/bash
# K5 / K3 at N = 1 (bench lines, events in the timed region), the default alternated with an A/B
# environment (AB_ENV, e.g. IBLB_WRAP_SPLIT=0), REPS times on one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05k5ab}
mkdir -p "$OUT"
for rep in $(seq ${REPS:-3}); do
  for w in ${WORKLOADS:-K5 K3}; do
    for v in def ab; do
      if [ $v = ab ]; then envs="$AB_ENV"; else envs=""; fi
      env $envs timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > "$OUT/${w}_${v}_$rep.json" 2> "$OUT/${w}_${v}_$rep.err" || { tail -5 "$OUT/${w}_${v}_$rep.err"; exit 1; }
      python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], (d.get("ib_band") or {}).get("cycle_ms"))' "$OUT/${w}_${v}_$rep.json" "$w $v"
    done
  done
done
echo "== done"
