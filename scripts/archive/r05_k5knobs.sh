#!/bin/bash
# K5 at N = 1: the band chain's CUs (IBLB_BAND_CUS 32 default / 40 / 48) and the merged chain
# (IBLB_BAND_MERGE=2 with MERGE=1; measured 0.65 vs 0.48 ms per cycle), alternated REPS times on one box (bench lines, events in the timed region).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05k5knobs}
mkdir -p "$OUT"
run() {  # tag, env assignments...
  local t=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --workload ${WL:-K5} --no-cpu-baseline > "$OUT/${t}_$rep.json" 2> "$OUT/${t}_$rep.err" || { tail -5 "$OUT/${t}_$rep.err"; return 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], (d.get("ib_band") or {}).get("cycle_ms"))' "$OUT/${t}_$rep.json" "$t"
}
for rep in $(seq ${REPS:-2}); do
  run def IBLB_X=0 || exit 1
  run cus40 IBLB_BAND_CUS=40 || exit 1
  run cus48 IBLB_BAND_CUS=48 || exit 1
  [ -n "$MERGE" ] && { run merge IBLB_BAND_MERGE=2 || exit 1; }
done
echo "== done"
