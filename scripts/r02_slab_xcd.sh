#!/bin/bash
# Self-ring slab timings after dealing the interior over all eight XCDs (CU-mask probe,
# profiles/r02n_xcc_probe.txt): default vs the old seven-XCD deal, and the reserve per XCD.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02o}
mkdir -p "$OUT"
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']))" "$2" "$1"; }
run() {  # label nx env...
  local lab=$1 nx=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --nx $nx --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events --rccl-self \
    > "$OUT/$lab.json" 2> "$OUT/$lab.err" || { tail -5 "$OUT/$lab.err"; exit 1; }
  one "$lab" "$OUT/$lab.json"
}
timeout -k 10 120 python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events > "$OUT/plain_4096.json" 2>/dev/null && one "plain 4096" "$OUT/plain_4096.json" || exit 1
for nx in 2048 1024 512; do
  run "ring_${nx}_x8" $nx IBLB_DEEP_XCDS=0 || exit 1
  run "ring_${nx}_x7" $nx IBLB_DEEP_XCDS=7 || exit 1
done
for r in 16 24 40 48; do run "ring_512_r$r" 512 IBLB_RESERVE_CUS=$r || exit 1; done
