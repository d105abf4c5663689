#!/bin/bash
# K5-width slab (1024 x 2048 f32, filaments on the slab edge), RCCL self ring and lone, same-phase regions:
# the band chain's CUs (IBLB_BAND_CUS: 32 = one XCD's worth, the slab default; 64; 96; 0 = one stream)
# and the chain flavour (IBLB_BAND_MERGE 0 / default).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04bc}
mkdir -p "$OUT"
for mode in ${RINGS:-ring lone}; do
  ring=""; [ "$mode" = ring ] && ring="--ring"
  for env in ${ENVS:-IBLB_BAND_CUS=32 IBLB_BAND_CUS=64 IBLB_BAND_CUS=96 IBLB_BAND_CUS=16 IBLB_BAND_MERGE=0 IBLB_BAND_CUS=0}; do
    echo -n "$env $ring: "
    env $env timeout -k 10 150 python3 scripts/ring_reps.py 1024 2048 f32 --k5 0 --same-phase --reps 5 $ring > "$OUT/tmp.json" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['env']=sys.argv[2]; print(d['median'], d['spread']); open(sys.argv[3],'a').write(json.dumps(d)+'\n')" "$OUT/tmp.json" "$env" "$OUT/reps.jsonl"
  done
done
