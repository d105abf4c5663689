#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01k
mkdir -p "$OUT"
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --nx 512 --ny 4096 --steps 400 --warmup 40 --no-cpu-baseline --no-profile-events $EXTRA \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$OUT/$tag.json" "$tag $*"
}
EXTRA="" run plain IBLB_DEBUG_SYNC=0
EXTRA="" run plain_mask8 IBLB_DEBUG_CUMASK=8
EXTRA="" run plain_mask8_rec IBLB_DEBUG_CUMASK=8 IBLB_DEBUG_SYNC=1
EXTRA="--rccl-self" run ring IBLB_DEBUG_NOCOMM=0
EXTRA="--rccl-self" run ring_nocomm IBLB_DEBUG_NOCOMM=1
EXTRA="--rccl-self" run ring_nocomm_nothread IBLB_DEBUG_NOCOMM=1 IBLB_COMM_THREAD=0
EXTRA="--rccl-self" run ring_nocomm_res0 IBLB_DEBUG_NOCOMM=1 IBLB_RESERVE_CUS=0
IBLB_DEBUG_NOCOMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_nocomm" -o trace \
  -- python bench.py --nx 512 --ny 4096 --steps 100 --warmup 20 --no-cpu-baseline --no-profile-events --rccl-self \
  > /dev/null 2> "$OUT/prof_nocomm.err" || { tail -20 "$OUT/prof_nocomm.err"; exit 1; }
