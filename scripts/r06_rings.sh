#!/bin/bash
# Strong-scaling rehearsal of the current tree (round 6): N = 1 bench line, then the per-rank slab of
# the 4096^2 lattice at N = 8 (512 x 4096 f64) lone and on the RCCL self ring, and the K5-width slab,
# each 7 timed regions in one process (ring_reps.py; RINGS: '|'-separated argument sets); VARIANTS: the
# same for IBLB_LIB builds or NAME=VALUE environment settings, REPS times.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06rings}
mkdir -p "$OUT"
for rep in $(seq ${REPS:-1}); do
for v in def ${VARIANTS}; do
  # a variant NAME=VALUE is the in-tree library under that environment setting
  case $v in
    def) lib="" ;;
    *=*) lib="$v" ;;
    *) lib="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_$v.so" ;;
  esac
  v=${v//=/-}
  env $lib timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/M_$v.json" 2> "$OUT/M_$v.err" || { tail -5 "$OUT/M_$v.err"; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms"])' "$OUT/M_$v.json" "M $v"
  IFS='|' read -ra sets <<< "${RINGS:-512 4096 f64|512 4096 f64 --ring}"
  for args in "${sets[@]}"; do
    env $lib timeout -k 10 150 python3 scripts/ring_reps.py $args >> "$OUT/reps_$v.jsonl" 2>> "$OUT/reps_$v.err" || { tail -5 "$OUT/reps_$v.err"; exit 1; }
    echo "$v $(tail -1 $OUT/reps_$v.jsonl)"
  done
done
done
echo "== done"
