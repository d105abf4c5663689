#!/bin/bash
# Edge flag (deep slab cycles): the slab-path GPU tests, then the self rings with IBLB_EDGE_FLAG 0 / 1
# alternated (7 regions each, one process per run).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05edge}
mkdir -p "$OUT"
[ -z "$SKIP_TESTS" ] && {
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    -k "rccl_slab_path_threads or rccl_self_ring or full_size_decomposed or rccl_slab_cells_per_lane" > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "passed|failed" "$OUT/pytest.log" | tail -3; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
  [ $rc -eq 0 ] || exit 1
}
for rep in 1 2; do
  for f in 0 1; do
    IFS='|' read -ra RUNS <<< "${RINGS:-512 4096 f64 --ring|1024 4096 f64 --ring|1024 2048 f32 --ring}"
    for args in "${RUNS[@]}"; do
      IBLB_EDGE_FLAG=$f timeout -k 10 150 python3 scripts/ring_reps.py $args >> "$OUT/reps_flag$f.jsonl" 2>> "$OUT/reps.err" || { tail -5 "$OUT/reps.err"; exit 1; }
      echo "flag=$f $(tail -1 $OUT/reps_flag$f.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["nx"], d["ny"], d["precision"], d["ring"], d["median"], d["spread"])')"
    done
  done
done
timeout -k 10 150 python3 scripts/ring_reps.py 4096 4096 f64 >> "$OUT/reps_n1.jsonl" 2>> "$OUT/reps.err" && tail -1 "$OUT/reps_n1.jsonl"
echo "== done"
