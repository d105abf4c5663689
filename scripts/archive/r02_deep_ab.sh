#!/bin/bash
# Deep-sweep change A/B: the sweep bit-identity and bulk parity tests, then the headline bench
# (f64 and f32) and K2 / K4.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ag}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "${KEXPR:-sweep or bulk or k2 or k4 or column or self_ring_bulk or full_size}" \
  > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
[ $rc -eq 0 ] || exit $rc
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['launch_ms'], r['frac'])" "$2" "$1"; }
run() { local name=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" && one "$name" "$OUT/$name.json" || return 1; }
run M --steps 500 --warmup 50 || exit 1
run M_f32 --steps 500 --warmup 50 --precision f32 || exit 1
run K2 --workload K2 --steps 500 --warmup 50 || exit 1
run K4 --workload K4 --steps 500 --warmup 50 || exit 1
