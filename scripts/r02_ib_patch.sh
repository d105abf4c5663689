#!/bin/bash
# IB band cycle with row patches: band tests, then K3 / K5 (moving points) with and without the
# row restriction, and the K5-width slab rehearsal.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02aa}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_bulk.py -k "band or k3 or k5 or moving or schedule" > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
[ $rc -eq 0 ] || exit $rc
one() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('ib_band'))" "$2" "$1"; }
for w in K3 K5; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w --steps 500 --warmup 50 > "$OUT/$w.json" 2> "$OUT/$w.err" && one "$w rows" "$OUT/$w.json" || exit 1
  IBLB_BAND_ROWS=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w --steps 500 --warmup 50 > "$OUT/${w}_cols.json" 2> "$OUT/${w}_cols.err" && one "$w cols" "$OUT/${w}_cols.json" || exit 1
done
TAG=${TAG:-r02aa} bash scripts/r02_ibslab_probe.sh
