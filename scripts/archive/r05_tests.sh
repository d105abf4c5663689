#!/bin/bash
# A selection of -m gpu tests (TESTS="-k ...", default: the full-size decomposed parity and the
# forced band-chain mock groups), optionally followed by the whole suite (ALL=1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05t}
mkdir -p "$OUT"
timeout -k 10 ${TLIM:-900} python -u -m pytest -v -s --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests \
  ${TESTS:--k "full_size_decomposed or band_cycle_threads_chain"} > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -40
exit $rc
