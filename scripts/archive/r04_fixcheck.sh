# the tests changed for depth 7
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04fc
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bulk.py tests/test_gpu_fused.py -k "rccl_self_ring_ib_band_cycle or cilia_band_cycle or ib_band_many_points" \
  > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "^E  " $OUT/pytest.log | head -10
exit $rc
