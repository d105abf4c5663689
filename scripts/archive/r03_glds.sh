#!/bin/bash
# LDS-DMA staging of the deep walk's next column (IBLB_GLDS=1 build, lib/variants/libiblb_glds.so):
# deep-sweep bit-identity tests with the variant, then M f64 A/B against the product library.
set -o pipefail
OUT=gpurun_out/${TAG:-r03gl}
mkdir -p "$OUT"
IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_glds.so timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_gpu_fused.py -k "deep or sweep or ib_band" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_glds.so timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_gpu_bulk.py -k "m_bulk or k1 or k2" > "$OUT/pytest_bulk.log" 2>&1 || { tail -30 "$OUT/pytest_bulk.log"; exit 1; }
tail -2 "$OUT/pytest_bulk.log"
for i in 1 2 3; do
  for v in base glds; do
    lib=""; [ "$v" != base ] && lib="IBLB_LIB=cuda_iblb_11_amd/lib/variants/libiblb_$v.so"
    env $lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 500 --warmup 50 > "$OUT/M_${v}_$i.json" 2> "$OUT/M_${v}_$i.err" || { tail -5 "$OUT/M_${v}_$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['roofline']['launch_ms'])" "$OUT/M_${v}_$i.json" "$v #$i"
  done
done
