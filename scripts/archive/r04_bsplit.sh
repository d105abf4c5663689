# the wall split in a slab's boundary sweeps (fixed sweeps): bit identity, mock slab groups, and the
# boundary sweeps' duration on the 512-column f64 self ring (rocprofv3 kernel trace) against the
# previous build (IBLB_LIB variant oldb: boundary sweeps without the split)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04bs
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_fused.py \
  -k "sweep_deep_bit_identical or rccl_slab_path_threads or rccl_self_ring" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_oldb.so; do
  tag=${lib:+old}; tag=${tag:-new}
  IBLB_LIB=$lib timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$tag" -o trace -- python3 scripts/ring_reps.py 512 4096 f64 --ring --reps 2 > "$OUT/r_$tag.json" 2> "$OUT/tr_$tag.err" || { tail -5 "$OUT/tr_$tag.err"; exit 1; }
  python3 - "$OUT/tr_$tag" "$tag" "$OUT/r_$tag.json" <<'PY'
import csv, glob, statistics, sys, json
kt = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
b = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt if "sweepk_kernel" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
i = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt if "sweepk_kernel" in r["Kernel_Name"] and "false" in r["Kernel_Name"]]
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[2], "boundary sweeps median us", round(statistics.median(b), 1), "n", len(b), "| interior median us", round(statistics.median(i), 1), "| ms/iter", d["median"])
PY
done
