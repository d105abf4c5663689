# band_level_kernel (the merged band chain's launches) built for 5 / 6 waves per SIMD (IBLB_LIB
# variants; default: no bound, 121 VGPRs, 4 waves) on the K5-width slab (640-wave launches on the
# chain's 32 CUs take two rounds at 4 waves per SIMD), lone and on the self ring, alternated
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04bl
mkdir -p $OUT
for rep in 1 2; do
  for args in "1024 2048 f32 --k5 0 --same-phase" "1024 2048 f32 --k5 0 --same-phase --ring" "1024 2048 f32 --k5 0.5 --ring"; do
    for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_bl5.so cuda_iblb_11_amd/lib/variants/libiblb_bl6.so; do
      IBLB_LIB=$lib timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 > "$OUT/r.json" 2>> "$OUT/err" || exit 1
      echo "$args ${lib:-default}: $(tail -1 $OUT/r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median"], d["spread"])')"
    done
  done
done
B="python3 bench.py --no-cpu-baseline --steps 420 --warmup 42"
for lib in "" cuda_iblb_11_amd/lib/variants/libiblb_bl6.so; do
  IBLB_LIB=$lib timeout -k 10 200 $B --workload K3 > "$OUT/b.json" 2> "$OUT/err" && echo "K3 ${lib:-default} $(python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(d['value'])")" || exit 1
done
