# HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the deep launches of K2 / K3 / K4 / K5 at
# depth 7 -> profiles/pmc_traffic.json keys as bench.py looks them up
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04pmcc
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --steps 70 --warmup 7 --prime-seconds 0.3 --no-profile-events"
for cfg in "K2 f64_2048x2048_n1_sweep7 sweepk_kernel<double,@2,@273,@7," "K4 f64_8192x2048_n1_sweep7 sweepk_kernel<double,@2,@273,@7," \
           "K3 f64_2048x2048_n1_ib256_sweep7 sweepk_kernel<double,@2,@273,@7," "K5 f32_8192x2048_n1_ib6144_sweep7 sweepk_kernel<float,@2,@81,@7,"; do
  set -- $cfg
  w=$1; key=$2; kn=$(echo "$3" | tr '@' ' ')
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$OUT/${w}_$c" -o pmc -- $B --workload $w > /dev/null 2> "$OUT/${w}_$c.err" \
      || { tail -20 "$OUT/${w}_$c.err"; exit 1; }
  done
  python3 scripts/pmc_summary.py $key "$OUT/${w}_FETCH_SIZE" "$OUT/${w}_WRITE_SIZE" "$OUT/pmc_traffic.json" --kernel "$kn" || exit 1
done
cat "$OUT/pmc_traffic.json"
