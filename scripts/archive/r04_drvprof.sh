# rocprofv3 kernel stats of the driver's exact bench command (20 steps: deep launches of 6 + 7 + 7)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04drv
mkdir -p $OUT
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -c 700 "$OUT/bench.json"; echo
find "$OUT/trace" -name "*kernel_stats.csv" -exec head -4 {} \;
