# depth 6 vs 5 beyond M: the other BASELINE configs (K2/K3/K4 f64, K5 f32 IB band cycle) and the
# strong-scaling slabs on the RCCL self ring.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04dep2
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
one() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']), (d['roofline'] or {}).get('launch_ms'), d.get('ib_band'))" "$2" "$1"; }
for rep in 1 2; do
  for w in K2 K3 K4 K5; do
    for k in 5 6; do
      IBLB_SWEEP_DEPTH=$k timeout -k 10 200 $B --workload $w --steps 480 > "$OUT/${w}_k${k}_$rep.json" 2> "$OUT/err" && one "$w K $k" "$OUT/${w}_k${k}_$rep.json" || exit 1
    done
  done
done
for args in "512 4096 f64 --ring" "1024 4096 f64 --ring" "2048 4096 f64 --ring" "512 4096 f32 --ring" "1024 4096 f32 --ring" "1024 2048 f32 --k5 0 --ring --same-phase"; do
  for k in 5 6; do
    IBLB_SWEEP_DEPTH=$k timeout -k 10 150 python3 scripts/ring_reps.py $args --reps 3 > "$OUT/reps.json" 2>> "$OUT/reps.err" || exit 1
    echo "K $k $args: $(tail -1 $OUT/reps.json | cut -c1-150)"
  done
done
