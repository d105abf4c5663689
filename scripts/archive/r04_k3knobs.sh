# K3 (f64, 2048^2 + 256 moving points) at depth 7: band chain knobs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k3
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --workload K3 --steps 420 --warmup 42"
for rep in 1 2; do
  for kv in "IBLB_X=0" "IBLB_BAND_MERGE=2" "IBLB_BAND_PAR=2" "IBLB_BAND_CUS=64" "IBLB_BAND_MERGE=2 IBLB_BAND_PAR=2"; do
    env $kv timeout -k 10 200 $B > "$OUT/b.json" 2> "$OUT/err" || exit 1
    echo "$kv: $(python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d['ib_band'])")"
  done
done
