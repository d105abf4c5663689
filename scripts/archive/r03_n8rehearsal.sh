#!/bin/bash
# bench.py's N = 8 branch end to end on one GPU (--same-device: 8 ranks under torch.distributed.run,
# gloo process group, every rank its slab as an RCCL self ring): M (512-column slabs) and K5
# (1024-column slabs, filaments on every slab edge).  The throughput of 8 ranks sharing one GPU is
# not a scaling number; the run exercises the driver's 8-rank command path.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03n8}
mkdir -p "$OUT"
for w in M K5; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 8 --same-device --workload $w --steps 40 --warmup 5 \
    --prime-seconds 0.3 --no-cpu-baseline > "$OUT/n8_$w.json" 2> "$OUT/n8_$w.err" || { tail -20 "$OUT/n8_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['n_gpus'], d['config']['parallelism'], round(d['value']), d['ms_per_step'], d['roofline']['kernel'][:60], d['roofline']['launch_timing'])" "$OUT/n8_$w.json"
done
echo "== done"
