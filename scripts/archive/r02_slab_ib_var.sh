set -o pipefail
mkdir -p gpurun_out/r02az
B="python3 bench.py --nx 1024 --ny 2048 --precision f32 --steps 300 --warmup 30 --no-cpu-baseline --workload K5"
for r in 1 2 3; do timeout -k 10 120 $B > gpurun_out/r02az/m$r.json 2>/dev/null || exit 1; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('moving', d['ms_per_step'], d['prime'], d['ib_band'])" gpurun_out/r02az/m$r.json; done
for r in 1 2; do timeout -k 10 120 $B --frozen > gpurun_out/r02az/f$r.json 2>/dev/null || exit 1; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('frozen', d['ms_per_step'], d['prime'], d['ib_band'])" gpurun_out/r02az/f$r.json; done
