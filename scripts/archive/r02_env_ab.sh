#!/bin/bash
# bench.py under several environment settings (CFGS: "label:VAR=v VAR2=w" ...), one line each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02aj}
mkdir -p "$OUT"
for cfg in $CFGS; do
  lab=${cfg%%:*}; ev=${cfg#*:}; ev=${ev//,/ }
  env $ev timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 500 --warmup 50 $BARGS > "$OUT/$lab.json" 2> "$OUT/$lab.err" || { tail -5 "$OUT/$lab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['launch_ms'], r['frac'])" "$OUT/$lab.json" "$lab"
done
