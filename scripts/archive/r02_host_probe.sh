#!/bin/bash
# Host submission vs completion time per iteration (scripts/host_probe.py) for the K5-width slab.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ae}
mkdir -p "$OUT"
P="timeout -k 10 120 python3 scripts/host_probe.py"
{
$P 1024 2048 f32 none &&
IBLB_BAND_FUSED=1 $P 1024 2048 f32 K5 &&
IBLB_BAND_FUSED=1 $P 1024 2048 f32 K5 frozen &&
IBLB_BAND_FUSED=0 $P 1024 2048 f32 K5 &&
IBLB_BAND_FUSED=0 $P 1024 2048 f32 K5 frozen &&
$P 1024 2048 f32 none rccl-self &&
IBLB_BAND_FUSED=0 $P 1024 2048 f32 K5 rccl-self &&
IBLB_BAND_SLAB_OV=0 IBLB_BAND_FUSED=0 $P 1024 2048 f32 K5 rccl-self &&
IBLB_BAND_FUSED=1 $P 1024 2048 f32 K5 rccl-self &&
IBLB_BAND_FUSED=1 $P 2048 2048 f64 K3 &&
IBLB_BAND_FUSED=0 $P 2048 2048 f64 K3
} 2>&1 | grep -v amdgpu.ids | tee "$OUT/host_probe.txt"
