#!/bin/bash
# Build libiblb.so with an alternative lbm_sweep.hip (kernel A/B on the GPU box, same process
# layout as the product): scripts/build_variant.sh NAME path/to/lbm_sweep.hip [extra hipcc flags]
set -e
name=$1; src=$2; shift 2
out=cuda_iblb_11_amd/lib/variants; mkdir -p $out /tmp/var_$name
cp $src /tmp/var_$name/lbm_sweep.hip
cp cuda_iblb_11_amd/csrc/*.h /tmp/var_$name/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I cuda_iblb_11_amd/csrc "$@" -c /tmp/var_$name/lbm_sweep.hip -o /tmp/var_$name/lbm_sweep.o
objs=$(ls cuda_iblb_11_amd/build/*.o | grep -v -e lbm_sweep.o -e mock_rccl.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libiblb_$name.so $objs /tmp/var_$name/lbm_sweep.o -lrccl
echo built $out/libiblb_$name.so
