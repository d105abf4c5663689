#!/bin/bash
# Build libiblb.so with alternative kernel sources (kernel A/B on the GPU box, same process layout
# as the product): scripts/build_variant.sh NAME DIR [extra hipcc flags] — every file in DIR
# (.h or .hip) replaces the csrc file of that name; the sweep units (lbm_sweep*.hip) and any
# replaced .hip are rebuilt, the other objects come from cuda_iblb_11_amd/build.
set -e
name=$1; dir=$2; shift 2
out=cuda_iblb_11_amd/lib/variants; tmp=cuda_iblb_11_amd/vbuild_$name  # csrc depth: ctx.h includes ../../include
rm -rf $tmp; mkdir -p $out $tmp
cp cuda_iblb_11_amd/csrc/*.h cuda_iblb_11_amd/csrc/*.hip $tmp/
cp $dir/* $tmp/ 2>/dev/null || true
rebuild="lbm_sweep lbm_sweepk3 lbm_sweepk4 lbm_sweepk5 lbm_sweepk6 lbm_sweepk7 $(cd $dir && ls *.hip 2>/dev/null | sed 's/\.hip$//')"
objs=""
for f in $(cd cuda_iblb_11_amd/csrc && ls *.hip | sed 's/\.hip$//'); do
  if echo " $rebuild " | grep -q " $f "; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c $tmp/$f.hip -o $tmp/$f.o &
    objs="$objs $tmp/$f.o"
  else
    objs="$objs cuda_iblb_11_amd/build/$f.o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libiblb_$name.so $objs -lrccl
echo built $out/libiblb_$name.so
