#!/bin/bash
# Build an A/B variant of libmd2hot.so: md2hot.hip (or another source given by
# SRC=path) compiled with extra flags, linked with the in-tree objects of the other
# sources.  Usage: tools/build_variant.sh NAME [-DFOO=1 ...]
# Output: abx/NAME/libmd2hot.so (run with MD2_LIB=abx/NAME/libmd2hot.so).
set -e
name=$1; shift
cd "$(dirname "$0")/.."
SRC=${SRC:-monodepth2_amd/csrc/md2hot.hip}
mkdir -p abx/$name
obj=abx/$name/$(basename ${SRC%.hip}).o
# the in-tree build flags of md2hot.hip (monodepth2_amd/build.py FLAGS)
slp=""
[ "$(basename $SRC)" = "md2hot.hip" ] && slp="-fno-slp-vectorize -mllvm --amdgpu-sched-strategy=iterative-ilp"
case "$(basename $SRC)" in conv.hip|bnorm.hip|decoder.hip) slp="-mllvm --amdgpu-sched-strategy=max-ilp";; esac
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Iinclude $slp "$@" -c $SRC -o $obj
others=$(ls monodepth2_amd/csrc/obj/*.o | grep -v "/$(basename ${SRC%.hip}).o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o abx/$name/libmd2hot.so $obj $others
rm -f $obj
echo abx/$name/libmd2hot.so
