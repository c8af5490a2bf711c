#!/bin/bash
# Build a tuning variant of libdppo_hip.so with extra compile flags into lib/variants/.
# usage: tools/variant_build.sh <tag> "<extra flags>"      (then: DPPO_LIB=<path> python tools/...)
set -e
tag=$1; extra=$2
cd "$(dirname "$0")/../diffusionpolicyoptimization_amd/csrc"
out=../lib/variants/libdppo_hip_$tag.so
mkdir -p ../lib/variants build/$tag
objs=""
for f in api pack sampler sampler_split scan rowtile update collective; do
    vf="-mllvm -amdgpu-mfma-vgpr-form"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -fvisibility=hidden \
        -I../../include $vf $extra -c $f.hip -o build/$tag/$f.o &
    objs="$objs build/$tag/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $objs
echo $out
