#!/bin/bash
# Build a libdppo_hip.so variant that differs only in sampler_split.hip's compile flags (the other
# objects are the main build's, csrc/build/*.o): lib/variants/libdppo_hip_<tag>.so
# usage: tools/split_variant.sh <tag> "<extra flags>"
set -e
tag=$1; extra=$2
cd "$(dirname "$0")/../diffusionpolicyoptimization_amd/csrc"
mkdir -p ../lib/variants build/v_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -fvisibility=hidden \
    -I../../include -mllvm -amdgpu-mfma-vgpr-form $extra -c sampler_split.hip -o build/v_$tag/sampler_split.o
objs="build/api.o build/pack.o build/sampler.o build/v_$tag/sampler_split.o build/scan.o build/rowtile.o build/update.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libdppo_hip_$tag.so $objs
echo ../lib/variants/libdppo_hip_$tag.so
