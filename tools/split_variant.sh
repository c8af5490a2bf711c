#!/bin/bash
# Build a variant of libdppo_hip.so whose sampler_split.hip gets extra compile flags, linked with
# the in-tree objects of the other sources (make first), into lib/variants/libdppo_hip_<tag>.so.
# usage: tools/split_variant.sh <tag> "<extra flags>"   (then tools/ab_variants.sh <tag>...)
set -e
tag=$1; extra=$2
cd "$(dirname "$0")/../diffusionpolicyoptimization_amd/csrc"
mkdir -p ../lib/variants build/$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -fvisibility=hidden \
    -I../../include -mllvm -amdgpu-mfma-vgpr-form $extra -c sampler_split.hip -o build/$tag/sampler_split.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/variants/libdppo_hip_$tag.so \
    build/api.o build/pack.o build/sampler.o build/$tag/sampler_split.o build/scan.o build/rowtile.o build/update.o
echo ../lib/variants/libdppo_hip_$tag.so
