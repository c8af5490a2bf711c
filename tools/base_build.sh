#!/bin/bash
# Build libdppo_hip.so from a git revision's sources into lib/variants/libdppo_hip_<tag>.so, for
# same-box A/B runs against the working tree (tools/_variants.sh <tag>).
# usage: tools/base_build.sh <tag> [rev=HEAD] ["<extra flags>"]
set -e
tag=$1; rev=${2:-HEAD}; extra=$3
root="$(cd "$(dirname "$0")/.." && pwd)"
src=$(mktemp -d /tmp/dppo_base.XXXX)
git -C "$root" archive "$rev" diffusionpolicyoptimization_amd/csrc include | tar -x -C "$src"
cd "$src/diffusionpolicyoptimization_amd/csrc"
out="$root/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$tag.so"
mkdir -p "$(dirname "$out")" obj
objs=""
for f in api pack sampler sampler_split scan rowtile update; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -fvisibility=hidden \
        -I../../include -mllvm -amdgpu-mfma-vgpr-form $extra -c $f.hip -o obj/$f.o &
    objs="$objs obj/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs
rm -rf "$src"
echo "$out"
