#!/bin/bash
# Builds libmrt.so with extra compile flags into gpu-ray-tracing_amd/lib/variants/NAME/
# (for tools/ab.py). Usage: build_variant.sh NAME "-DFOO=0 -DBAR=1" [git revision]
# With a revision, the sources (csrc/, include/) are those of that commit.
set -e
NAME=$1; FLAGS=$2; REV=$3
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/gpu-ray-tracing_amd/lib/variants/$NAME; B=/tmp/mrt_variant_$NAME
mkdir -p $OUT $B
if [ -n "$REV" ]; then
    rm -rf $B/src && mkdir -p $B/src
    git -C $REPO archive "$REV" gpu-ray-tracing_amd/csrc include | tar -x -C $B/src
    D=$B/src/gpu-ray-tracing_amd
else
    D=$REPO/gpu-ray-tracing_amd
fi
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fgpu-flush-denormals-to-zero -ffp-contract=off -Wall -Wno-unused-result -I$D/../include"
/opt/rocm/bin/hipcc $HIPFLAGS -fno-slp-vectorize $FLAGS -c $D/csrc/trace_kernel.hip -o $B/trace_kernel.o
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c $D/csrc/raygen_kernel.hip -o $B/raygen_kernel.o
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -x hip -c $D/csrc/mrt_api.cpp -o $B/mrt_api.o
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -x hip -c $D/csrc/wide_bvh.cpp -o $B/wide_bvh.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o $OUT/libmrt.so $B/trace_kernel.o $B/raygen_kernel.o $B/mrt_api.o $B/wide_bvh.o
echo "built $OUT/libmrt.so ($FLAGS${REV:+ at $REV})"
