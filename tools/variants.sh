#!/bin/bash
# Build library variants for a same-box A/B (run here, then tools/ab_variants.sh on the GPU box):
#   tools/variants.sh NAME [extra hipcc flags...]   -> openglgaussiansplattingrenderer_amd/lib/variants/NAME.so
#   ARCH=gfx950:xnack- tools/variants.sh NAME   -> a variant for another target id
# built from the working tree (use `git stash` / a scratch checkout for HEAD variants).
set -e
cd "$(git rev-parse --show-toplevel)/openglgaussiansplattingrenderer_amd"
NAME=$1; shift
mkdir -p lib/variants /tmp/variant_$NAME
F="-O3 -std=c++17 -fPIC --offload-arch=${ARCH:-gfx950} -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-result -I../include $*"
for s in gs_capi gs_render gs_sort gs_load gs_util; do
  X=""; [ $s = gs_render ] && X="-mllvm -amdgpu-sched-strategy=max-memory-clause"  # as the Makefile
  /opt/rocm/bin/hipcc $F $X -c csrc/$s.hip -o /tmp/variant_$NAME/$s.o &
done
/opt/rocm/bin/hipcc $F -x hip -c csrc/gs_host.cpp -o /tmp/variant_$NAME/gs_host.o &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=${ARCH:-gfx950} -fPIC -o lib/variants/$NAME.so /tmp/variant_$NAME/*.o
echo built lib/variants/$NAME.so
