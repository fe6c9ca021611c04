#!/bin/bash
# builds tools/micro/rocprim_sort against the in-tree libgsplat_hip.so (tools only)
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 rocprim_sort.hip -o rocprim_sort \
  -L../../openglgaussiansplattingrenderer_amd/lib -lgsplat_hip -Wl,-rpath,'$ORIGIN/../../openglgaussiansplattingrenderer_amd/lib'
