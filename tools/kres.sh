#!/bin/bash
# kernel resource usage (VGPRs, scratch, occupancy) of one source file: tools/kres.sh gs_render [kernel-substring]
cd "$(dirname "$0")/../openglgaussiansplattingrenderer_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -I../include \
  -c "csrc/$1.hip" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v k="${2:-}" '/Function Name:/ {show = index($0, k) > 0; if (show) print} show && /VGPRs:|ScratchSize|Occupancy|SGPRs:/ {print}'
