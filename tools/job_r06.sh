#!/bin/bash
# round-6 GPU job: light-trace timelines of the blend for the variants in $TL (lib/variants/NAME.so,
# tools/timeline.py -> gpurun_out/timeline_NAME.txt), then a same-box A/B of the variants given as
# arguments (tools/ab_variants.sh; SWEEP=1 adds the camera sweeps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
for v in $TL; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  timeout -k 10 200 python tools/timeline.py c3 > gpurun_out/timeline_$v.txt 2>&1 || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  head -6 gpurun_out/timeline_$v.txt
done
cp /tmp/orig.so $L/libgsplat_hip.so
[ $# -gt 0 ] && bash tools/ab_variants.sh "$@"
