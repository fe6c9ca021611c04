#!/bin/bash
# kernel trace of the GS_SORT11 prototype on the 64M sort (lib/variants/s11.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
L=openglgaussiansplattingrenderer_amd/lib; R=$(pwd)
cp $L/libgsplat_hip.so /tmp/main_t.so && cp $L/variants/s11.so $L/libgsplat_hip.so || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s11trace -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2> $R/gpurun_out/s11trace.err
rc=$?
cp /tmp/main_t.so $R/$L/libgsplat_hip.so
cut -d, -f1-4 $R/gpurun_out/s11trace/run_kernel_stats.csv | head -14
exit $rc
