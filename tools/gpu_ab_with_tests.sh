#!/bin/bash
# GPU tests with lib/variants/$1.so (the in-tree library restored afterwards), draw stats, then a
# same-box A/B of lib/variants (the remaining args)
set -o pipefail
cd $GRAFT_REPO_ROOT
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig_lib.so
cp $L/variants/$1.so $L/libgsplat_hip.so
shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/gputests.log
[ $rc -le 1 ] || { cp /tmp/orig_lib.so $L/libgsplat_hip.so; exit $rc; }
timeout -k 10 120 python tools/timeline.py c3 > gpurun_out/timeline.log 2>&1 || { cp /tmp/orig_lib.so $L/libgsplat_hip.so; exit 1; }
tail -4 gpurun_out/timeline.log
cp /tmp/orig_lib.so $L/libgsplat_hip.so
bash tools/ab_variants.sh "$@"
