#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
cp $L/variants/statsnev.so $L/libgsplat_hip.so
timeout -k 10 200 python tools/timeline.py c3 > gpurun_out/tl_nev_c3.txt 2>&1; rc=$?
timeout -k 10 200 python tools/timeline.py c4 > gpurun_out/tl_nev_c4.txt 2>&1
cp /tmp/orig.so $L/libgsplat_hip.so
exit $rc
