#!/bin/bash
# C4 (3840x2160): per-block draw timeline, then the draw forms (16x16 / 8x8 sub-blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python tools/timeline.py c4 > gpurun_out/tl_c4.txt 2>&1 || { echo FAIL tl; tail -5 gpurun_out/tl_c4.txt; exit 1; }
bash tools/gpu_r03_c4sub.sh
