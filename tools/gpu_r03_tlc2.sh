#!/bin/bash
# per-block draw timeline of C2 (8x8 form)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python tools/timeline.py c2 > gpurun_out/tl_c2.txt 2>&1 || { echo FAIL tl; tail -5 gpurun_out/tl_c2.txt; exit 1; }
