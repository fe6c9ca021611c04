#!/bin/bash
# per-block draw timelines (GS_FLAG_DRAW_STATS) of the small C5 views and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in v2 v4 c3; do
  timeout -k 10 240 python tools/timeline.py $c > gpurun_out/tl_$c.txt 2>&1 || { echo FAIL $c; tail -5 gpurun_out/tl_$c.txt; exit 1; }
done
