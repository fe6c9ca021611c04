#!/bin/bash
# Kernel trace of K frames of a config (rocprofv3 --kernel-trace --stats), summarised per kernel.
#   bash tools/ktrace.sh TAG [cfg] [flags] [frames] [lanes]      (run from the repo root on the GPU box)
set -eo pipefail
TAG=${1:-kt}; CFG=${2:-c3}; FLAGS=${3:-0}; K=${4:-10}; LANES=${5:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 $R/tools/frames.py $CFG $FLAGS $K $LANES > $OUT/frames.log 2>&1
python3 $R/tools/trace_summary.py $OUT/run_kernel_trace.csv > $OUT/summary.txt
cat $OUT/summary.txt
