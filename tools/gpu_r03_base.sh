#!/bin/bash
# round-3 baseline on one box: bench c3 + c2 lines, C2/C3 blend timelines, a kernel trace of C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_base; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo C3_FAIL; tail $O/c3.err; exit 1; }
timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline --no-sort-bench > $O/c2.json 2> $O/c2.err || { echo C2_FAIL; exit 1; }
timeout -k 10 200 python tools/timeline.py c2 > $O/tl_c2.txt 2>&1 || { echo TL_FAIL; exit 1; }
timeout -k 10 200 python tools/timeline.py c3 > $O/tl_c3.txt 2>&1 || { echo TL3_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trc2 -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config c2 --no-cpu-baseline --no-sort-bench --steps 50 > $GRAFT_REPO_ROOT/$O/c2_tr.json 2> $GRAFT_REPO_ROOT/$O/c2_tr.err || { echo TR_FAIL; exit 1; }
echo done
