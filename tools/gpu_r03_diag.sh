#!/bin/bash
# diagnostics: GPU suite, C5 view-4 and C2 blend timelines, C2 kernel trace by pass
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_diag; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/timeline.py v4 > $O/tl_v4.txt 2>&1 || { echo TL_FAIL; exit 1; }
timeout -k 10 200 python tools/timeline.py c2 > $O/tl_c2.txt 2>&1 || { echo TL_FAIL; exit 1; }
timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline --no-sort-bench > $O/c2.json 2>> $O/err.log || { echo C2_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trc2 -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config c2 --no-cpu-baseline --no-sort-bench > $GRAFT_REPO_ROOT/$O/c2_tr.json 2> $GRAFT_REPO_ROOT/$O/c2_tr.err || { echo TR_FAIL; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/trace_passes.py $GRAFT_REPO_ROOT/$O/trc2/run_kernel_trace.csv 50 10 100 > $GRAFT_REPO_ROOT/$O/c2_by_pass.txt
echo done
