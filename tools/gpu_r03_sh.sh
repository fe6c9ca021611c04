#!/bin/bash
# SH parity tests, then the SH bench line and a kernel trace of it
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "sh or SH" tests > gpurun_out/sh_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/sh_tests.log; exit 1; }
tail -1 gpurun_out/sh_tests.log
timeout -k 10 200 python bench.py --sh --no-cpu-baseline --no-sort-bench > gpurun_out/sh.json 2> gpurun_out/sh.err || { echo SH_FAIL; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/sh.json')); print('sh', d['value'], d['frame']['stage_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sh_trace -o run --output-format csv -- python3 $R/bench.py --sh --no-cpu-baseline --no-sort-bench > /dev/null 2>&1 || { echo TRACE_FAIL; exit 1; }
python3 $R/tools/trace_passes.py $R/gpurun_out/sh_trace/run_kernel_trace.csv 50 10 100 | sed -n '/one-lane stage/,/warm-up/p'
