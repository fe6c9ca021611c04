#!/bin/bash
# the round-end driver's sequence on one box, from the committed tree: GPU tests, smoke(), the
# default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/dc_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 $O/dc_tests.log; exit 1; }
tail -1 $O/dc_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/dc_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/dc_smoke.log; exit 1; }
tail -1 $O/dc_smoke.log
timeout -k 10 300 python bench.py > $O/dc_bench.json 2> $O/dc_bench.err || { echo BENCH_FAIL; tail -5 $O/dc_bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/dc_bench.json'))
print('bench', d['value'], d['unit'], 'draw', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
