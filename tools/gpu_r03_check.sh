#!/bin/bash
# the GPU suite, then bench lines of C3 (headline), C2 and C5 views 2 / 4 / 7 at the defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_chk; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench $2 > $O/$1.json 2>> $O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/$1.json')); fr=d['frame']
print('$1', d['value'], 'fps', d['ms_per_step'], 'ms; serial', fr['serial_ms_per_frame'], 'E', fr['E'], 'sub', fr['draw_sub_block'], fr['stage_ms'])"; }
b c3 ""
b c2 "--config c2"
for v in 2 4 7; do b v$v "--view $v"; done
echo done
