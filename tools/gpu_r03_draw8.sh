#!/bin/bash
# draw forms: parity (both forms forced) and the config sweep with 8 vs 16
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_d8; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
b() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench --steps 50 $2 > $O/$1.json 2>> $O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/$1.json')); fr=d['frame']
print('$1', d['value'], 'fps', d['ms_per_step'], 'ms; serial', fr['serial_ms_per_frame'], 'E', fr['E'], 'sub', fr['draw_sub_block'], fr['stage_ms'])"; }
for s in 8 16; do
  b c2_s$s "--config c2 --draw-sub $s"
  for v in 1 2 4 7; do b v${v}_s$s "--view $v --draw-sub $s"; done
done
b c3_s0 ""
echo done
