#!/bin/bash
# the 64M-pair sort: timing, then a kernel trace of it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/bigsort; mkdir -p $OUT
cd $R && timeout -k 10 300 python tools/bigsort.py > $OUT/bigsort.json 2> $OUT/err.log || { echo FAIL; tail $OUT/err.log; exit 1; }
cat $OUT/bigsort.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2>> $OUT/err.log || { echo TRACE_FAIL; exit 1; }
python3 - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/bigsort/trace/run_kernel_stats.csv')))
for r in rows:
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
