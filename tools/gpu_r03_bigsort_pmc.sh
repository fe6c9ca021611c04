#!/bin/bash
# FETCH_SIZE and WRITE_SIZE of the 64M-pair sort (separate passes), per sort: the counter bytes
# per key the bench line quotes (sort.beyond_cache.counter_bytes_per_key)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/bigsort_pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2> $OUT/fetch.err || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2> $OUT/write.err || { echo WRITE_FAIL; exit 1; }
python3 $R/tools/pmc_summary.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $OUT/pmc.json > $OUT/pmc.txt
cat $OUT/pmc.txt
python3 - <<'PY'
import json, os
d = json.load(open(os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/bigsort_pmc/pmc.json'))
n = 1 << 26
per_sort = 0.0
for k in ("k_upsweep", "k_scan_rows", "k_downsweep"):
    v = d[k]
    per_sort += v["hbm_bytes_per_launch"] * 4  # four launches of each per sort
print("counter bytes per key: %.1f (fetch x2 + write, per sort / 64M)" % (per_sort / n))
PY
