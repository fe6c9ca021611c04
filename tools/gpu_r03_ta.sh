#!/bin/bash
# texture-address / L1 counters of the C3 frame's kernels (is the blend's chunk walk -- 64
# random 8-byte box gathers per chunk -- bound by the address path?)  One counter group per pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ta; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o -E "\b(TA|TD|TCP)_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/names.txt || true
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr -d $OUT/p1 -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/p1.err || { echo P1_FAIL; tail -3 $OUT/p1.err; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/p2.err || { echo P2_FAIL; tail -3 $OUT/p2.err; }
cd $R
for p in p1 p2; do f=$(ls $OUT/$p/run_counter_collection.csv 2>/dev/null) && python3 tools/pmc.py $f; done
wc -l $OUT/names.txt
