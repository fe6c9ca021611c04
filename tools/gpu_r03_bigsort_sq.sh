#!/bin/bash
# SQ counters of the 64M-pair sort's kernels (what bounds the upsweep and downsweep)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/bsq; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM \
    -d $OUT/p1 -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2> $OUT/p1.err || { echo P1_FAIL; tail -3 $OUT/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY \
    -d $OUT/p2 -o run --output-format csv -- python3 $R/tools/bigsort.py > /dev/null 2> $OUT/p2.err || { echo P2_FAIL; tail -3 $OUT/p2.err; exit 1; }
cd $R
python3 tools/pmc.py $OUT/p1/run_counter_collection.csv $OUT/p2/run_counter_collection.csv
