#!/bin/bash
# Round profile collection on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command itself
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate passes; no trace domains beside --pmc)
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries into profiles/<round>/.
set -eo pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $OUT/bench_under_trace.json 2> $OUT/trace.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/fetch.err
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/write.err
# SQ pass (instruction mix and wave cycles; 8 SQ counters, a pass of its own)
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/sq.err
python3 $R/tools/pmc_summary.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
    $OUT/pmc_summary.json $OUT/sq/run_counter_collection.csv > $OUT/pmc_summary.txt
python3 $R/tools/trace_summary.py $OUT/trace/run_kernel_trace.csv > $OUT/bench_kernel_trace_summary.txt
cp $OUT/pmc_summary.json $R/profiles/pmc_summary.json
# the bench line itself (with the CPU baseline), against the fresh PMC summary
timeout -k 10 300 python3 $R/bench.py > $OUT/bench_latest.json 2> $OUT/bench.err
echo done
