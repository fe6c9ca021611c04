#!/bin/bash
# Round-3 profile collection on the GPU box: kernel trace of the default bench command (split by
# pass), FETCH / WRITE / SQ passes (separate runs), the bench line after; C2 and a small C5 view
# traced too.  Outputs in gpurun_out/prof_r03/; the summaries are copied into profiles/r03/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > gpurun_out/prof_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/prof_tests.log; exit 1; }
tail -1 gpurun_out/prof_tests.log
OUT=$R/gpurun_out/prof_r03
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo TRACE_FAIL; exit 1; }
python3 $R/tools/trace_passes.py $OUT/trace/run_kernel_trace.csv 50 10 100 > $OUT/bench_trace_by_pass.txt
python3 $R/tools/trace_summary.py $OUT/trace/run_kernel_trace.csv > $OUT/bench_kernel_trace_summary.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/fetch.err || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/write.err || { echo WRITE_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/sq.err || { echo SQ_FAIL; exit 1; }
python3 $R/tools/pmc_summary.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
    $OUT/pmc_summary.json $OUT/sq/run_counter_collection.csv > $OUT/pmc_summary.txt
cp $OUT/pmc_summary.json $R/profiles/pmc_summary.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_c2 -o run --output-format csv -- \
    python3 $R/bench.py --config c2 --no-cpu-baseline --no-sort-bench > $OUT/c2_under_trace.json 2> $OUT/c2.err || { echo C2_FAIL; exit 1; }
python3 $R/tools/trace_passes.py $OUT/trace_c2/run_kernel_trace.csv 50 10 100 > $OUT/c2_trace_by_pass.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_v4 -o run --output-format csv -- \
    python3 $R/bench.py --view 4 --no-cpu-baseline --no-sort-bench > $OUT/v4_under_trace.json 2> $OUT/v4.err || { echo V4_FAIL; exit 1; }
python3 $R/tools/trace_passes.py $OUT/trace_v4/run_kernel_trace.csv 50 10 100 > $OUT/v4_trace_by_pass.txt
cd $R
timeout -k 10 200 python3 bench.py --sh --no-cpu-baseline --no-sort-bench > $OUT/sh.json 2> $OUT/sh.err || { echo SH_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py > $OUT/bench_latest.json 2> $OUT/bench.err || { echo BENCH_FAIL; exit 1; }
echo done
