#!/bin/bash
# prefix tests + a one-lane kernel trace of C3 + one bench run
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_frames.py -x -q --timeout 200 --timeout-method thread > gpurun_out/prefix_tests.log 2>&1
rc=$?; echo tests rc=$rc; tail -3 gpurun_out/prefix_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ktrace.sh ktq c3 0 12 1 > /dev/null 2>&1 || { echo trace failed; exit 1; }
head -24 gpurun_out/ktq/summary.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench > gpurun_out/bench_q.json 2> gpurun_out/bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_q.json')); fr=d['frame']
print('fps', d['value'], d['ms_per_step'], fr['stage_ms'], 'serial', fr['serial_ms_per_frame'], 'draw', d['roofline']['avg_launch_ms'])"
