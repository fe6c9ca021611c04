#!/bin/bash
# prefix-sort check on the GPU box: its tests, then the full GPU suite and two bench runs
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefix.py -x -v --timeout 200 --timeout-method thread > gpurun_out/prefix_tests.log 2>&1
rc=$?; echo prefix tests rc=$rc; tail -5 gpurun_out/prefix_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo gpu tests rc=$rc; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench > gpurun_out/bench_p$r.json 2> gpurun_out/bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_p$r.json')); fr=d['frame']
print('fps', d['value'], d['ms_per_step'], fr['stage_ms'], 'serial', fr['serial_ms_per_frame'], 'draw', d['roofline']['avg_launch_ms'])"
done
