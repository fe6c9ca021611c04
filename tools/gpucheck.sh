#!/bin/bash
# GPU tests + two bench runs (A/B env in $AB, e.g. AB="GS_STREAM_PRIO=0"), summarised
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; echo tests rc=$?; tail -2 gpurun_out/gputests.log
run() { timeout -k 10 200 env $1 python bench.py --no-cpu-baseline --no-sort-bench > gpurun_out/bench_$2.json 2> gpurun_out/bench.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_$2.json')); fr=d['frame']
print('$1', d['value'], d['ms_per_step'], fr['stage_ms'], 'serial', fr['serial_ms_per_frame'], 'draw', d['roofline']['avg_launch_ms'])"; }
run "X=1" a1 && run "${AB:-X=1}" b1 && run "X=1" a2 && run "${AB:-X=1}" b2
