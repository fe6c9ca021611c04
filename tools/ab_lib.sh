#!/bin/bash
# A/B of an alternative library build: bench twice with lib/libgsplat_hip.so, then twice with $1
L=openglgaussiansplattingrenderer_amd/lib
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench > gpurun_out/ab_$2.json 2> gpurun_out/ab.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$2.json')); fr=d['frame']
print('$1', d['value'], d['ms_per_step'], fr['stage_ms'], 'serial', fr['serial_ms_per_frame'], 'draw', d['roofline']['avg_launch_ms'])"; }
run base a1 && run base a2 && cp $L/$1 $L/libgsplat_hip.so && run $1 b1 && run $1 b2
