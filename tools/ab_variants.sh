#!/bin/bash
# On the GPU box: for each lib/variants/*.so (args: names, in order), swap it in and measure:
# the frame bench (3 lanes, 100 frames) and the draw alone (diag: one lane, stage timing).
# Alternates the order twice (a b c a b c) against box drift.  Restores the original library.
# BENCH_ARGS (environment): extra bench.py arguments, e.g. "--view 4"; SWEEP=1: with the camera
# sweep (frame.camera_sweep, prefix frames/s and frames rendered again printed).
set -o pipefail
cd $GRAFT_REPO_ROOT
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/libgsplat_hip.orig.so
for round in 1 2; do
  for v in "$@"; do
    cp $L/variants/$v.so $L/libgsplat_hip.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench $([ "$SWEEP" = 1 ] || echo --no-sweep) $BENCH_ARGS > gpurun_out/ab_${v}_$round.json 2> gpurun_out/ab.err || { cp /tmp/libgsplat_hip.orig.so $L/libgsplat_hip.so; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_${v}_$round.json')); fr=d['frame']
print('$v r$round fps %.1f' % d['value'], 'serial', fr['serial_ms_per_frame'], 'stages', fr['stage_ms'], 'draw1', d['roofline']['avg_launch_ms'])
sw = fr.get('camera_sweep')
if sw: print('   sweep', {k: (v['prefix']['frames_per_s'], v['prefix']['rendered_again'], v['prefix']['prefix_frames'], v['full_sort']['frames_per_s'], v.get('static_same_poses_fps')) for k, v in sw.items() if isinstance(v, dict)})"
  done
done
cp /tmp/libgsplat_hip.orig.so $L/libgsplat_hip.so
