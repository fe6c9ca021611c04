#!/bin/bash
# A/B of the working tree's library against HEAD's (tools/build_ab.sh): GPU tests on the new one,
# then bench new, old, new, old
cd $GRAFT_REPO_ROOT
L=openglgaussiansplattingrenderer_amd/lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo gpu tests rc=$rc; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit 1
cp $L/libgsplat_hip.so /tmp/new.so
for r in 1 2; do
  for v in new old; do
    if [ $v = new ]; then cp /tmp/new.so $L/libgsplat_hip.so; else cp $L/libgsplat_hip_old.so $L/libgsplat_hip.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench > gpurun_out/ab_$v$r.json 2> gpurun_out/ab.err || { cp /tmp/new.so $L/libgsplat_hip.so; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v$r.json')); fr=d['frame']
print('$v r$r fps %.1f' % d['value'], 'serial', fr['serial_ms_per_frame'], 'stages', fr['stage_ms'], 'draw1', d['roofline']['one_frame']['avg_launch_ms'])"
  done
done
cp /tmp/new.so $L/libgsplat_hip.so
