#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for sb in 16 8; do
  timeout -k 10 200 python bench.py --config c4 --draw-sub $sb --no-cpu-baseline --no-sort-bench > gpurun_out/c4_$sb.json 2>>gpurun_out/c4.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c4_$sb.json')); fr=d['frame']; print('c4 sub$sb fps %.0f' % d['value'], 'serial', fr['serial_ms_per_frame'], 'draw', fr['stage_ms']['draw'])"
done
