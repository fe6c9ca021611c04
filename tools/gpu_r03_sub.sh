#!/bin/bash
# draw time by sub-block form (--draw-sub 8 / 16) at C2 and C5 views 2 / 4 / 7
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sub; mkdir -p $O
for c in "c2:--config c2" "v2:--view 2" "v4:--view 4" "v7:--view 7"; do
  name=${c%%:*}; args=${c#*:}
  for sb in 8 16; do
    timeout -k 10 200 python bench.py $args --draw-sub $sb --no-cpu-baseline --no-sort-bench > $O/${name}_$sb.json 2>>$O/err.log || exit 1
    python3 -c "import json; d=json.load(open('$O/${name}_$sb.json')); fr=d['frame']; print('$name sub$sb fps %.0f' % d['value'], 'serial', fr['serial_ms_per_frame'], 'draw', fr['stage_ms']['draw'])"
  done
done
