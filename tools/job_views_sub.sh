#!/bin/bash
# the C5 views' blend in both sub-block forms (gs_ctx_set_draw_sub 16 / 8), alternated twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/views_sub; mkdir -p $O
for r in 1 2; do
  for v in 2 6 7 4; do
    for sub in 16 8; do
      timeout -k 10 200 python bench.py --view $v --draw-sub $sub --no-cpu-baseline --no-sort-bench --no-sweep --no-facade \
          > $O/v${v}_s${sub}_$r.json 2>> $O/err.log || exit 1
      python3 -c "
import json; d=json.load(open('$O/v${v}_s${sub}_$r.json')); fr=d['frame']
print('view $v sub $sub r$r fps %.1f' % d['value'], 'draw1', d['roofline']['avg_launch_ms'], 'serial', fr['serial_ms_per_frame'])"
    done
  done
done
