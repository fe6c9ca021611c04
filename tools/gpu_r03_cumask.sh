#!/bin/bash
# spatial partition experiment: the blend on a CU subset (gs_ctx_set_blend_cus), C3 headline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_cu; mkdir -p $O
b() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench $2 > $O/$1.json 2>> $O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/$1.json')); fr=d['frame']
print('$1', d['value'], 'fps', d['ms_per_step'], 'ms; serial', fr['serial_ms_per_frame'], 'draw live', d['roofline']['timed_region']['avg_launch_ms'], fr['stage_ms'])"; }
b base3 ""
for c in 224 192 160; do b cu${c}_l3 "--blend-cus $c"; b cu${c}_l2 "--blend-cus $c --lanes 2"; done
b base3b ""
b base2 "--lanes 2"
echo done
