#!/bin/bash
# bench lines for the other configs / modes and every C5 view (pose k via RANK=k, one GPU)
O=gpurun_out/configs; mkdir -p $O
b() { timeout -k 10 200 env $1 python bench.py --no-cpu-baseline --no-sort-bench $2 > $O/$3.json 2>> $O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/$3.json')); fr=d['frame']
print('$3', d['value'], 'fps', d['ms_per_step'], 'ms; serial', fr['serial_ms_per_frame'], 'E', fr['E'], fr['stage_ms'], 'draw frac', d['roofline']['frac'])"; }
[ -n "$VIEWS_ONLY" ] || { b X=1 "--config c4" c4 && b X=1 "--sh" sh && b X=1 "--clean" clean && b X=1 "--fast-exp" fastexp && b X=1 "--config c2" c2; } || exit 1
for k in 0 1 2 3 4 5 6 7; do b X=1 "--view $k" view$k || exit 1; done
