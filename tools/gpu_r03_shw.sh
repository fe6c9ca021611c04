#!/bin/bash
# SH bench (k_sh_colour waves per SIMD variants), two alternating rounds, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
for r in 1 2; do for v in "$@"; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  timeout -k 10 200 python bench.py --sh --no-cpu-baseline --no-sort-bench > gpurun_out/shw_$v.json 2>>gpurun_out/shw.err || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/shw_$v.json')); print('$v', round(d['value'],1), d['frame']['stage_ms'])"
done; done
cp /tmp/orig.so $L/libgsplat_hip.so
