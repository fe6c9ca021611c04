#!/bin/bash
# the 64M-pair sort for each lib/variants/NAME.so given, twice, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
for r in 1 2; do for v in "$@"; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  timeout -k 10 300 python tools/bigsort.py > gpurun_out/bs_$v.json 2>>gpurun_out/bs.err || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bs_$v.json')); print('$v', d['ms_pairs'], d['gkeys_per_s'], d['hbm_frac_algorithmic'], d['sorted_ok'])"
done; done
cp /tmp/orig.so $L/libgsplat_hip.so
