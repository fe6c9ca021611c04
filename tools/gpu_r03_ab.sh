#!/bin/bash
# The GPU suite on the working-tree library, then a same-box A/B of lib/variants (args) at C3
# (tools/ab_variants.sh) and at C5 views 2 / 4 / C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_variants.sh "$@" || exit 1
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
for v in "$@"; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  for c in "--view 2" "--view 4" "--config c2"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench $c > $O/x.json 2>>$O/err.log || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
    python3 -c "import json; d=json.load(open('$O/x.json')); fr=d['frame']; print('$v', '$c', 'fps %.1f' % d['value'], 'serial', fr['serial_ms_per_frame'], fr['stage_ms'])"
  done
done
cp /tmp/orig.so $L/libgsplat_hip.so
