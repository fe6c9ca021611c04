#!/bin/bash
# GS_SORT11 prototype: the >=16M pair-sort tests on it, then the 64M sort (tools/bigsort.py),
# s8 (default) / s11 alternated twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/job_variant_tests.sh s11 tests/test_gpu_sort.py || exit 1
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/main_s.so
for r in 1 2; do
  for v in s8 s11; do
    cp $L/variants/$v.so $L/libgsplat_hip.so
    timeout -k 10 120 python tools/bigsort.py > gpurun_out/bigsort_${v}_${r}.json 2>> gpurun_out/bigsort.err || { cp /tmp/main_s.so $L/libgsplat_hip.so; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bigsort_${v}_${r}.json')); print('$v r$r', d.get('ms_pairs'), d.get('gkeys_per_s'), d.get('sorted_ok'))"
  done
done
cp /tmp/main_s.so $L/libgsplat_hip.so
