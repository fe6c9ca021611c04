#!/bin/bash
# the GPU sort tests on the working-tree library, then the 64M-pair A/B of lib/variants (args)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sort.py > gpurun_out/up2_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/up2_tests.log; exit 1; }
tail -1 gpurun_out/up2_tests.log
bash tools/gpu_r03_bigsort_ab.sh "$@"
