#!/bin/bash
# prefix tests on the working library, then tools/ab_variants.sh over lib/variants/*.so (args)
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_prefix.py -x -q --timeout 100 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/pt.log; exit 1; }
bash tools/ab_variants.sh "$@"
