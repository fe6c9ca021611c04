#!/bin/bash
# GPU tests on the working-tree library, draw stats, then a same-box A/B of lib/variants (args)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/diag.py c3 10 ref > gpurun_out/diag.log 2>&1 || exit 1
tail -2 gpurun_out/diag.log
bash tools/ab_variants.sh "$@"
