#!/bin/bash
# GPU tests of a file on a variant library (lib/variants/$1.so), then the main library restored:
#   bash tools/job_variant_tests.sh VARIANT TESTFILE [-k EXPR]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
L=openglgaussiansplattingrenderer_amd/lib
v=$1; shift; f=$1; shift
cp $L/libgsplat_hip.so /tmp/main_vt.so && cp $L/variants/$v.so $L/libgsplat_hip.so || exit 1
timeout -k 10 400 python -u -m pytest $f -x -q -m gpu --timeout 120 --timeout-method thread "$@" > gpurun_out/vt_$v.log 2>&1
rc=$?
cp /tmp/main_vt.so $L/libgsplat_hip.so
tail -3 gpurun_out/vt_$v.log
exit $rc
