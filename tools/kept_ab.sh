#!/bin/bash
# Round-5 kept-emission validation on the GPU box: the prefix tests on a GS_PREFIX_TRACE build of the
# working tree (per-frame miss lines), every GPU test, the turned-frame kept form's prefix tests
# (kturntr, not fatal), then the same-box A/B of kept0 / kept1 / kturn with the camera sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
L=openglgaussiansplattingrenderer_amd/lib
O=gpurun_out
cp $L/libgsplat_hip.so /tmp/main.so
run_prefix() {  # $1 variant, $2 log, $3 -k expression
  cp $L/variants/$1.so $L/libgsplat_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_prefix.py -x -v -s -m gpu --timeout 120 --timeout-method thread ${3:+-k "$3"} > $O/$2 2>&1
  local rc=$?
  cp /tmp/main.so $L/libgsplat_hip.so
  grep -E "prefix seen.*miss 1|passed|failed" $O/$2 | tail -8
  return $rc
}
run_prefix ktrace ktrace.log || exit 1
bash tools/gpu_run.sh tests || exit 1
run_prefix kturntr kturn.log "moving_camera or kept_frames"
SWEEP=1 BENCH_ARGS=--no-facade bash tools/gpu_run.sh variants kept0 kept1 kturn
