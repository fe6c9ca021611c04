#!/bin/bash
# round-6 GPU job: light-trace timelines of the blend for the variants in $TL (lib/variants/NAME.so,
# tools/timeline.py -> gpurun_out/timeline_NAME.txt), then a same-box A/B of the variants given as
# arguments (tools/ab_variants.sh; SWEEP=1 adds the camera sweeps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
L=openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
# TESTV=NAME: every GPU test on lib/variants/NAME.so first (stops the job if one fails)
if [ -n "$TESTV" ]; then
  cp $L/variants/$TESTV.so $L/libgsplat_hip.so
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/tests_$TESTV.log 2>&1
  rc=$?; tail -2 gpurun_out/tests_$TESTV.log
  cp /tmp/orig.so $L/libgsplat_hip.so
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/tests_$TESTV.log | head -5; exit 1; }
fi
for v in $TL; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  timeout -k 10 200 python tools/timeline.py c3 > gpurun_out/timeline_$v.txt 2>&1 || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  head -6 gpurun_out/timeline_$v.txt
done
cp /tmp/orig.so $L/libgsplat_hip.so
[ $# -gt 0 ] && { bash tools/ab_variants.sh "$@" || exit 1; }
# SWEEPV="a b": a second same-box A/B of those variants with the camera sweeps
[ -n "$SWEEPV" ] && SWEEP=1 bash tools/ab_variants.sh $SWEEPV
exit 0
