#!/bin/bash
# SQ and FETCH counters of C3 frames for each lib/variants/NAME.so given (one pmc pass each).
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/openglgaussiansplattingrenderer_amd/lib
cp $L/libgsplat_hip.so /tmp/orig.so
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT=$R/gpurun_out/sqab/$v; mkdir -p $OUT
  cp $L/variants/$v.so $L/libgsplat_hip.so
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/fetch.err || { echo FETCH_FAIL; cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/write.err || { echo WRITE_FAIL; cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $OUT/sq.err || { echo SQ_FAIL; cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
  python3 $R/tools/pmc_summary.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
      $OUT/pmc_summary.json $OUT/sq/run_counter_collection.csv > $OUT/pmc_summary.txt
  echo "== $v"; grep -A1 "k_preprocess" $OUT/pmc_summary.txt
done
cp /tmp/orig.so $L/libgsplat_hip.so
