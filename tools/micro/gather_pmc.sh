#!/bin/bash
# On the GPU box (repo root): FETCH_SIZE / WRITE_SIZE calibration of random gathers and the
# sort's HBM bytes (sortTests input, 64M pairs).  Separate PMC passes, each under its own limit.
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
M=$R/tools/micro
timeout -k 10 120 $M/gather 3 > $OUT/gather_plain.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/g_$C -o run --output-format csv -- $M/gather 2 > $OUT/gather_$C.txt 2> $OUT/g_$C.err
done
for K in 0 3; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/s${K}_$C -o run --output-format csv -- $M/rocprim_sort 3 $K > $OUT/sort${K}_$C.txt 2> $OUT/s${K}_$C.err
  done
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/s${K}_trace -o run --output-format csv -- $M/rocprim_sort 10 $K > $OUT/sort${K}_trace.txt 2> $OUT/s${K}_trace.err
done
echo CALIB_DONE
