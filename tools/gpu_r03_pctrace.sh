#!/bin/bash
# kernel trace of the C2 and view-4 bench lines (precull kernels), split by pass
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pctrace; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in "c2:--config c2" "v4:--view 4"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- \
      python3 $R/bench.py $args --no-cpu-baseline --no-sort-bench > $OUT/$name.json 2> $OUT/$name.err || { echo FAIL $name; exit 1; }
  python3 $R/tools/trace_passes.py $OUT/$name/run_kernel_trace.csv 50 10 100 > $OUT/${name}_by_pass.txt
  echo "== $name"; sed -n '/one-lane stage pass/,/warm-up/p' $OUT/${name}_by_pass.txt
done
