#!/bin/bash
# round 5: the config lines, the fast-exp blend's SQ counters beside the default's, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out; R=$(pwd); P=$R/$O/fastexp_sq; mkdir -p $P
bash tools/gpu_run.sh configs || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $P/sq -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 2 6 > /dev/null 2> $P/sq.err || { echo SQ_FAIL; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- \
    python3 $R/tools/frames.py c3 2 12 1 > /dev/null 2> $P/trace.err || { echo TRACE_FAIL; exit 1; }
cd $R
python3 - $P/sq/run_counter_collection.csv > $P/sq_summary.txt <<'PY'
import collections, csv, sys
acc = collections.defaultdict(list)
for x in csv.DictReader(open(sys.argv[1])):
    if "k_draw" in x["Kernel_Name"]:
        acc[x["Counter_Name"]].append(float(x["Counter_Value"]))
print("k_draw (fast exp), mean per dispatch:", {k: round(sum(v) / len(v), 1) for k, v in sorted(acc.items())})
PY
cat $P/sq_summary.txt
grep k_draw $P/trace/run_kernel_stats.csv | cut -c1-60,200-400
timeout -k 10 300 python bench.py > $O/bench_r05b.json 2> $O/bench_r05b.err || { tail -5 $O/bench_r05b.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_r05b.json')); fr=d['frame']
print('fps', d['value'], 'traffic', d['roofline'].get('traffic'), d['roofline'].get('traffic_source'), d['roofline']['issue'])
print('sort', json.dumps(d['sort']['beyond_cache']))"
