#!/bin/bash
# On the GPU box: one SQ counter pass (8 SQ counters, its own rocprofv3 run) of six C3 frames per
# lib/variants/NAME.so, k_draw's mean per dispatch printed side by side.  Restores the library.
#   bash tools/pmc_variants.sh NAME...        (COUNTERS env: another set of <= 8 SQ counters;
#                                              KERNEL env: another kernel name pattern, default k_draw)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd); L=$R/openglgaussiansplattingrenderer_amd/lib; O=$R/gpurun_out/pmc_variants; mkdir -p $O
C=${COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU"}
cp $L/libgsplat_hip.so /tmp/libgsplat_hip.pmc_orig.so
rc=0
for v in "$@"; do
  cp $L/variants/$v.so $L/libgsplat_hip.so
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$v -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $O/$v.err) || { echo "$v: PMC_FAIL"; rc=1; break; }
  python3 - "$v" $O/$v/run_counter_collection.csv "${KERNEL:-k_draw}" <<'EOF'
import collections, csv, re, sys
acc = collections.defaultdict(list)
for x in csv.DictReader(open(sys.argv[2])):
    if re.search(sys.argv[3], x["Kernel_Name"]):
        acc[x["Counter_Name"]].append(float(x["Counter_Value"]))
print(sys.argv[1], {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(acc.items())})
EOF
done
cp /tmp/libgsplat_hip.pmc_orig.so $L/libgsplat_hip.so
exit $rc
