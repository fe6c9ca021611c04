"""Idle time between consecutive GPU operations of a rocprofv3 --kernel-trace (+ memory-copy)
run: per-frame GPU busy vs wall, and the largest gaps with the operations around them.
python tools/gaps.py trace_dir"""
import csv
import re
import glob
import os
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "*kernel_trace.csv")) + glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
    for x in csv.DictReader(open(f)):
        name = x.get("Kernel_Name") or ("copy " + x.get("Direction", ""))
        rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), name[:60]))
rows.sort()
# steady state: from the 10th frame (k_preprocess launch) on
pre = [i for i, r in enumerate(rows) if "k_preprocess" in r[2]]
if len(pre) > 12:
    rows = rows[pre[10]:pre[-1]]
    print(f"frames {len(pre) - 11} (steady state)")
busy = sum(e - s for s, e, _ in rows)
span = rows[-1][1] - rows[0][0]
print(f"ops {len(rows)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {100 * (1 - busy / span):.1f} %")
gaps = []
for a, b in zip(rows, rows[1:]):
    gaps.append((b[0] - a[1], a[2], b[2]))
gaps.sort(reverse=True)
tot = {}
for g, a, b in gaps:
    if g > 0:
        k = (re.sub(r"^(void )?gs::\(anonymous namespace\)::", "", a).split("(")[0][-40:],
             re.sub(r"^(void )?gs::\(anonymous namespace\)::", "", b).split("(")[0][-40:])
        tot[k] = tot.get(k, 0) + g
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v / 1e3:9.1f} us  after {k[0]:40s} before {k[1]}")
