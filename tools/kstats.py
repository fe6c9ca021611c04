"""Summarise a rocprofv3 kernel_trace.csv: per kernel (and grid) count / mean / max us, regs."""
import collections
import csv
import re
import sys

r = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
info = {}
for x in r:
    m = re.search(r"(k_\w+(<[^>]*>)?|__amd_\w+)", x["Kernel_Name"])
    n = m.group(1) if m else x["Kernel_Name"][:40]
    key = (n, x["Grid_Size_X"])
    d[key].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
    info[key] = (x["VGPR_Count"], x["SGPR_Count"], x["LDS_Block_Size"], x["Scratch_Size"])
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0][:44]:44s} grid {k[1]:>9s} n={len(v):4d} mean {sum(v)/len(v):9.1f} us  max {max(v):9.1f}"
          f"  vgpr/sgpr/lds/scratch {info[k]}")
