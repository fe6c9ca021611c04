"""Summarise rocprofv3 --pmc counter_collection.csv: per kernel, mean counter value per dispatch."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for x in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+(<[^>]*>)?|__amd_\w+)", x["Kernel_Name"])
        n = m.group(1) if m else x["Kernel_Name"][:40]
        acc[n][x["Counter_Name"]].append(float(x["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
