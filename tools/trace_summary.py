"""Per-kernel summary of a rocprofv3 kernel_trace.csv (grid, launches, mean/max duration,
resources): python tools/trace_summary.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

acc = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("gs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    key = (n, r["Grid_Size_X"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = acc.setdefault(key, dict(n=0, s=0.0, mx=0.0, res=(r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"],
                                                          r["Scratch_Size"])))
    a["n"] += 1
    a["s"] += d
    a["mx"] = max(a["mx"], d)
for (n, grid), a in sorted(acc.items(), key=lambda kv: -kv[1]["s"]):
    print(f"{n[:44]:44s} grid {int(grid):9d} n={a['n']:4d} mean {a['s'] / a['n']:9.1f} us  max {a['mx']:9.1f}  "
          f"vgpr/sgpr/lds/scratch {a['res']}")
