"""Mean duration of one kernel's dispatches [first, first + count) in a rocprofv3
kernel_trace.csv, in dispatch order -- e.g. the bench's timed region (its warm-up draws come
first): python tools/trace_window.py run_kernel_trace.csv k_draw 10 100"""
import csv
import sys

path, name, first, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[first:first + count]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
print(f"{name}: dispatches {first}..{first + len(sel) - 1} of {len(rows)}: mean {sum(d) / len(d):.1f} us "
      f"(min {min(d):.1f}, max {max(d):.1f})")
