"""Per-kernel mean durations of a rocprofv3 kernel trace of `bench.py`, split by the bench's passes
(the draw dispatches mark them: 2 untimed frames, the one-lane latency pass, the one-lane stage
pass, the warm-up, the timed region with frames in flight).  The bench line's
roofline.avg_launch_ms is the one-lane latency pass's k_draw mean; this is its trace-side check.
python tools/trace_passes.py run_kernel_trace.csv NSER WARMUP STEPS"""
import collections
import csv
import sys

path, nser, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def short(r):
    n = r["Kernel_Name"].replace("gs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n[:48]


draws = [r for r in rows if "k_draw" in r["Kernel_Name"]]
bounds = [0, 2, 2 + nser, 2 + 2 * nser, 2 + 2 * nser + warm, 2 + 2 * nser + warm + steps]
names = ["untimed", "one-lane latency pass", "one-lane stage pass", "warm-up", "timed region (frames in flight)"]
for p in range(len(names)):
    if bounds[p + 1] > len(draws) or bounds[p] >= bounds[p + 1]:
        continue
    t0 = int(draws[bounds[p]]["Start_Timestamp"])
    t1 = int(draws[bounds[p + 1] - 1]["End_Timestamp"])
    # the pass's kernels: from the end of the previous pass's last draw to this pass's last draw
    lo = int(draws[bounds[p] - 1]["End_Timestamp"]) if bounds[p] > 0 else 0
    acc = collections.OrderedDict()
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > t1:
            continue
        a = acc.setdefault(short(r), [0, 0.0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] = max(a[2], (e - s) / 1e3)
    print(f"== {names[p]}: draws {bounds[p]}..{bounds[p + 1] - 1}, span {(t1 - t0) / 1e3:.1f} us")
    for n, (c, tot, mx) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        print(f"   {n:48s} n={c:5d} mean {tot / c:8.1f} us  max {mx:8.1f} us")
