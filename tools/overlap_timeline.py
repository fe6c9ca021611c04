"""Concurrency in a window of a rocprofv3 kernel trace: time with 0 / 1 / 2+ kernels running,
and per kernel name the time it ran alone vs beside another kernel.
python tools/overlap_timeline.py run_kernel_trace.csv FIRST_DRAW NUM_FRAMES"""
import collections
import csv
import sys

path, first, nfr = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].replace("gs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
rows.sort(key=lambda r: r["s"])
draws = [r for r in rows if r["n"].startswith("k_draw")]
t0, t1 = draws[first]["e"], draws[first + nfr]["e"]  # nfr frames: draw end to draw end
win = [r for r in rows if r["e"] > t0 and r["s"] < t1]
ev = []
for r in win:
    ev.append((max(r["s"], t0), 1, r["n"]))
    ev.append((min(r["e"], t1), -1, r["n"]))
ev.sort()
busy = collections.Counter()
alone = collections.Counter()
shared = collections.Counter()
running = collections.Counter()
prev = t0
for t, d, n in ev:
    k = sum(running.values())
    busy[min(k, 2)] += t - prev
    for name, c in running.items():
        if c:
            (alone if k == 1 else shared)[name.split("<")[0]] += (t - prev) * c
    running[n] += d
    prev = t
tot = t1 - t0
print(f"{nfr} frames, {tot / nfr / 1e3:.1f} us/frame: idle {busy[0] / tot:.1%}, one kernel {busy[1] / tot:.1%}, "
      f"two or more {busy[2] / tot:.1%}")
for n in sorted(set(alone) | set(shared), key=lambda n: -(alone[n] + shared[n])):
    print(f"  {n:22s} per frame: alone {alone[n] / nfr / 1e3:7.1f} us, beside another {shared[n] / nfr / 1e3:7.1f} us")
