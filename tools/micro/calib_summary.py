"""Summarise tools/micro/gather_pmc.sh's output (gpurun_out/calib) into profiles/<round>/calibration.txt:
  1. FETCH_SIZE per random gather (4/8/16/32-B elements; tables inside / beyond the Infinity Cache),
     against the known counts (idx stream 4n B coalesced -- reported at 1/2 on gfx950 --, n gathers);
  2. the radix sort's measured HBM bytes per key and GB/s (sortTests input, 64M uniform pairs), gsplat
     (k_upsweep / k_scan_rows / k_downsweep) beside rocPRIM's radix_sort_pairs on the same box.
usage: python tools/micro/calib_summary.py gpurun_out/calib profiles/r02/calibration.txt"""
import collections
import csv
import os
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
out = []
n = 10_000_000

# ---- 1. gathers
rows = {c: [r for r in csv.DictReader(open(os.path.join(src, f"g_{c}", "run_counter_collection.csv")))
            if "k_gather" in r["Kernel_Name"]] for c in ("FETCH_SIZE", "WRITE_SIZE")}
cfg = [dict(x.split("=") for x in l.split()[1:]) for l in open(os.path.join(src, "gather_FETCH_SIZE.txt"))
       if l.startswith("CONFIG")]
plain = [dict(x.split("=") for x in l.split()[1:]) for l in open(os.path.join(src, "gather_plain.txt"))
         if l.startswith("CONFIG")]
reps = int(cfg[0]["reps"])
out.append("FETCH_SIZE calibration, random gathers (tools/micro/gather.hip, n = 10M, last of %d dispatches per config)" % reps)
out.append("  known bytes: idx stream 40 MB coalesced (FETCH_SIZE reports 1/2: 20 MB), out stream 40 MB written")
for i, c in enumerate(cfg):
    f = float(rows["FETCH_SIZE"][i * reps + reps - 1]["Counter_Value"]) * 1024
    w = float(rows["WRITE_SIZE"][i * reps + reps - 1]["Counter_Value"]) * 1024
    per = (f - 2 * n) / n
    t = plain[i]
    out.append(f"  elem {int(c['elem']):2d} B, table {float(c['table_mb']):6.0f} MiB: FETCH {f / 1e6:6.1f} MB -> "
               f"{per:5.1f} B per gather; WRITE {w / 1e6:5.1f} MB; {float(t['best_us']):6.1f} us "
               f"({float(t['ggathers']):.1f} G gathers/s)")
out.append("  => a random gather of 4-32 B is tallied as one 64-B request per L2 miss (64 B exactly when the table")
out.append("     is beyond the caches; fewer when L2 absorbs repeats): FETCH_SIZE x1 is the calibrated reading of")
out.append("     gather traffic (k_draw), x2 stays the reading of wide coalesced streams.")
out.append("")

# ---- 2. sort bytes


def per_kernel(case, counter):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(src, f"s{case}_{counter}", "run_counter_collection.csv"))):
        k = r["Kernel_Name"]
        m = re.match(r"^(?:void )?(?:gs::)?(?:\(anonymous namespace\)::)?(k_upsweep|k_scan_rows|k_downsweep)\b", k)
        if m:
            name = "gsplat:" + m.group(1)
        elif "rocprim" in k:
            name = "rocprim"
        else:
            name = "other"
        acc[name] += float(r["Counter_Value"]) * 1024
    return acc


for case, nk, label in ((0, 5_119_993, "sortTests input (tests/sortTests.cpp:181, 5,119,993 keys)"),
                        (3, 64 << 20, "uniform 32-bit, 64M pairs (beyond the 256 MiB Infinity Cache)")):
    f, w = per_kernel(case, "FETCH_SIZE"), per_kernel(case, "WRITE_SIZE")
    times = [l for l in open(os.path.join(src, f"sort{case}_FETCH_SIZE.txt")) if "gsplat" in l]
    tl = open(os.path.join(src, f"sort{case}_trace.txt")).read().strip()
    m = re.search(r"rocprim\s+([\d.]+) us.*gsplat\s+([\d.]+) us", tl)
    t_roc, t_gs = float(m.group(1)), float(m.group(2))
    sorts = 6  # 3 warm + 3 timed sorts per implementation (rocprim_sort 3 <case>)
    gf = sum(v for k, v in f.items() if k.startswith("gsplat")) / sorts
    gw = sum(v for k, v in w.items() if k.startswith("gsplat")) / sorts
    rf, rw = f["rocprim"] / sorts, w["rocprim"] / sorts
    g_bytes, r_bytes = 2 * gf + gw, 2 * rf + rw
    out.append(f"Radix sort (u32 key, u32 value), {label}")
    out.append(f"  gsplat : {t_gs:8.1f} us, {nk / t_gs / 1e3:6.2f} Gkeys/s; HBM {g_bytes / 1e6:8.1f} MB/sort = "
               f"{g_bytes / nk:5.1f} B/key (FETCH x2 {2 * gf / 1e6:.1f} + WRITE {gw / 1e6:.1f}) -> "
               f"{g_bytes / (t_gs * 1e-6) / 1e12:.2f} TB/s = {g_bytes / (t_gs * 1e-6) / 8e12:.1%} of 8 TB/s; "
               f"algorithmic 68 B/key -> {68 * nk / (t_gs * 1e-6) / 1e12:.2f} TB/s")
    for k in sorted(f):
        if k.startswith("gsplat"):
            out.append(f"      {k:22s} FETCH raw {f[k] / sorts / 1e6:8.1f} MB  WRITE {w.get(k, 0) / sorts / 1e6:8.1f} MB per sort")
    out.append(f"  rocPRIM: {t_roc:8.1f} us, {nk / t_roc / 1e3:6.2f} Gkeys/s; HBM {r_bytes / 1e6:8.1f} MB/sort = "
               f"{r_bytes / nk:5.1f} B/key -> {r_bytes / (t_roc * 1e-6) / 1e12:.2f} TB/s  (gsplat/rocPRIM time {t_gs / t_roc:.2f})")
    out.append("")
os.makedirs(os.path.dirname(dst), exist_ok=True)
open(dst, "w").write("\n".join(out) + "\n")
print("\n".join(out))
