"""Build profiles/pmc_summary.json from rocprofv3 --pmc runs (FETCH_SIZE and WRITE_SIZE in
separate passes, as MI355X_MICROARCH.md prescribes).

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch.  gfx950 correction: FETCH_SIZE counts 128-B
streaming requests at 64 B (reads 1/2 of a wide coalesced stream), so for kernels whose reads
are wide coalesced streams the fetch is doubled.  The blend's reads are 4-32-B random gathers:
calibrated on a known byte count (tools/micro/gather.hip + gather_pmc.sh ->
profiles/r02/calibration.txt), each such gather that misses L2 is tallied as exactly one 64-B
request, so its fetch is used as-is (x1).  Both numbers are recorded.
usage: python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json [SQ.csv]
The optional SQ pass adds each kernel's mean SQ_* counters per dispatch ("sq"); bench.py prices
the blend's VALU issue ceiling from SQ_INSTS_VALU.
"""
import collections
import csv
import json
import re
import sys

GATHER_KERNELS = {"k_draw"}  # reads are random gathers: FETCH_SIZE taken as exact

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:3]:
    for x in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+|__amd_\w+)", x["Kernel_Name"])
        n = m.group(1) if m else x["Kernel_Name"][:40]
        acc[n][x["Counter_Name"]].append(float(x["Counter_Value"]))
out = {}
for k, cs in acc.items():
    f = cs.get("FETCH_SIZE", [])
    w = cs.get("WRITE_SIZE", [])
    if not f or not w:
        continue
    fetch = sum(f) / len(f) * 1024.0
    write = sum(w) / len(w) * 1024.0
    corr = 1.0 if k in GATHER_KERNELS else 2.0
    out[k] = {"dispatches": len(f), "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
              "fetch_correction": corr, "hbm_bytes_per_launch": fetch * corr + write}
if len(sys.argv) > 4:  # SQ pass: mean per dispatch
    sq = collections.defaultdict(lambda: collections.defaultdict(list))
    for x in csv.DictReader(open(sys.argv[4])):
        m = re.search(r"(k_\w+|__amd_\w+)", x["Kernel_Name"])
        n = m.group(1) if m else x["Kernel_Name"][:40]
        sq[n][x["Counter_Name"]].append(float(x["Counter_Value"]))
    for k, cs in sq.items():
        if k in out:
            out[k]["sq"] = {c: sum(v) / len(v) for c, v in cs.items()}
json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
for k, v in sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
    print(f"{k:24s} {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch  (fetch raw {v['fetch_size_bytes_raw'] / 1e6:.1f} "
          f"x{v['fetch_correction']:.0f}, write {v['write_size_bytes'] / 1e6:.1f})")
    if "sq" in v:
        q = v["sq"]
        wc = max(q.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        print(f"{'':24s} SQ: valu {q.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} any {q.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
              f"wait_any {q.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst {q.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} of wave "
              f"cycles; insts valu {q.get('SQ_INSTS_VALU', 0):.3g} salu {q.get('SQ_INSTS_SALU', 0):.3g} per launch")
