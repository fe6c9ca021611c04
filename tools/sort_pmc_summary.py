"""Counter bytes per key of the beyond-cache pair sort (bench.sort_bench_big, 64M uniform
pairs), from rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs) of tools/bigsort.py:
FETCH_SIZE x2 (the gfx950 correction for wide coalesced streams, MI355X_MICROARCH.md) +
WRITE_SIZE, summed over the sort kernels' dispatches, per sort, over n keys.
usage: python tools/sort_pmc_summary.py FETCH.csv WRITE.csv out.json [n]"""
import collections
import csv
import json
import re
import sys

n = int(sys.argv[4]) if len(sys.argv) > 4 else 64 << 20
SORT = ("k_upsweep", "k_scan_rows", "k_downsweep")
tot = collections.defaultdict(float)
cnt = collections.Counter()
for path, counter in ((sys.argv[1], "FETCH_SIZE"), (sys.argv[2], "WRITE_SIZE")):
    for x in csv.DictReader(open(path)):
        if x["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+)", x["Kernel_Name"])
        if not m or m.group(1) not in SORT:
            continue
        tot[(m.group(1), counter)] += float(x["Counter_Value"]) * 1024.0  # KiB per dispatch
        if counter == "FETCH_SIZE":
            cnt[m.group(1)] += 1
sorts = cnt["k_downsweep"] / 4.0
per_kernel = {k: {"dispatches": cnt[k], "fetch_bytes_x2": 2 * tot[(k, "FETCH_SIZE")] / sorts,
                  "write_bytes": tot[(k, "WRITE_SIZE")] / sorts} for k in SORT}
b = sum(v["fetch_bytes_x2"] + v["write_bytes"] for v in per_kernel.values()) / n
out = {"n": n, "sorts": sorts, "counter_bytes_per_key": b, "per_sort": per_kernel,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs) of tools/bigsort.py; FETCH x2 + WRITE"}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(f"counter bytes per key: {b:.2f} over {sorts:g} sorts of {n} keys")
for k, v in per_kernel.items():
    print(f"  {k:12s} {v['dispatches']:4d} dispatches  fetch x2 {v['fetch_bytes_x2'] / 1e6:8.1f} MB  "
          f"write {v['write_bytes'] / 1e6:8.1f} MB per sort")
