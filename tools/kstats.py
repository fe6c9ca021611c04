"""Summarise a rocprofv3 kernel_stats.csv: python tools/kstats.py <csv>"""
import csv
import sys

for x in csv.DictReader(open(sys.argv[1])):
    n = x["Name"].replace("gs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print(f"{n[:44]:44s} calls {x['Calls']:>5s} avg {float(x['AverageNs']) / 1e3:8.1f} us  "
          f"min {float(x['MinNs']) / 1e3:7.1f}  max {float(x['MaxNs']) / 1e3:7.1f}  {float(x['Percentage']):5.1f}%")
