"""Average of each counter over the launches whose kernel name contains PATTERN in a rocprofv3 --pmc directory.
usage: python tools/pmc_kernel.py DIR PATTERN"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
c = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if sys.argv[2] in r["Kernel_Name"]:
        c[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(c.items()):
    print(f"{k:28s} launches {len(v):3d}  avg {sum(v) / len(v):.4g}")
