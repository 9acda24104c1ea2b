"""Print calls / average us of the kernels matching a substring in rocprofv3 kernel_stats.csv files."""
import csv
import sys

pat = sys.argv[1]
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        if pat in r["Name"]:
            print(f"{f}: {r['Calls']} calls, avg {float(r['AverageNs']) / 1e3:.1f} us, min {float(r['MinNs']) / 1e3:.1f}")
