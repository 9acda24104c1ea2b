"""Per-call durations (us) of kernels matching a substring in rocprofv3 kernel_trace.csv files."""
import csv
import sys

pat = sys.argv[1]
for f in sys.argv[2:]:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    print(f, " ".join(f"{x:.0f}" for x in d))
