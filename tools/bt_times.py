"""Average bottleneck kernel durations per variant from tools/bt_ab.sh traces.  usage: bt_times.py TAG..."""
import csv
import glob
import sys

for t in sys.argv[1:]:
    d = {}
    for f in glob.glob(f"gpurun_out/btab/p_{t}_1/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "bottleneck" in n:
                k = "first" if ("first" in n or "ILi64" in n) else "s1"
                d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(t, {k: (len(v), round(sum(v) / len(v), 1)) for k, v in sorted(d.items())})
