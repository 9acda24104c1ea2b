"""Per-launch kernel durations of one ResNet chunk from a rocprofv3 kernel trace (single stream):
the last chunk that starts with the stem kernel.  usage: python tools/chunk_trace.py trace.csv [...]"""
import csv
import sys


def chunk(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
    starts = [i for i, k in enumerate(ks) if "stem" in k[0]]
    i0 = starts[-2] if len(starts) > 1 else starts[-1]
    i1 = starts[-1] if len(starts) > 1 else len(ks)
    out = []
    for name, d in ks[i0:i1]:
        if "pool_fc" in name:
            out.append((name, d))
            break
        out.append((name, d))
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:40]


cols = [chunk(p) for p in sys.argv[1:]]
n = max(len(c) for c in cols)
for i in range(n):
    cells = []
    for c in cols:
        cells.append(f"{c[i][1]:8.1f} {short(c[i][0]):40s}" if i < len(c) else " " * 49)
    print(" | ".join(cells))
print(" | ".join(f"{sum(d for _, d in c):8.1f} {'TOTAL':40s}" for c in cols))
