"""Kernels inside the compensated tier's windows (sim_f32* ... pool_fc_f32 on one stream) of a bench trace,
timed region only: ms per step and calls per kernel (--seq: the first window launch by launch).
usage: x3_breakdown.py TRACE_DIR DUMP.json [--seq]"""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import roofline_from_trace as R  # noqa: E402

d = json.load(open(sys.argv[2]))
rows = sorted(R.in_region(R._csv(sys.argv[1], "kernel_trace.csv"), d.get("region_ns")), key=lambda r: int(r["Start_Timestamp"]))
steps = d["steps"]
win, open_at = [], {}
for r in rows:
    n, s = r["Kernel_Name"], R._stream(r)
    if "sim_f32" in n and s not in open_at:
        open_at[s] = int(r["Start_Timestamp"])
    elif "pool_fc_f32" in n and s in open_at:
        win.append((s, open_at.pop(s), int(r["End_Timestamp"])))
c, k = collections.Counter(), collections.Counter()
for r in rows:
    s, t = R._stream(r), int(r["Start_Timestamp"])
    if any(ws == s and a <= t <= b for ws, a, b in win):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        c[n] += (int(r["End_Timestamp"]) - t) / 1e6 / steps
        k[n] += 1
print(f"windows {len(win)} ({len(win) / steps:.1f} per step), span {sum(b - a for _, a, b in win) / 1e6 / steps:.2f} ms per step")
for n, v in c.most_common(25):
    print(f"{v:8.2f} ms/step {k[n] / steps:6.1f} calls  {n}")
print(f"{sum(c.values()):8.2f} total")
if len(sys.argv) > 3 and sys.argv[3] == "--seq" and win:   # the first window's launches in order (layer by layer)
    s0, a0, b0 = win[0]
    for r in rows:
        t = int(r["Start_Timestamp"])
        if R._stream(r) == s0 and a0 <= t <= b0:
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            print(f"{(int(r['End_Timestamp']) - t) / 1e3:9.1f} us  {n}")
