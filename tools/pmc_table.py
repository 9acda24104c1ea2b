"""Per-kernel table from one rocprofv3 --pmc pass (run_counter_collection.csv): for every kernel name, the launches,
the average duration and the average of each counter; with SQ wave counters, the fractions of wave cycles parked
(SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY, of which LDS: SQ_WAIT_INST_LDS) and issuing (SQ_ACTIVE_INST_ANY), the
MFMA pipe's busy share (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs... per XCD-summed counters) and the
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).  The passes serialise the kernels, so durations are isolated ones.
usage: python tools/pmc_table.py DIR [regex]"""
import collections
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
c = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if rx and not rx.search(n):
        continue
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:48]
    c[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[n][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for n, cs in sorted(c.items(), key=lambda kv: -sum(dur[kv[0]].values())):
    a = {k: sum(v) / len(v) for k, v in cs.items()}
    d = sum(dur[n].values()) / len(dur[n])
    line = f"{n:48s} n={len(dur[n]):4d} {d:8.1f}us"
    wc = a.get("SQ_WAVE_CYCLES")
    if wc:
        for k, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"), ("SQ_WAIT_INST_LDS", "ldsstall"),
                       ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_ACTIVE_INST_LDS", "lds")):
            if k in a:
                line += f" {lab}={a[k] / wc:5.3f}"
    g = a.get("GRBM_GUI_ACTIVE")
    if g:
        line += f" clk={g / 8 / d / 1e3:5.2f}GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            line += f" mfma_busy={a['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):5.3f}"
    others = {k: v for k, v in a.items() if k not in ("SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")}
    print(line)
    print("    " + " ".join(f"{k}={v:.4g}" for k, v in sorted(others.items())))
