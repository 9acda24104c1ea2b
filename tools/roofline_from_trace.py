"""Recompute bench.py's roofline figures from rocprofv3 output of the timed region alone.

bench.py --prof-dump records the timed region's CLOCK_MONOTONIC bounds (the clock of rocprofv3's
timestamps); kernels of a whole-run trace that start inside them are the timed steps (setup, keyword-DB
projection and warmup excluded).  From them this tool rebuilds the numbers bench.py reports from its own
hipEvents:

* the KWS bf16 conv family (conv_igemm* / conv_ring / conv_stream / bottleneck*) of the scoring pass:
  launches on the encoder's stream (the stream attention_kernel runs on: the clip pipeline's front end) are
  the encoder's GEMMs, and launches inside a re-scoring window (sim_f32*_kernel ... pool_fc_f32_kernel on the
  scoring stream) belong to the compensated-bf16 tier; the rest is the family bench.py times;
* the union of their [start, end] intervals per step (two scoring streams overlap) -> achieved TFLOP/s with
  the algorithmic FLOPs per step (bench.py --prof-dump, or 9.81 GFLOP x K);
* with the PMC passes (`--pmc FETCH_SIZE` / `--pmc WRITE_SIZE`, each with --kernel-trace so dispatches join
  the trace), fabric-side bytes of the same launches per step and per launch (FETCH_SIZE x2, the gfx950
  correction of MI355X_MICROARCH.md; both counters in KB);
* per_kernel (round 6): per tier and kernel the trace's launches and average duration, the dump's algorithmic
  GFLOP per launch (bench.py records each launch's kernel name) and the fraction of the 2.5 PFLOP/s bf16 peak.

usage: python tools/roofline_from_trace.py TRACE_DIR [--dump prof_dump.json]
       [--fetch PMC_DIR --fetch-dump DUMP --write PMC_DIR --write-dump DUMP] [--steps N] [--keywords K]
       [--out summary.json]
"""
import argparse
import csv
import glob
import gzip
import json
import os
from collections import defaultdict

CONV = ("conv_igemm", "conv_ring", "conv_stream", "bottleneck")   # bottleneck_s1* (r01) / bottleneck_kernel<CIN> (r02)
GFLOP_PER_PAIR_CONV = 9.8075   # the 52 convs of ResNet-50 at LEF maps [3, 75, 750] (bench.py algorithmic_tflop/K)


def _csv(d, suffix):
    """The rocprofv3 CSV ``*suffix`` under directory d, or d itself when it is a (.csv or .csv.gz) file."""
    if os.path.isfile(d):
        f = [d]
    else:
        f = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not f:
        raise SystemExit(f"no *{suffix} under {d}")
    opener = gzip.open if f[0].endswith(".gz") else open
    with opener(f[0], "rt") as fh:
        return list(csv.DictReader(fh))


def _stream(r):
    for k in ("Stream_Id", "Queue_Id"):
        if k in r and r[k] not in ("", None):
            return r[k]
    return "0"


def in_region(rows, region):
    if not region:
        return rows
    a, b = region
    return [r for r in rows if a <= int(r["Start_Timestamp"]) <= b]


def classify(rows):
    """rows of kernel_trace.csv -> (kws conv rows, x3 conv rows, encoder conv rows, other rows)."""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    enc_streams = {_stream(r) for r in rows if "attention_kernel" in r["Kernel_Name"]}
    windows, open_at = [], {}
    for r in rows:
        n, s = r["Kernel_Name"], _stream(r)
        if "sim_f32" in n and s not in open_at:   # sim_f32_kernel / sim_f32_e64_kernel
            open_at[s] = int(r["Start_Timestamp"])
        elif "pool_fc_f32_kernel" in n and s in open_at:
            windows.append((s, open_at.pop(s), int(r["End_Timestamp"])))
    kws, x3, enc, other = [], [], [], []
    for r in rows:
        n, s, t = r["Kernel_Name"], _stream(r), int(r["Start_Timestamp"])
        if not any(c in n for c in CONV):
            other.append(r)
        elif s in enc_streams:
            enc.append(r)
        elif any(ws == s and a <= t <= b for ws, a, b in windows):
            x3.append(r)
        else:
            kws.append(r)
    return kws, x3, enc, other


def union_ns(rows):
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    tot, cs, ce = 0, None, None
    for a, b in iv:
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        tot += ce - cs
    return tot


def pmc_bytes(d, counter, region_ns):
    """Sum of `counter` (KB -> bytes) over the KWS bf16 conv launches of the timed region of a PMC pass
    (its counter_collection.csv carries kernel names, queues and timestamps, so it classifies like a trace)."""
    rows = [r for r in _csv(d, "counter_collection.csv") if r.get("Counter_Name", counter) == counter]
    kws = classify(in_region(rows, region_ns))[0]
    return sum(float(r["Counter_Value"]) for r in kws) * 1024.0, len(kws)


def short_name(n: str) -> str:
    """rocprofv3 kernel name -> the runtime's short name (cbw_kws_profile_kernels): template arguments kept, the
    namespace / signature dropped; the mangled stage-1 block names mapped to their source names."""
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    if "bottleneck_ring_kernel" in n:
        return "bottleneck_ring_kernel"
    if "bottleneck_kernelILi64" in n:
        return "bottleneck_kernel<64>"
    depth, out = 0, []
    for ch in n:   # cut the argument list: the first "(" outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).strip()


def per_kernel(kws, x3, dump, steps, peak=2500.0):
    """Per (tier, kernel): launches per step and average duration from the trace, algorithmic GFLOP per launch
    from the --prof-dump records (bench.py: per launch its FLOPs, tier and kernel name), the fraction of the dense
    bf16 MFMA peak, and the hipEvent average of the same launches beside the trace's (the join check)."""
    gf, ev = {}, {}
    if dump and "kernel" in dump:
        for nm, f, t, a, b in zip(dump["kernel"], dump["flop"], dump["tier"], dump["start_ms"], dump["end_ms"]):
            k = ("bf16_scoring" if t == 0 else "compensated_rescoring" if t == 1 else "fp8_first_tier", nm)
            gf.setdefault(k, []).append(f / 1e9)
            ev.setdefault(k, []).append((b - a) * 1e3)
    rows = []
    for tier, rs in (("bf16_scoring", kws), ("compensated_rescoring", x3)):
        acc = defaultdict(list)
        for r in rs:
            acc[short_name(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for nm, d in acc.items():
            avg = sum(d) / len(d)
            g = gf.get((tier, nm))
            row = {"tier": tier, "kernel": nm, "launches_per_step": round(len(d) / steps, 2),
                   "ms_per_step": round(sum(d) / 1e3 / steps, 3), "avg_us": round(avg, 1)}
            if g:
                row["gflop_per_launch"] = round(sum(g) / len(g), 2)
                row["frac"] = round(sum(g) / len(g) * 1e9 / (avg * 1e-6) / 1e12 / peak, 4)
                row["hipevent_avg_us"] = round(sum(ev[(tier, nm)]) / len(ev[(tier, nm)]), 1)
                row["launches_joined"] = len(g) == len(d)
            rows.append(row)
    return sorted(rows, key=lambda r: -r["ms_per_step"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--dump", default=None)
    ap.add_argument("--fetch", default=None)
    ap.add_argument("--write", default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--fetch-dump", default=None, help="--prof-dump JSON of the FETCH_SIZE pass (its region)")
    ap.add_argument("--write-dump", default=None, help="--prof-dump JSON of the WRITE_SIZE pass (its region)")
    ap.add_argument("--keywords", type=int, default=10000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dump = json.load(open(a.dump)) if a.dump else None
    rows = in_region(_csv(a.trace, "kernel_trace.csv"), dump.get("region_ns") if dump else None)
    kws, x3, enc, other = classify(rows)
    steps = a.steps or (dump["steps"] if dump else 1)
    tier = dump.get("tier") if dump else None   # round-2 dumps: 0 bf16 scoring, 1 compensated tier
    flop_all = (sum(dump["flop"]) / steps) if dump else GFLOP_PER_PAIR_CONV * 1e9 * a.keywords
    flop_step = (sum(f for f, t in zip(dump["flop"], tier) if t == 0) / steps) if tier else flop_all
    u = union_ns(kws) / 1e6 / steps
    s = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kws) / 1e6 / steps
    span = (max(int(r["End_Timestamp"]) for r in rows) - min(int(r["Start_Timestamp"]) for r in rows)) / 1e6
    out = {
        "steps": steps, "trace_span_ms": round(span, 3), "trace_span_ms_per_step": round(span / steps, 3),
        "kws_conv_launches": len(kws), "kws_conv_launches_per_step": len(kws) / steps,
        "kws_conv_union_ms_per_step": round(u, 3), "kws_conv_sum_ms_per_step": round(s, 3),
        "algorithmic_tflop_per_step": round(flop_step / 1e12, 4),
        "achieved_tflops": round(flop_step / (u * 1e-3) / 1e12, 2),
        "frac_of_2500": round(flop_step / (u * 1e-3) / 1e12 / 2500.0, 4),
        "x3_conv_launches_per_step": len(x3) / steps,
        "x3_conv_sum_ms_per_step": round(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in x3) / 1e6 / steps, 3),
        "encoder_conv_launches_per_step": len(enc) / steps,
    }
    if tier:   # both tiers of the conv family (they overlap when bench.py runs --x3-overlap)
        ub = union_ns(kws + x3) / 1e6 / steps
        out.update({"both_tiers_conv_union_ms_per_step": round(ub, 3), "both_tiers_tflop_per_step": round(flop_all / 1e12, 4),
                    "both_tiers_achieved_tflops": round(flop_all / (ub * 1e-3) / 1e12, 2),
                    "both_tiers_frac_of_2500": round(flop_all / (ub * 1e-3) / 1e12 / 2500.0, 4),
                    # bench.py's headline since r03: algorithmic FLOPs (each pair once, the bf16 tier's) over the
                    # union of both tiers' launches; the compensated tier's FLOPs are exactness overhead
                    "algorithmic_over_both_tiers_tflops": round(flop_step / (ub * 1e-3) / 1e12, 2),
                    "algorithmic_over_both_tiers_frac": round(flop_step / (ub * 1e-3) / 1e12 / 2500.0, 4)})
    if dump:
        # the same union from bench.py's own hipEvents (per launch, relative ms)
        iv = sorted(zip(dump["start_ms"], dump["end_ms"]))
        tot, cs, ce = 0.0, None, None
        for x, y in iv:
            if ce is None or x > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = x, y
            else:
                ce = max(ce, y)
        if ce is not None:
            tot += ce - cs
        out["hipevent_union_ms_per_step"] = round(tot / steps, 3)
        out["hipevent_launches"] = dump["launches"]
    out["per_kernel"] = per_kernel(kws, x3, dump, steps)
    per = defaultdict(lambda: [0, 0])
    for r in rows:
        k = per[r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]]
        k[0] += 1
        k[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    top = sorted(per.items(), key=lambda kv: -kv[1][1])[:20]
    tot_ns = sum(v[1] for v in per.values())
    out["top_kernels"] = [{"kernel": k, "calls": v[0], "ms_per_step": round(v[1] / 1e6 / steps, 3),
                           "avg_us": round(v[1] / v[0] / 1e3, 1), "pct": round(100.0 * v[1] / tot_ns, 2)} for k, v in top]
    if a.fetch and a.write:
        rf = json.load(open(a.fetch_dump))["region_ns"] if a.fetch_dump else None
        rw = json.load(open(a.write_dump))["region_ns"] if a.write_dump else None
        fb, nf = pmc_bytes(a.fetch, "FETCH_SIZE", rf)
        wb, nw = pmc_bytes(a.write, "WRITE_SIZE", rw)
        fb *= 2.0   # gfx950: FETCH_SIZE counts half the bytes of wide (16 B/lane) reads
        # the FETCH pass's records carry durations too, and counter collection serialises the kernels: the same
        # per-kernel table isolated (each launch alone on the GPU), joined with that pass's --prof-dump
        if a.fetch_dump:
            fd = json.load(open(a.fetch_dump))
            frows = [r for r in _csv(a.fetch, "counter_collection.csv") if r.get("Counter_Name", "FETCH_SIZE") == "FETCH_SIZE"]
            fk, fx, _, _ = classify(in_region(frows, fd.get("region_ns")))
            out["per_kernel_isolated"] = [{k: v for k, v in r.items() if k != "hipevent_avg_us"}
                                          for r in per_kernel(fk, fx, fd, fd["steps"])]
            out["per_kernel_isolated_note"] = ("durations from the FETCH_SIZE pass (counter collection serialises the "
                                               "kernels: each launch alone on the GPU); in-bench, three scoring "
                                               "streams share the CUs (per_kernel)")
        out["pmc"] = {"launches_fetch_pass": nf, "launches_write_pass": nw,
                      "fetch_bytes_per_step": fb / steps, "write_bytes_per_step": wb / steps,
                      "bytes_per_step": (fb + wb) / steps,
                      "bytes_per_launch": (fb / max(nf, 1)) + (wb / max(nw, 1)),
                      "correction": "FETCH_SIZE x2 (gfx950), KB -> bytes x1024; fabric-side bytes"}
    js = json.dumps(out, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
