"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel family.

usage: python tools/pmc_summary.py gpurun_out/pmc_TAG_FETCH_SIZE gpurun_out/pmc_TAG_WRITE_SIZE [name-substring ...]

FETCH_SIZE and WRITE_SIZE are in KB (rocprofv3 derived counters).  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, global_load and buffer/global_load ... lds alike, so
it is doubled here; WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits are
counted as fetches, so these are fabric-side bytes, an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f[0])):
        k = out[r["Kernel_Name"]]
        k[0] += 1
        k[1] += float(r["Counter_Value"])
    return out


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    pats = sys.argv[3:] or ["conv_igemm|conv_ring|conv_stream|bottleneck"]   # '|' = any of (one family)
    res = {}
    for p in pats:
        alts = p.split("|")
        hit = lambda k: any(a in k for a in alts)   # noqa: E731
        n = sum(v[0] for k, v in fetch.items() if hit(k))
        fb = 2 * 1024 * sum(v[1] for k, v in fetch.items() if hit(k))
        wb = 1024 * sum(v[1] for k, v in write.items() if hit(k))
        res[p] = {"launches": n, "fetch_bytes": fb, "write_bytes": wb,
                  "bytes_per_launch": (fb + wb) / max(1, n)}
    per = defaultdict(dict)
    for k, v in fetch.items():
        per[k]["n"] = v[0]
        per[k]["fetch_MB"] = round(2 * v[1] / 1024, 1)
    for k, v in write.items():
        per[k]["write_MB"] = round(v[1] / 1024, 1)
    for k, v in sorted(per.items(), key=lambda kv: -kv[1].get("fetch_MB", 0))[:15]:
        print(f"{k[:80]:80s} n={v.get('n')} fetch {v.get('fetch_MB')} MB write {v.get('write_MB')} MB")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
