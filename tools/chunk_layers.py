"""One scoring chunk's conv launches in order, with isolated durations, from a rocprofv3 --pmc pass over bench.py
(the counter passes serialise the kernels): the launches of one queue between two stem launches, each named by its
ResNet-50 layer (LEF maps [3, 75, 750]) and priced against max(MFMA at 1.1 PF, HBM bytes at 5.5 TB/s).
usage: [CHUNK_PAIRS=834] python tools/chunk_layers.py DIR [chunk_index]  (CHUNK_PAIRS = bench.py --chunk of the pass)"""
import collections
import os
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
want = int(sys.argv[2]) if len(sys.argv) > 2 else 3
disp = {}
for r in csv.DictReader(open(f)):
    k = int(r["Dispatch_Id"])
    if k not in disp:
        disp[k] = (r["Queue_Id"], re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")[:44],
                   int(r["Grid_Size"]) // int(r["Workgroup_Size"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
byq = collections.defaultdict(list)
for k in sorted(disp):
    byq[disp[k][0]].append(disp[k])
P = int(os.environ.get("CHUNK_PAIRS", "834"))
layers = ["stem+pool", "s1b0 fused", "s1b1 fused", "s1b2 fused", "s2b0 reduce", "s2b0 3x3s2", "s2b0 expand+sc"]
layers += [f"s2b{b} {n}" for b in (1, 2, 3) for n in ("reduce", "3x3", "expand+res")]
layers += ["s3b0 reduce", "s3b0 3x3s2", "s3b0 expand+sc"] + [f"s3b{b} {n}" for b in range(1, 6) for n in ("reduce", "3x3", "expand+res")]
layers += ["s4b0 reduce", "s4b0 3x3s2", "s4b0 expand+sc"] + [f"s4b{b} {n}" for b in (1, 2) for n in ("reduce", "3x3", "expand+res")]
# (M, N, K, bytes) per layer per pair for the roofline price
def shapes():
    out = [(38 * 375, 64, 147, (75 * 750 * 8 + 19 * 188 * 128))]
    H, W, cin = 19, 188, 64
    for st, (mid, co, nb) in enumerate([(64, 256, 3), (128, 512, 4), (256, 1024, 6), (512, 2048, 3)]):
        for b in range(nb):
            s = 2 if (b == 0 and st > 0) else 1
            Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
            if st == 0:
                k = cin * 64 + 576 * 64 + 64 * co + (cin * co if b == 0 else 0)
                out.append((H * W, 1, k, 2 * (H * W * cin + H * W * co)))
            else:
                out.append((H * W, mid, cin, 2 * (H * W * cin + H * W * mid)))
                out.append((Ho * Wo, mid, 9 * mid, 2 * (H * W * mid + Ho * Wo * mid)))
                kk = mid + (cin if b == 0 else 0)
                out.append((Ho * Wo, co, kk, 2 * (Ho * Wo * mid + (Ho * Wo * cin if b == 0 else 2 * Ho * Wo * co) + Ho * Wo * co)))
            H, W, cin = Ho, Wo, co
    return out
sh = shapes()
for q, l in byq.items():
    st = [i for i, x in enumerate(l) if x[1].startswith("stem_pool")]
    if len(st) <= want:
        continue
    seq = l[st[want]:st[want + 1]] if want + 1 < len(st) else l[st[want]:]
    if os.environ.get("RAW"):   # RAW=1: the chunk's launches as recorded (any pass: the fp8 tier's chunk too)
        for _, n, g, d in seq:
            print(f"{n:44s} grid={g:5d} {d:7.1f}us")
        print(f"chunk total {sum(x[3] for x in seq):.0f} us over {len(seq)} launches ({P} pairs)")
        break
    tot = totr = 0.0
    for i, (_, n, g, d) in enumerate(seq[:len(layers)]):
        M, N, K, B = sh[i]
        fl = 2.0 * M * N * K * P
        t_roof = max(fl / 1.1e15, B * P / 5.5e12) * 1e6
        tot += d
        totr += t_roof
        print(f"{layers[i]:18s} {n:44s} grid={g:5d} {d:7.1f}us  {fl / d / 1e6:6.0f}TF/s {B * P / d / 1e6:5.2f}TB/s  roof {t_roof:6.1f}us x{d / t_roof:4.2f}")
    print(f"chunk total {tot:.0f} us, roofline {totr:.0f} us ({P} pairs: {tot / P:.2f} us per pair)")
    break
