"""Audit inline-asm VGPR loads in a hipcc -save-temps .s file: every read of an asm load's
destination register must come after an asm `s_waitcnt vmcnt` (cdna_hip_programming.md §5.7
item 1: hipcc treats the destination as written at ASMEND).  Linear scan per kernel -- a
heuristic over the layout order, not the CFG; prints suspicious reads.
usage: python tools/audit_asm_loads.py file.s"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
bad = 0
pending = {}   # reg range -> line of the asm load
in_asm = False
for i, l in enumerate(lines):
    t = l.strip()
    if t.startswith(";;#ASMSTART"):
        in_asm = True
        continue
    if t.startswith(";;#ASMEND"):
        in_asm = False
        continue
    if t.startswith(".section") or t.endswith(":") and not t.startswith("."):
        if re.match(r"^_Z.*:$", t):
            pending.clear()
    if in_asm:
        m = re.match(r"global_load_dwordx?\d*\s+(v\[\d+:\d+\]|v\d+),", t)
        if m:
            pending[m.group(1)] = i + 1
        elif t.startswith("s_waitcnt") and "vmcnt" in t:
            pending.clear()
        continue
    if not pending or not t or t.startswith(";"):
        continue
    parts = t.split(None, 1)
    if len(parts) < 2:
        continue
    ops = parts[1].split(",")
    srcs = ",".join(ops[1:]) if not parts[0].startswith(("global_store", "buffer_store", "ds_write")) else parts[1]
    for r, ln in list(pending.items()):
        if r in srcs:
            print(f"line {i + 1}: reads {r} loaded at line {ln} before any asm vmcnt wait: {t}")
            bad += 1
        if r in ops[0] and not parts[0].startswith(("global_store", "buffer_store", "ds_write", "s_")):
            pending.pop(r, None)   # overwritten
print("suspicious reads:", bad)
sys.exit(1 if bad else 0)
