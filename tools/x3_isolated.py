"""The compensated (x3) re-scoring tier alone on LEF pairs (maps 75 x 750, large-v3 LEF widths), serialised on one
stream: ms per call for X3_N pairs (default 400, the bench's band size).  Under rocprofv3 --kernel-trace, `--seq
TRACE.csv` prints the last call's launches in order (layer by layer) with their durations.
usage: x3_isolated.py | x3_isolated.py --seq run_kernel_trace.csv"""
import csv
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--seq":
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "sim_f32" in r["Kernel_Name"]]
    tot = 0.0
    for r in rows[starts[-1]:]:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += us
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{us:9.1f} us  grid {int(r.get('Grid_Size', 0) or 0) // max(1, int(r.get('Workgroup_Size', 1) or 1)):6d}  {n}")
        if "pool_fc_f32" in n:
            break
    print(f"{tot:9.1f} us total")
    sys.exit(0)

import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.kws import KwsEngine  # noqa: E402

N = int(os.environ.get("X3_N", "400"))
hp = dict(n_layers=3, embedding_dim=1280, learn_features=True, proj_mlp=True, frames_conv=True)
eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
d = eng.device
g = torch.Generator(device=d).manual_seed(0)
kwd = torch.randn((N, 3, 75, 64), generator=g, device=d)
kwd = kwd / kwd.norm(dim=-1, keepdim=True)
utt = torch.randn((3, 750, 64), generator=g, device=d)
utt = utt / utt.norm(dim=-1, keepdim=True)
km, um = torch.ones((N, 3, 75), device=d), torch.ones((3, 750), device=d)
logits = torch.zeros((N, 2), device=d)
sel = torch.arange(N, device=d, dtype=torch.int32)
eng.rescore(utt, um, kwd, km, logits, sel, tier="x3")
torch.cuda.synchronize()
reps = int(os.environ.get("X3_REPS", "5"))
t = time.perf_counter()
for _ in range(reps):
    eng.rescore(utt, um, kwd, km, logits, sel, tier="x3")
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / reps
print(f"x3 tier: {N} pairs in {dt * 1e3:.2f} ms -> {dt * 1e3 / N:.4f} ms per pair")
