"""Time the fp32 re-scoring path (cbw_kws_rescore) on LEF pairs (large-v3 D, maps 75x750)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.kws import KwsEngine  # noqa: E402

N = int(os.environ.get("RS_N", "64"))
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
eng.rescore(utt, um, kwd, km, logits, sel)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    eng.rescore(utt, um, kwd, km, logits, sel)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 3
print(f"fp32 re-score: {N} pairs in {dt * 1e3:.1f} ms -> {N / dt:.0f} pairs/s, {N * 10.08e9 / dt / 1e12:.1f} TFLOP/s")
