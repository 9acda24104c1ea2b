"""Run the LEF ResNet-50 classifier once on K random maps (for rocprofv3 kernel/PMC passes)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.kws import KwsEngine  # noqa: E402

K = int(os.environ.get("CO_K", "1000"))
REPS = int(os.environ.get("CO_REPS", "2"))
hp = dict(n_layers=3, embedding_dim=1280, learn_features=True, proj_mlp=True, frames_conv=True)
eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
g = torch.Generator(device=eng.device)
g.manual_seed(0)
maps = torch.rand((K, 3, 75, 750), generator=g, device=eng.device) * 2 - 1
for _ in range(REPS):
    logits = eng.classify(maps, chunk=500)
torch.cuda.synchronize()
print("ok", float(logits.abs().sum()))
