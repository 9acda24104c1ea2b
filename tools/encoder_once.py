"""Run the Whisper-large-v3 encoder (all layers) on one synthetic clip a few times (rocprofv3 kernel
traces of the encoder alone).  usage: python tools/encoder_once.py [model]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.whisper import EncoderEngine, default_layer_ids, log_mel  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
B = int(os.environ.get("ENC_B", "1"))
dev = torch.device("cuda:0")
cfg = synth.WHISPER_CONFIGS[model]
enc = EncoderEngine(cfg, synth.synth_whisper_encoder_state_dict(model, seed=0), dev)
ids = default_layer_ids(cfg[2])
_, pk = log_mel(torch.from_numpy(synth.synth_clip(0)).to(dev), cfg[0], packed=True)
pk = pk.unsqueeze(0).expand(B, -1, -1).contiguous()
for _ in range(2):
    hs = enc.hidden_states(pk, ids)
torch.cuda.synchronize()
t = time.time()
for _ in range(5):
    hs = enc.hidden_states(pk, ids)
torch.cuda.synchronize()
print(f"encoder {model} B={B}: {(time.time() - t) / 5 * 1e3:.2f} ms per call", float(hs.abs().sum()))
