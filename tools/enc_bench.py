"""Whisper encoder timing (large-v3 by default, all layers, one 30 s clip per call) on cuda:0: the mean of N calls of
EncoderEngine.hidden_states after warm-up.  usage: python tools/enc_bench.py [model] [N]  (CBW_ENC_ATTN_V1=1: the
unpipelined attention kernel)"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.whisper import EncoderEngine, log_mel  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = synth.WHISPER_CONFIGS[name]
eng = EncoderEngine(cfg, synth.synth_whisper_encoder_state_dict(name, seed=0))
_, pk = log_mel(torch.from_numpy(synth.synth_clip(1)).to(eng.device), cfg[0], packed=True)
ids = list(range(cfg[2] + 1))[-3:]
for _ in range(3):
    eng.hidden_states(pk, ids)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(n):
    eng.hidden_states(pk, ids)
torch.cuda.synchronize()
print(f"encoder {name}: {(time.perf_counter() - t) / n * 1e3:.3f} ms per clip "
      f"(CBW_ENC_ATTN_V1={os.environ.get('CBW_ENC_ATTN_V1', '0')})")
