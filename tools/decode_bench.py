"""Whisper decoder step timing (large-v3 by default) at 5 beams: cross-KV precompute per 30 s window and
one decode step per token (KV cache append, self + cross attention, MLP, vocabulary projection), against
the step's HBM roofline (every decoder weight + the KV caches read once per step).
usage: python tools/decode_bench.py [model] [beams] [steps]; DB_POS0=P: the timed steps start at position P (the
keyword-prompted windows of C5 / e2e decode from ~150-230 prefix tokens: self-attention over several key chunks)"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from cbw.decoder import DecoderEngine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
beams = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 64
dev = torch.device("cuda:0")
cfg = synth.WHISPER_DECODERS[model]
V, D, L, H, F = cfg
sd = synth.synth_whisper_decoder_state_dict(model, seed=0)
dec = DecoderEngine(cfg, sd, dev)
enc = torch.randn((1, 1500, D), device=dev)
for _ in range(2):
    dec.start(enc, beams)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5):
    dec.start(enc, beams)
torch.cuda.synchronize()
t_cross = (time.perf_counter() - t) / 5
tok = [50258] * beams
pos0 = int(os.environ.get("DB_POS0", "4"))
dec.start(enc, beams)
for p in range(pos0):
    dec.step(tok, p)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for p in range(pos0, pos0 + steps):
    dec.step(tok, p)
e1.record()
torch.cuda.synchronize()
t_step = e0.elapsed_time(e1) / steps * 1e-3
# bytes per step: bf16 weights of every decoder linear (self qkv/out, cross q/out, fc1, fc2) + the
# vocabulary projection (tied embedding V x D) + self KV caches (mean length, per beam) + the window's
# cross KV (1500 rows, shared by the beams)
w_bytes = 2 * (L * (4 * D * D + 2 * D * D + 2 * D * F) + V * D)
kv_bytes = 2 * L * 2 * D * (beams * (pos0 + steps / 2) + 1500)
bytes_step = w_bytes + kv_bytes
print(f"decoder {model} beams={beams} pos0={pos0} self_split={os.environ.get('CBW_DEC_SELF_SPLIT', '0')}: cross-KV {t_cross * 1e3:.2f} ms/window, step {t_step * 1e3:.3f} ms "
      f"({1 / t_step:.0f} steps/s, {beams / t_step:.0f} beam-tokens/s); {bytes_step / 1e9:.2f} GB/step -> "
      f"{bytes_step / t_step / 1e12:.2f} TB/s = {bytes_step / t_step / 8e12:.1%} of 8 TB/s")
