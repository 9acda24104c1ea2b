"""End-to-end CB-Whisper window on one MI355X (config C5's per-window work at bf16): for each synthetic
30 s window, log-mel -> large-v3 encoder (hidden states for the spotter) -> LEF utterance projection ->
10 000-keyword LEF/ResNet-50 scoring -> argmax decision -> keyword prompt (<|startofprev|> + the top spotted
keywords' tokens, capped) -> the generation encoder pass -> cross-KV -> HF 4.37 beam search (5 beams) on the
GPU decoder, at most MAX_NEW tokens.  Seeded random weights, so the transcripts are meaningless and the
number of generated tokens is whatever the synthetic decoder produces (printed); the timing splits spotting
from decoding so per-token costs can be compared with tools/decode_bench.py.
usage: python tools/e2e_bench.py [windows] [max_new_tokens]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from bench import build_keyword_db  # noqa: E402
from cbw import synth  # noqa: E402
from cbw.kws import KwsEngine, spot  # noqa: E402
from cbw.whisper import default_layer_ids, log_mel  # noqa: E402
from model.pba_whisper import PBAWhisper  # noqa: E402

windows = int(sys.argv[1]) if len(sys.argv) > 1 else 4
max_new = int(sys.argv[2]) if len(sys.argv) > 2 else 128
K, beams, prompt_cap = 10000, 5, 32
dev = torch.device("cuda:0")
enc_cfg, dec_cfg = synth.WHISPER_CONFIGS["large-v3"], synth.WHISPER_DECODERS["large-v3"]
sd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict("large-v3", seed=0).items()}
sd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict("large-v3", seed=0).items()})
whisper = PBAWhisper(enc_cfg, dec_cfg, sd, device=dev)
del sd
hp = dict(n_layers=3, embedding_dim=enc_cfg[1], learn_features=True, proj_mlp=True, frames_conv=True,
          proj_mlp_units=64, resnet_version="resnet-50")
kws = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp), dev)
db, dbm = build_keyword_db(kws, K, enc_cfg[1])
ids = default_layer_ids(enc_cfg[2])
n_mel = enc_cfg[0]
kw_tokens = lambda i: [1000 + (i * 7919) % 40000, 1000 + (i * 104729) % 40000]   # noqa: E731  synthetic spellings


def window(i):
    t = {}
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    pcm = torch.from_numpy(synth.synth_clip(i)).to(dev)
    e[0].record()
    _, pk = log_mel(pcm, n_mel, packed=True)
    hs = whisper.encoder.hidden_states(pk, ids, normalize=True)
    u, um = kws.project(hs, torch.ones((1, 3, 1500), device=dev))
    logits = kws.score(u[0], um[0], db, dbm, chunk=625)
    _, idx = spot(logits, None, 0.5, mode="argmax")
    e[1].record()
    spotted = sorted(set(idx.tolist()))
    prompt = [whisper.tokens.startofprev] + [t for k in spotted[:prompt_cap] for t in kw_tokens(k)]
    prefix = prompt + whisper.tokens.init_tokens("english", "transcribe", False)
    enc = whisper.encode(pk.unsqueeze(0) if pk.dim() == 2 else pk)
    e[2].record()
    seq = whisper.decode_window(enc, prefix, beams, max_new_tokens=max_new)
    e[3].record()
    torch.cuda.synchronize()
    t["spot_ms"] = e[0].elapsed_time(e[1])
    t["gen_encoder_ms"] = e[1].elapsed_time(e[2])
    t["decode_ms"] = e[2].elapsed_time(e[3])
    t["new_tokens"] = len(seq) - len(prefix)
    t["spotted"] = len(spotted)
    return t


window(0)   # warm-up
t0 = time.perf_counter()
rows = [window(1 + i) for i in range(windows)]
wall = time.perf_counter() - t0
toks = sum(r["new_tokens"] for r in rows)
dec = sum(r["decode_ms"] for r in rows)
print(f"e2e large-v3 + LEF {K} kw, beam {beams}: {windows / wall:.3f} windows/s ({wall / windows * 1e3:.0f} ms/window); "
      f"spotting {sum(r['spot_ms'] for r in rows) / windows:.1f} ms, generation encoder "
      f"{sum(r['gen_encoder_ms'] for r in rows) / windows:.1f} ms, decoding {dec / windows:.0f} ms for "
      f"{toks / windows:.0f} tokens/window ({dec / max(toks, 1):.2f} ms/token incl. host beam search); "
      f"30-min audio (60 windows) ~{60 * wall / windows:.0f} s on one GPU")
