"""Near-threshold statistics at the bench operating point (large-v3 + LEF, 10k keywords).

For one synthetic clip through the bench path: the distribution of |p_bf16 - thr| over all K pairs
(how many pairs a band of half-width delta holds), and on a random sample of pairs the bf16-vs-fp32
probability error (how wide the band must be for the re-scored decisions to equal the fp32 ones).
Also times the fp32 re-score per pair.  Prints one JSON line.

BS_CAL=n (> 0): then the same statistics again after KwsEngine.calibrate_bias on the database's first n keywords
against a calibration clip that is never scored (id 999 999; bench.py's calibration), under "clips_cal".
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
import bench  # noqa: E402
from cbw import synth  # noqa: E402
from cbw.kws import KwsEngine  # noqa: E402
from cbw.whisper import EncoderEngine, default_layer_ids, log_mel  # noqa: E402

K = int(os.environ.get("BS_K", "10000"))
NS = int(os.environ.get("BS_SAMPLE", "512"))
thr = float(os.environ.get("BS_THR", "0.5"))
dev = torch.device("cuda:0")
cfg = synth.WHISPER_CONFIGS["large-v3"]
n_mel, D, nl, _, _ = cfg
enc = EncoderEngine(cfg, synth.synth_whisper_encoder_state_dict("large-v3", seed=0), dev)
hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True, proj_mlp_units=64,
          resnet_version="resnet-50", threshold=thr)
kws = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp), dev)
db, dbm, db32 = bench.build_keyword_db(kws, K, D, f32=True)
out = {"K": K, "threshold": thr, "clips": []}
um = torch.ones((1, 3, 1500), device=dev)


def clip_proj(clip):
    _, pk = log_mel(torch.from_numpy(synth.synth_clip(clip)).to(dev), n_mel, packed=True)
    hs = enc.hidden_states(pk, default_layer_ids(nl), normalize=True)
    pu, pum = kws.project(hs, um)
    pu32, _ = kws.project_f32(hs, um)
    return pu, pum, pu32


def eval_clip(clip, key):
    pu, pum, pu32 = clip_proj(clip)
    logits = kws.score(pu[0], pum[0], db, dbm, chunk=625)
    p = torch.softmax(logits, -1)[:, 1]
    dist = (p - thr).abs()
    counts = {str(d): int((dist <= d).sum()) for d in (0.001, 0.003, 0.01, 0.02, 0.03, 0.05, 0.1)}
    g = torch.Generator(device="cpu").manual_seed(clip)
    sel = torch.randperm(K, generator=g)[:NS].sort().values.to(dev, torch.int32)
    l32 = logits.clone()
    torch.cuda.synchronize()
    t = time.perf_counter()
    kws.rescore(pu32[0], pum[0], db32, dbm, l32, sel)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    p32 = torch.softmax(l32, -1)[:, 1]
    lx3 = logits.clone()
    kws.rescore(pu32[0], pum[0], db32, dbm, lx3, sel, tier="x3")
    torch.cuda.synchronize()
    t = time.perf_counter()
    kws.rescore(pu32[0], pum[0], db32, dbm, lx3, sel, tier="x3")
    torch.cuda.synchronize()
    dtx3 = time.perf_counter() - t
    px3 = torch.softmax(lx3, -1)[:, 1]
    s = sel.long()
    if os.environ.get("BS_DUMP"):   # per-pair logits of the sample (bf16 and fp32) for offline error models
        import numpy as np
        np.savez(f"{os.environ['BS_DUMP']}_{key}_{clip}.npz", sel=sel.cpu().numpy(), bf16=logits[s].cpu().numpy(),
                 fp32=l32[s].cpu().numpy())
    ex3 = (px3[s] - p32[s]).abs()
    err = (p[s] - p32[s]).abs()
    lerr = (logits[s] - l32[s]).abs().max(dim=1).values
    flips = int(((p[s] >= thr) != (p32[s] >= thr)).sum())
    out[key].append({
        "clip": clip, "band_counts": counts, "p_quantiles": [round(float(x), 4) for x in
                                                          torch.quantile(p.float(), torch.tensor([0.01, 0.1, 0.5, 0.9, 0.99], device=dev))],
        "spotted": int((p >= thr).sum()),
        "sample": NS, "prob_err_max": float(err.max()), "prob_err_p99": float(torch.quantile(err, 0.99)),
        "logit_err_max": float(lerr.max()), "flips_in_sample": flips,
        "rescore_ms_per_pair": dt * 1e3 / NS,
        "x3_prob_err_max": float(ex3.max()), "x3_logit_err_max": float((lx3[s] - l32[s]).abs().max()),
        "x3_flips_in_sample": int(((px3[s] >= thr) != (p32[s] >= thr)).sum()),
        "x3_ms_per_pair": dtx3 * 1e3 / NS})
n_clips = int(os.environ.get("BS_CLIPS", "2"))
for clip in range(n_clips):
    eval_clip(clip, "clips")
n_cal = int(os.environ.get("BS_CAL", "0"))
if n_cal > 0:
    # as bench.py --bias-calibrate: the database's first n_cal keywords vs clip 999 999 (never scored here)
    pu, pum, pu32 = clip_proj(999_999)
    cal = torch.arange(min(n_cal, K), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    off = kws.calibrate_bias(pu32[0], pum[0], db32, dbm, cal,
                             **({} if os.environ.get("BS_NO_OFFSET") else dict(utt=pu[0], kwd=db)))
    out["logit_offset"] = None if off is None else [float(v) for v in off]
    out["calibration"] = {"pairs": n_cal, "clip": 999_999, "keywords": "first", "s": round(time.perf_counter() - t, 3)}
    out["clips_cal"] = []
    for clip in range(n_clips):
        eval_clip(clip, "clips_cal")
print(json.dumps(out), flush=True)
