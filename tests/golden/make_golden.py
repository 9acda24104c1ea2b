"""Generate golden vectors by running the REFERENCE's own modules (this container
only — /root/reference does not exist on the GPU box).

    python tests/golden/make_golden.py

* KWS: imports ``efficient_kws.model.KWSModel`` from /root/reference/src with
  three host-only stub modules (pytorch_lightning, torchmetrics,
  confidence_intervals; SURVEY.md Appendix B — they touch only training/metric
  code, not ``forward``), loads the seeded state dict from ``cbw.synth`` with
  ``strict=True`` and runs ``forward`` + the ``test_step`` decision
  (model.py:782-799) on seeded inputs.  LEF masks are max-pooled first
  (the reference LEF crashes otherwise).
* mel / encoder: the third-party modules the reference calls
  (HF ``WhisperFeatureExtractor`` — call site src/utils.py:186-187 — and HF
  ``WhisperEncoder`` — call site src/model/cb_whisper.py:100-104), installed
  transformers 5.15.0 (reference pins 4.37.2; drift noted in DESIGN.md).

Only inputs' seeds + outputs are stored; weights/inputs are regenerated from the
seed by ``cbw.synth`` wherever the fixtures are checked.
"""
from __future__ import annotations

import hashlib
import inspect
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "enhance-cb-whisper_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from cbw import synth  # noqa: E402

REF_SRC = "/root/reference/src"

from golden_cases import KWS_CASES, THRESHOLDS  # noqa: E402



def _stub_host_deps():
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(torch.nn.Module):
        def save_hyperparameters(self):
            f = inspect.currentframe().f_back
            a = inspect.getargvalues(f)
            hp = {k: a.locals[k] for k in a.args if k != "self"}
            hp.update(a.locals.get("kwargs", {}))
            self.hparams = types.SimpleNamespace(**hp)

    pl.LightningModule = LightningModule
    pl.LightningDataModule = object
    sys.modules["pytorch_lightning"] = pl
    tm = types.ModuleType("torchmetrics")
    tm.PrecisionRecallCurve = tm.Accuracy = type("N", (), {"__init__": lambda s, *a, **k: None})
    sys.modules["torchmetrics"] = tm
    ci = types.ModuleType("confidence_intervals")
    ci.evaluate_with_conf_int = None
    sys.modules["confidence_intervals"] = ci
    sys.path.insert(0, REF_SRC)


def digest(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def make_kws():
    _stub_host_deps()
    from efficient_kws.model import KWSModel  # reference code, unmodified

    torch.set_num_threads(os.cpu_count() or 8)
    for name, (hp, bk) in KWS_CASES.items():
        model = KWSModel(features_size=(150, 1500), **hp)
        sd = synth.synth_kws_state_dict(seed=0, **hp)
        model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=True)
        model.eval()
        b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
        kwd_mask, utt_mask = torch.from_numpy(b["kwd_mask"]), torch.from_numpy(b["utt_mask"])
        if hp.get("frames_conv"):
            pool = torch.nn.MaxPool1d(3, 2, 1)
            kwd_mask, utt_mask = pool(kwd_mask), pool(utt_mask)
        with torch.inference_mode():
            out = model.forward(kwd_features=torch.from_numpy(b["kwd"]), utt_features=torch.from_numpy(b["utt"]),
                                labels=None, kwd_mask=kwd_mask, utt_mask=utt_mask)
        logits = out.logits.double().numpy()
        feats = out.features.float().numpy()
        probs = (out.logits.softmax(dim=-1)[:, 1] * torch.from_numpy(b["ghost_mask"])).double().numpy()
        rec = dict(logits=logits, probs=probs, feat_shape=np.array(feats.shape),
                   feat_sum=feats.astype(np.float64).sum(axis=(2, 3)),
                   feat_sub=feats[:, :, ::7, ::11].copy(),
                   argmax_idx=torch.argwhere(torch.argmax(out.logits, dim=1)).squeeze(1).numpy(),
                   input_digest=np.array(digest(b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"])))
        if name == "LEF":
            rec["feat_full_k0"] = feats[:1].copy()
        for t in THRESHOLDS:
            rec[f"idx_{t}"] = np.nonzero(probs >= t)[0]
        np.savez_compressed(os.path.join(HERE, f"kws_{name}.npz"), **rec)
        print(name, "logits", logits.round(4).tolist(), "probs", probs.round(4).tolist())


def make_mel():
    from transformers import WhisperFeatureExtractor
    for n_mel in (80, 128):
        fe = WhisperFeatureExtractor(feature_size=n_mel)
        rec = {}
        clips = {"noise_sines": synth.synth_clip(0), "silence": np.zeros(480000, np.float32),
                 "short_7s": synth.synth_clip(2, seconds=7.3)}
        for cname, x in clips.items():
            m = fe(x, sampling_rate=16000, return_tensors="np", padding="max_length").input_features[0]
            if cname == "noise_sines":
                rec[cname] = m.astype(np.float32)
            else:
                rec[cname + "_sub"] = m[:, ::9].astype(np.float32)
                rec[cname + "_sum"] = np.array(m.astype(np.float64).sum())
        np.savez_compressed(os.path.join(HERE, f"mel_{n_mel}.npz"), **rec)
        print("mel", n_mel, {k: v.shape for k, v in rec.items()})


def make_encoder():
    from transformers import WhisperConfig, WhisperFeatureExtractor
    from transformers.models.whisper.modeling_whisper import WhisperEncoder
    n_mel, d, nl, nh, ffn = synth.WHISPER_CONFIGS["micro"]
    cfg = WhisperConfig(num_mel_bins=n_mel, d_model=d, encoder_layers=nl, encoder_attention_heads=nh,
                        encoder_ffn_dim=ffn, decoder_layers=1, decoder_attention_heads=nh, decoder_ffn_dim=ffn,
                        max_source_positions=1500)
    cfg._attn_implementation = "eager"
    enc = WhisperEncoder(cfg)
    sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    enc.eval()
    mel = WhisperFeatureExtractor(feature_size=n_mel)(synth.synth_clip(0), sampling_rate=16000,
                                                       return_tensors="pt").input_features
    with torch.inference_mode():
        hs = enc(input_features=mel, output_hidden_states=True, return_dict=True)["hidden_states"]
    hs = torch.stack(hs, 0)[:, 0].float().numpy()
    np.savez_compressed(os.path.join(HERE, "encoder_micro.npz"), hidden_states=hs, mel=mel[0].numpy())
    print("encoder", hs.shape)


if __name__ == "__main__":
    what = sys.argv[1:] or ["kws", "mel", "encoder"]
    if "mel" in what:
        make_mel()
    if "encoder" in what:
        make_encoder()
    if "kws" in what:
        make_kws()
