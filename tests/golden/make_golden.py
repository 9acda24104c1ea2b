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


BEAM_PREFIX = [50361, 1000, 1001, 1002, 50258, 50259, 50359, 50363]
SUPPRESS = [1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93, 359, 503, 522, 542, 873]
DECODER_TOKENS = [50361] + list(range(1000, 1012)) + [50258, 50259, 50359, 50363] + list(range(3000, 3040, 2))


def make_decoder():
    """Teacher-forced decoder logits of HF WhisperForConditionalGeneration (micro config,
    seeded encoder + decoder weights) for a prompt-injected token sequence laid out as
    PBAWhisper builds it: <|startofprev|> keyword tokens <|startoftranscript|> <|en|>
    <|transcribe|> <|notimestamps|> text (pba_whisper.py:283-338, :478-548)."""
    from transformers import WhisperConfig, WhisperFeatureExtractor, WhisperForConditionalGeneration
    n_mel, d, nl, nh, ffn = synth.WHISPER_CONFIGS["micro"]
    V, dd, dnl, dnh, dffn = synth.WHISPER_DECODERS["micro"]
    cfg = WhisperConfig(vocab_size=V, num_mel_bins=n_mel, d_model=d, encoder_layers=nl, encoder_attention_heads=nh,
                        encoder_ffn_dim=ffn, decoder_layers=dnl, decoder_attention_heads=dnh, decoder_ffn_dim=dffn,
                        max_source_positions=1500, max_target_positions=448)
    cfg._attn_implementation = "eager"
    model = WhisperForConditionalGeneration(cfg)
    sd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict("micro", seed=0).items()}
    sd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict("micro", seed=0).items()})
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all("proj_out" in m for m in missing), (missing, unexpected)
    model.eval()
    mel = WhisperFeatureExtractor(feature_size=n_mel)(synth.synth_clip(0), sampling_rate=16000,
                                                       return_tensors="pt").input_features
    tok = torch.tensor([DECODER_TOKENS])
    with torch.inference_mode():
        enc = model.model.encoder(input_features=mel).last_hidden_state
        logits = model(encoder_outputs=(enc,), decoder_input_ids=tok).logits[0].double().numpy()
    top_v, top_i = torch.from_numpy(logits).topk(20, dim=-1)
    lse = torch.logsumexp(torch.from_numpy(logits), dim=-1).numpy()
    # beam search (num_beams=5) through GenerationMixin.generate, as PBAWhisper's short-form path
    # does (pba_whisper.py:323-331); transformers 5.15 semantics: decoder_prompt_len = len(prefix)
    from transformers import GenerationConfig
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin
    gc = GenerationConfig(decoder_start_token_id=BEAM_PREFIX[0], eos_token_id=50257, pad_token_id=50257, num_beams=5,
                          do_sample=False, max_new_tokens=24, suppress_tokens=SUPPRESS, begin_suppress_tokens=[220, 50257],
                          length_penalty=1.0, early_stopping=False)
    with torch.inference_mode():
        beam = super(WhisperGenerationMixin, model).generate(input_features=mel, decoder_input_ids=torch.tensor(
            [BEAM_PREFIX]), generation_config=gc)[0].numpy()
    print("beam", beam.tolist())
    np.savez_compressed(os.path.join(HERE, "decoder_micro.npz"), tokens=np.array(DECODER_TOKENS),
                        beam_prefix=np.array(BEAM_PREFIX), beam_out=beam, suppress=np.array(SUPPRESS),
                        enc_out=enc[0].float().numpy(), top_v=top_v.numpy(), top_i=top_i.numpy(), lse=lse,
                        logits_last=logits[-1].astype(np.float32), logits_16=logits[16].astype(np.float32))
    print("decoder", logits.shape, "top1", top_i[:, 0].tolist())


KWDB_LENGTHS = [17, None, 160, 40, 9, None, 150, 151, 33]   # None = ghost (no .bin)


def kwdb_inputs():
    """Seeded keyword hs as utils.py:188-201 stores them: fp32 [12, T, D], per-frame L2-normalised."""
    g = np.random.default_rng(7)
    out = []
    for T in KWDB_LENGTHS:
        if T is None:
            out.append(None)
            continue
        x = g.standard_normal((12, T, 8)).astype(np.float32)
        out.append(x / np.linalg.norm(x, axis=-1, keepdims=True))
    return out


def make_kwdb():
    """efficient_kws.dataset.ACL6060KeywordDataset (reference code, unmodified) on a synthetic
    split folder: keyword database load, ghosts, groups of 4, pad/truncate to 150 frames
    (efficient_kws/dataset.py:1677-1796).  Module-level imports it does not use on this path
    (torchvision, torchaudio, whisper.audio) are stubbed."""
    import tempfile
    from transformers import WhisperFeatureExtractor  # noqa: F401  (resolved before the stubs below exist)
    _stub_host_deps()
    for name in ("torchvision", "torchaudio"):
        sys.modules.setdefault(name, types.ModuleType(name))
    wa = types.ModuleType("whisper.audio")
    wa.SAMPLE_RATE, wa.N_SAMPLES = 16000, 480000
    sys.modules.setdefault("whisper", types.ModuleType("whisper"))
    sys.modules["whisper.audio"] = wa
    from efficient_kws.dataset import ACL6060KeywordDataset
    hs = kwdb_inputs()
    keywords = [f"kw{i}" for i in range(len(hs))]
    with tempfile.TemporaryDirectory() as root:
        sf = os.path.join(root, "2", "acl_6060", "dev")
        for d in ("text/tagged_terminology", "text/txt", "text/xml", "keywords-hs/tts"):
            os.makedirs(os.path.join(sf, d))
        open(os.path.join(sf, "text/keywords.txt"), "w").write("\n".join(keywords) + "\n")
        open(os.path.join(sf, "text/txt/ACL.6060.dev.en-xx.en.txt"), "w").write("we use kw2 here\nnothing\n")
        open(os.path.join(sf, "text/tagged_terminology/ACL.6060.dev.tagged.en-xx.en.txt"), "w").write(
            "we use [kw2] here\nnothing\n")
        open(os.path.join(sf, "text/xml/ACL.6060.dev.en-xx.en.xml"), "w").write(
            '<m><s><doc><seg id="1">a</seg><seg id="2">b</seg></doc></s></m>')
        width = len(str(len(keywords) - 1))
        for i, x in enumerate(hs):
            if x is not None:
                with open(os.path.join(sf, "keywords-hs/tts", str(i).zfill(width) + ".bin"), "wb") as f:
                    torch.save(torch.from_numpy(x), f)
        ds = ACL6060KeywordDataset(root, split="dev", size=(150, 1500), keywords_per_group=4, kw_type="tts")
    rec = {"n_groups": np.array(len(ds.database))}
    for gi, g in enumerate(ds.database):
        rec[f"g{gi}_keywords"] = np.array(g["keywords"])
        rec[f"g{gi}_mask"] = g["mask"].numpy()
        rec[f"g{gi}_max_length"] = np.array(g["max_length"])
        rec[f"g{gi}_kwd"] = torch.stack(g["kwd"]).numpy()
        rec[f"g{gi}_kwd_mask"] = torch.stack(g["kwd_mask"]).numpy()
        rec[f"g{gi}_hs_lengths"] = np.array([h.shape[1] for h in g["hidden_states"]])
    np.savez_compressed(os.path.join(HERE, "kwdb_acl.npz"), **rec)
    print("kwdb", {k: v.shape for k, v in rec.items()})


CNN12_TK = [9, 40, 150, 171, 1]


def cnn12_inputs(D: int = 128):
    """Seeded, per-frame L2-normalised hs: utterance [12, 1500, D], keywords [12, Tk, D]."""
    g = np.random.default_rng(11)

    def nrm(x):
        return (x / np.linalg.norm(x, axis=-1, keepdims=True)).astype(np.float32)
    utt = nrm(g.standard_normal((12, 1500, D)))
    kwd = [nrm(g.standard_normal((12, T, D))) for T in CNN12_TK]
    kwd[1][:, 10:30] = utt[:, 400:420]          # one planted match
    kwd[1] = nrm(kwd[1])
    return utt, kwd


def make_cnn12():
    """CB-Whisper's own spotter: similarity matrices (cb_whisper.py:196), resize to (150, 750)
    (cb_whisper.py:206; torchvision's tensor resize = F.interpolate bilinear, align_corners=False,
    antialias=False — torchvision is not installed, the stand-in is that kernel), and the
    reference's model.model.KWSModel forward (12-channel ResNet-50, model/model.py:55-93)."""
    _stub_host_deps()
    for m in [k for k in sys.modules if k == "model" or k.startswith("model.")]:
        del sys.modules[m]
    # the reference's src/model is a namespace package: our regular package of the same name
    # (enhance-cb-whisper_amd/model) would win the lookup, so it leaves sys.path for this import
    pkg = os.path.join(REPO, "enhance-cb-whisper_amd")
    saved = list(sys.path)
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != pkg]
    try:
        from model.model import KWSModel as CBKWSModel   # reference code, unmodified
    finally:
        sys.path[:] = saved
    hp = dict(n_layers=12, embedding_dim=128, learn_features=False, proj_mlp=False)
    model = CBKWSModel()
    sd = synth.synth_kws_state_dict(seed=3, **hp)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=True)
    model.eval()
    utt, kwd = cnn12_inputs()
    torch.set_num_threads(os.cpu_count() or 8)
    with torch.inference_mode():
        u = torch.from_numpy(utt)[None]                                        # [S=1, 12, 1500, D]
        sims = [torch.matmul(torch.from_numpy(k), u.transpose(2, 3))[0] for k in kwd]
        maps = torch.stack([torch.nn.functional.interpolate(m[None], size=(150, 750), mode="bilinear",
                                                            align_corners=False, antialias=False)[0] for m in sims])
        out = model.forward(input_features=maps)
    logits = out.logits.double().numpy()
    rec = dict(logits=logits, argmax_idx=torch.argwhere(torch.argmax(out.logits, dim=1)).squeeze(1).numpy(),
               maps_sum=maps.double().sum(dim=(2, 3)).numpy(), maps_k1_sub=maps[1, :, ::7, ::11].numpy(),
               tk=np.array(CNN12_TK))
    np.savez_compressed(os.path.join(HERE, "cnn12.npz"), **rec)
    print("cnn12 logits", logits.round(4).tolist())


LONGFORM_CLIPS = (0, 1, 2)          # synth clips concatenated (the last one cut to 10 s): 70 s of audio


def longform_hf_model():
    from transformers import GenerationConfig, WhisperConfig, WhisperForConditionalGeneration
    n_mel, d, nl, nh, ffn = synth.WHISPER_CONFIGS["micro"]
    V, dd, dnl, dnh, dffn = synth.WHISPER_DECODERS["micro"]
    cfg = WhisperConfig(vocab_size=V, num_mel_bins=n_mel, d_model=d, encoder_layers=nl, encoder_attention_heads=nh,
                        encoder_ffn_dim=ffn, decoder_layers=dnl, decoder_attention_heads=dnh, decoder_ffn_dim=dffn,
                        max_source_positions=1500, max_target_positions=448)
    cfg._attn_implementation = "eager"
    model = WhisperForConditionalGeneration(cfg)
    sd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict("micro", seed=0).items()}
    sd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict("micro", seed=0).items()})
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    model.eval()
    model.generation_config = GenerationConfig(
        decoder_start_token_id=50258, eos_token_id=50257, pad_token_id=50257, bos_token_id=50257,
        no_timestamps_token_id=50363, is_multilingual=True, lang_to_id={"<|en|>": 50259},
        task_to_id={"transcribe": 50359, "translate": 50358}, suppress_tokens=[1, 2, 7],
        begin_suppress_tokens=[220, 50257], max_initial_timestamp_index=50, prev_sot_token_id=50361, max_length=448)
    return model


def make_longform():
    """Long-form generation with timestamps (the seek loop PBAWhisper.generate runs for > 30 s of audio,
    pba_whisper.py:343-475): transformers 5.15 WhisperForConditionalGeneration.generate on the micro model
    (seeded weights), greedy, return_timestamps=True, no condition on previous tokens.  Recorded per window
    (by wrapping generate_with_fallback / _get_input_segment): seek, window length, decoder prompt, the
    window's tokens after the post-processing; plus the final sequence and segments."""
    from transformers import WhisperFeatureExtractor
    from transformers.models.whisper import generation_whisper as gw
    model = longform_hf_model()
    n_mel = synth.WHISPER_CONFIGS["micro"][0]
    clip = np.concatenate([synth.synth_clip(LONGFORM_CLIPS[0]), synth.synth_clip(LONGFORM_CLIPS[1]),
                           synth.synth_clip(LONGFORM_CLIPS[2])[:160000]])
    feat = WhisperFeatureExtractor(feature_size=n_mel)(clip, sampling_rate=16000, return_tensors="pt",
                                                        truncation=False, padding="longest", return_attention_mask=True)
    log = {"seek": [], "nframes": [], "prefix": [], "window": []}
    orig_seg = gw.WhisperGenerationMixin._get_input_segment
    orig_fb = gw.WhisperGenerationMixin.generate_with_fallback

    def seg_hook(input_features, seek, seek_num_frames, *a, **k):
        log["seek"].append(int(seek[0]))
        log["nframes"].append(int(seek_num_frames[0]))
        return orig_seg(input_features, seek, seek_num_frames, *a, **k)

    def fb_hook(self, *a, **k):
        out = orig_fb(self, *a, **k)
        log["prefix"].append(k["decoder_input_ids"][0].tolist())
        log["window"].append(out[0][0].tolist())
        return out

    gw.WhisperGenerationMixin._get_input_segment = staticmethod(seg_hook)
    gw.WhisperGenerationMixin.generate_with_fallback = fb_hook
    try:
        with torch.inference_mode():
            out = model.generate(input_features=feat.input_features, attention_mask=feat.attention_mask,
                                 return_timestamps=True, return_segments=True, language="en", task="transcribe",
                                 condition_on_prev_tokens=False, num_beams=1)
    finally:
        gw.WhisperGenerationMixin._get_input_segment = staticmethod(orig_seg)
        gw.WhisperGenerationMixin.generate_with_fallback = orig_fb
    segs = out["segments"][0]
    W = len(log["window"])
    pad = lambda rows: np.array([r + [-1] * (max(map(len, rows)) - len(r)) for r in rows])   # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "longform_micro.npz"), features=feat.input_features[0].numpy().astype(np.float32),
        seek=np.array(log["seek"]), nframes=np.array(log["nframes"]), prefix=pad(log["prefix"]),
        window=pad(log["window"]), sequence=out["sequences"][0].numpy(),
        seg_start=np.array([float(s["start"]) for s in segs]), seg_end=np.array([float(s["end"]) for s in segs]),
        seg_tokens=pad([s["tokens"].tolist() for s in segs]))
    print("longform: windows", W, "seek", log["seek"], "segments", len(segs), "tokens", out["sequences"].shape)


LONGFORM_KEYWORDS = [2000 + 7 * i for i in range(12)]   # a fixed keyword prompt for every window


def make_longform_keywords():
    """Long-form with a keyword prompt in every window and conditioning on the previous windows (the C5 path:
    PBAWhisper.generate(condition_on_prev_tokens=True) with keyword_spotting, pba_whisper.py:343-475): transformers
    5.15 long-form generate on the micro model with prompt_ids = <|startofprev|> + LONGFORM_KEYWORDS and
    prompt_condition_type="all-segments" (5.15's way of keeping a prompt in front of every window's previous-text
    context), greedy, timestamps, the longform_micro audio.  Recorded per window as make_longform does: seek, window
    length, decoder prompt, the window's post-processed tokens; plus the final sequence."""
    from transformers import WhisperFeatureExtractor
    from transformers.models.whisper import generation_whisper as gw
    model = longform_hf_model()
    n_mel = synth.WHISPER_CONFIGS["micro"][0]
    clip = np.concatenate([synth.synth_clip(LONGFORM_CLIPS[0]), synth.synth_clip(LONGFORM_CLIPS[1]),
                           synth.synth_clip(LONGFORM_CLIPS[2])[:160000]])
    feat = WhisperFeatureExtractor(feature_size=n_mel)(clip, sampling_rate=16000, return_tensors="pt",
                                                        truncation=False, padding="longest", return_attention_mask=True)
    log = {"seek": [], "nframes": [], "prefix": [], "window": []}
    orig_seg = gw.WhisperGenerationMixin._get_input_segment
    orig_fb = gw.WhisperGenerationMixin.generate_with_fallback

    def seg_hook(input_features, seek, seek_num_frames, *a, **k):
        log["seek"].append(int(seek[0]))
        log["nframes"].append(int(seek_num_frames[0]))
        return orig_seg(input_features, seek, seek_num_frames, *a, **k)

    def fb_hook(self, *a, **k):
        out = orig_fb(self, *a, **k)
        log["prefix"].append(k["decoder_input_ids"][0].tolist())
        log["window"].append(out[0][0].tolist())
        return out

    gw.WhisperGenerationMixin._get_input_segment = staticmethod(seg_hook)
    gw.WhisperGenerationMixin.generate_with_fallback = fb_hook
    try:
        with torch.inference_mode():
            out = model.generate(input_features=feat.input_features, attention_mask=feat.attention_mask,
                                 return_timestamps=True, return_segments=True, language="en", task="transcribe",
                                 condition_on_prev_tokens=True, num_beams=1,
                                 prompt_ids=torch.tensor([50361] + LONGFORM_KEYWORDS),
                                 prompt_condition_type="all-segments")
    finally:
        gw.WhisperGenerationMixin._get_input_segment = staticmethod(orig_seg)
        gw.WhisperGenerationMixin.generate_with_fallback = orig_fb
    pad = lambda rows: np.array([r + [-1] * (max(map(len, rows)) - len(r)) for r in rows])   # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "longform_keywords_micro.npz"), seek=np.array(log["seek"]), nframes=np.array(log["nframes"]),
        prefix=pad(log["prefix"]), window=pad(log["window"]), sequence=out["sequences"][0].numpy(),
        keywords=np.array(LONGFORM_KEYWORDS))
    print("longform keywords: windows", len(log["window"]), "seek", log["seek"], "prefix lengths",
          [len(p) for p in log["prefix"]])


LONGFORM_BATCH_SECONDS = (70.0, 45.0, 95.0)   # three audios of different lengths (batch_size > 1, attention_mask)


def longform_batch_audio(i: int) -> np.ndarray:
    n = int(LONGFORM_BATCH_SECONDS[i] * 16000)
    return np.concatenate([synth.synth_clip(10 * i + q) for q in range(n // 480000 + 1)])[:n]


def make_longform_batched():
    """Batched long-form generation (pba_whisper.py:351-475 with batch_size > 1): transformers 5.15
    WhisperForConditionalGeneration.generate on the micro model over three audios of different lengths (padded
    features + attention_mask), greedy, return_timestamps=True, condition_on_prev_tokens=False -- every window's
    decoder input is the init tokens, so no prompt is padded and the 4.37.2 / 5.15 difference in attending to
    left pads does not arise (that is pinned by make_padded_beams).  Recorded per generate_with_fallback call: the
    active audios (batch_idx_map), their seeks and window lengths, each row's decoder input and post-processed
    tokens; plus every audio's final sequence and segments."""
    from transformers import WhisperFeatureExtractor
    from transformers.models.whisper import generation_whisper as gw
    model = longform_hf_model()
    n_mel = synth.WHISPER_CONFIGS["micro"][0]
    audios = [longform_batch_audio(i) for i in range(len(LONGFORM_BATCH_SECONDS))]
    feat = WhisperFeatureExtractor(feature_size=n_mel)(audios, sampling_rate=16000, return_tensors="pt",
                                                        truncation=False, padding="longest", return_attention_mask=True)
    calls = []
    orig_seg = gw.WhisperGenerationMixin._get_input_segment
    orig_fb = gw.WhisperGenerationMixin.generate_with_fallback

    def seg_hook(input_features, seek, seek_num_frames, num_segment_frames, cur_bsz, batch_idx_map):
        calls.append({"map": list(batch_idx_map), "seek": [int(seek[b]) for b in batch_idx_map],
                      "nframes": [int(seek_num_frames[b]) for b in batch_idx_map]})
        return orig_seg(input_features, seek, seek_num_frames, num_segment_frames, cur_bsz, batch_idx_map)

    def fb_hook(self, *a, **k):
        out = orig_fb(self, *a, **k)
        calls[-1]["prefix"] = [r.tolist() for r in k["decoder_input_ids"]]
        calls[-1]["window"] = [r.tolist() for r in out[0]]
        return out

    gw.WhisperGenerationMixin._get_input_segment = staticmethod(seg_hook)
    gw.WhisperGenerationMixin.generate_with_fallback = fb_hook
    try:
        with torch.inference_mode():
            out = model.generate(input_features=feat.input_features, attention_mask=feat.attention_mask,
                                 return_timestamps=True, return_segments=True, language="en", task="transcribe",
                                 condition_on_prev_tokens=False, num_beams=1)
    finally:
        gw.WhisperGenerationMixin._get_input_segment = staticmethod(orig_seg)
        gw.WhisperGenerationMixin.generate_with_fallback = orig_fb
    pad = lambda rows: np.array([r + [-1] * (max(map(len, rows)) - len(r)) for r in rows])   # noqa: E731
    rec = {"features": feat.input_features.numpy().astype(np.float32),
           "attention_mask": feat.attention_mask.numpy().astype(np.int32),
           "call_map": pad([c["map"] for c in calls]), "call_seek": pad([c["seek"] for c in calls]),
           "call_nframes": pad([c["nframes"] for c in calls]),
           "call_prefix": np.array([pad(c["prefix"]).tolist() + [[-1] * len(c["prefix"][0])] * (3 - len(c["prefix"]))
                                    for c in calls]),
           "call_window": pad([w for c in calls for w in c["window"]]),
           "call_rows": np.array([len(c["window"]) for c in calls])}
    for b in range(len(audios)):
        segs = out["segments"][b]
        rec[f"sequence_{b}"] = out["sequences"][b].numpy()
        rec[f"seg_start_{b}"] = np.array([float(s_["start"]) for s_ in segs])
        rec[f"seg_end_{b}"] = np.array([float(s_["end"]) for s_ in segs])
        rec[f"seg_tokens_{b}"] = pad([s_["tokens"].tolist() for s_ in segs])
    np.savez_compressed(os.path.join(HERE, "longform_batched_micro.npz"), **rec)
    print("longform batched: calls", len(calls), "active", [c["map"] for c in calls],
          "segments", [len(out["segments"][b]) for b in range(len(audios))])


PADDED_PROMPTS = ([1000, 1001, 1002], [2000 + 3 * i for i in range(11)], [])   # keyword prompts of one batch


def make_padded_beams():
    """One window of the batched long-form loop with keyword prompts of different lengths, as transformers 4.37.2
    decodes it (pba_whisper.py:478-548 left-pads the prompts with the pad token; 4.37.2's
    WhisperForConditionalGeneration.prepare_inputs_for_generation hands the decoder decoder_attention_mask=None, so
    the pads are attended as tokens at their positions): GenerationMixin beam search (num_beams 5, 24 new tokens,
    the suppression processors) over the three left-padded decoder inputs as ONE batch, without a decoder attention
    mask.  Each row's output is what the window's own beam search from its padded row gives (batch elements
    independent); transformers 5.15 semantics for decoder_prompt_len (= the padded length)."""
    from transformers import GenerationConfig, WhisperFeatureExtractor
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin
    model = longform_hf_model()
    n_mel = synth.WHISPER_CONFIGS["micro"][0]
    init = [50258, 50259, 50359, 50363]
    width = max(len(p) for p in PADDED_PROMPTS)
    rows = [[50361] + [50257] * (width - len(p)) + list(p) + init for p in PADDED_PROMPTS]
    mel = WhisperFeatureExtractor(feature_size=n_mel)([synth.synth_clip(20 + i) for i in range(3)], sampling_rate=16000,
                                                       return_tensors="pt").input_features
    gc = GenerationConfig(decoder_start_token_id=50361, eos_token_id=50257, pad_token_id=50257, num_beams=5,
                          do_sample=False, max_new_tokens=24, suppress_tokens=SUPPRESS, begin_suppress_tokens=[220, 50257],
                          length_penalty=1.0, early_stopping=False)
    with torch.inference_mode():
        enc = model.model.encoder(input_features=mel).last_hidden_state
        out = super(WhisperGenerationMixin, model).generate(input_features=mel, decoder_input_ids=torch.tensor(rows),
                                                            generation_config=gc).numpy()
        alone = [super(WhisperGenerationMixin, model).generate(input_features=mel[i:i + 1],
                                                               decoder_input_ids=torch.tensor([rows[i]]),
                                                               generation_config=gc)[0].numpy() for i in range(3)]
    for i in range(3):   # batch elements are independent: the batched row (right-padded) is the row decoded alone
        a = alone[i]
        assert (out[i, :len(a)] == a).all() and (out[i, len(a):] == 50257).all(), (out[i].tolist(), a.tolist())
    np.savez_compressed(os.path.join(HERE, "padded_beams_micro.npz"), rows=np.array(rows), out=out,
                        enc_out=enc.float().numpy(), suppress=np.array(SUPPRESS))
    print("padded beams", [r[len(rows[0]):].tolist() for r in out])


BEAM_SAMPLE_SEEDS = [11, 12, 13]


def make_beam_sample():
    """Beam-sample decoding (do_sample=True, num_beams=3, temperature 0.7, top_k 50) through GenerationMixin.generate
    as PBAWhisper's short-form call reaches it (pba_whisper.py:318-329), micro model on the CPU, the global CPU RNG
    seeded with torch.manual_seed(seed) before each call (the draws: torch.multinomial without replacement over
    softmax(processed + warped log-probs + beam scores) of all beams x vocab).  EOS is suppressed (added to
    suppress_tokens), so every step's 2 num_beams draws are non-EOS: transformers 5.15 keeps the sampled candidates in
    draw order where 4.37.2 sorts them by score, which matters only for ranking EOS candidates; without them both
    pick the running beams as the best-scored draws.  transformers 5.15 semantics for decoder_prompt_len."""
    from transformers import GenerationConfig
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin
    model = longform_hf_model()
    g = np.load(os.path.join(HERE, "decoder_micro.npz"))
    enc = torch.from_numpy(g["enc_out"])[None]
    from transformers.modeling_outputs import BaseModelOutput
    gc = GenerationConfig(decoder_start_token_id=BEAM_PREFIX[0], eos_token_id=50257, pad_token_id=50257, num_beams=3,
                          do_sample=True, temperature=0.7, top_k=50, max_new_tokens=16,
                          suppress_tokens=SUPPRESS + [50257], begin_suppress_tokens=[220, 50257], length_penalty=1.0,
                          early_stopping=False)
    outs = []
    for seed in BEAM_SAMPLE_SEEDS:
        torch.manual_seed(seed)
        with torch.inference_mode():
            o = super(WhisperGenerationMixin, model).generate(encoder_outputs=BaseModelOutput(last_hidden_state=enc),
                                                              decoder_input_ids=torch.tensor([BEAM_PREFIX]),
                                                              generation_config=gc)[0].numpy()
        outs.append(o)
        print("beam sample", seed, o[len(BEAM_PREFIX):].tolist())
    np.savez_compressed(os.path.join(HERE, "beam_sample_micro.npz"), prefix=np.array(BEAM_PREFIX),
                        seeds=np.array(BEAM_SAMPLE_SEEDS), out=np.stack(outs), suppress=np.array(SUPPRESS + [50257]),
                        num_beams=3, temperature=0.7, top_k=50, max_new_tokens=16)


LANG_CLIPS = (0, 3, 7)


def make_language():
    """Language detection for ``language=None`` (PBAWhisper.detect_language): transformers 5.15
    WhisperGenerationMixin.detect_language on the micro model (seeded weights, 99 language tokens) over the HF log-mel
    of synth clips LANG_CLIPS.  Stores the detected token ids and the decoder's logits at the 99 language tokens (the
    GPU test's tolerance for bf16 near-ties)."""
    from cbw.tokens import LANGUAGES
    from transformers import WhisperFeatureExtractor
    model = longform_hf_model()
    n_mel = synth.WHISPER_CONFIGS["micro"][0]
    model.generation_config.lang_to_id = {f"<|{c}|>": 50259 + i for i, c in enumerate(LANGUAGES[:99])}
    ids, logits = [], []
    for c in LANG_CLIPS:
        mel = WhisperFeatureExtractor(feature_size=n_mel)(synth.synth_clip(c), sampling_rate=16000,
                                                           return_tensors="pt").input_features
        with torch.inference_mode():
            lid = model.detect_language(input_features=mel, generation_config=model.generation_config)
            enc = model.model.encoder(input_features=mel).last_hidden_state
            lg = model(encoder_outputs=(enc,), decoder_input_ids=torch.tensor([[50258]])).logits[0, -1]
        ids.append(int(lid[0]))
        logits.append(lg[50259:50259 + 99].double().numpy())
    np.savez_compressed(os.path.join(HERE, "language_micro.npz"), clips=np.array(LANG_CLIPS), lang_ids=np.array(ids),
                        lang_logits=np.array(logits))
    print("language ids", ids, "margins", [float(np.sort(l)[-1] - np.sort(l)[-2]) for l in logits])


FREE_HEAD = BEAM_PREFIX[:5]   # <|startofprev|> 1000 1001 1002 <|startoftranscript|>: the language position is free


def make_free_language():
    """Short-form ``language=None`` as transformers 4.37.2 decodes it for pba_whisper.py:287-331: forced_decoder_ids
    (1, None) leaves the position after <|startoftranscript|> to the search and forces <|transcribe|> (and
    <|notimestamps|>) after it.  transformers 5.15 (installed) has no ForceTokensLogitsProcessor, so the 4.37.2
    processor is restated here as a LogitsProcessor (every score -inf, the forced token's 0, at the forced
    positions) with 4.37.2's begin suppression at the first position after the forced ids; GenerationMixin greedy /
    beam search (5 beams) from the forced head FREE_HEAD, 24 new tokens, the suppression list, micro model; with
    timestamps: WhisperTimeStampLogitsProcessor (begin_index = the first position after the forced ids) -- which
    4.37.2 also applies at the free position (<|notimestamps|> suppressed, the timestamp-mass rule).  transformers
    5.15 semantics for decoder_prompt_len (= len(FREE_HEAD))."""
    from transformers import GenerationConfig, LogitsProcessor, LogitsProcessorList
    from transformers.generation.logits_process import WhisperTimeStampLogitsProcessor
    from transformers.modeling_outputs import BaseModelOutput
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin

    class ForceAt(LogitsProcessor):
        def __init__(self, forced):
            self.forced = dict(forced)

        def __call__(self, input_ids, scores):
            t = self.forced.get(input_ids.shape[-1])
            if t is not None:
                scores = torch.full_like(scores, float("-inf"))
                scores[:, t] = 0
            return scores

    class SuppressAt(LogitsProcessor):
        def __init__(self, pos, tokens):
            self.pos, self.tokens = pos, list(tokens)

        def __call__(self, input_ids, scores):
            if input_ids.shape[-1] == self.pos:
                scores = scores.clone()
                scores[:, self.tokens] = float("-inf")
            return scores

    model = longform_hf_model()
    g = np.load(os.path.join(HERE, "decoder_micro.npz"))
    enc = torch.from_numpy(g["enc_out"])[None]
    L = len(FREE_HEAD)
    rec = {"head": np.array(FREE_HEAD), "suppress": np.array(SUPPRESS)}
    for ts in (False, True):
        forced = {L + 1: 50359} if ts else {L + 1: 50359, L + 2: 50363}
        begin = L + 1 + len(forced)
        for nb in (1, 5):
            gc = GenerationConfig(decoder_start_token_id=FREE_HEAD[0], eos_token_id=50257, pad_token_id=50257,
                                  num_beams=nb, do_sample=False, max_new_tokens=24, suppress_tokens=SUPPRESS,
                                  length_penalty=1.0, early_stopping=False, no_timestamps_token_id=50363,
                                  max_initial_timestamp_index=50)
            procs = [ForceAt(forced), SuppressAt(begin, [220, 50257])]
            if ts:
                procs.append(WhisperTimeStampLogitsProcessor(gc, begin_index=begin))
            with torch.inference_mode():
                o = super(WhisperGenerationMixin, model).generate(
                    encoder_outputs=BaseModelOutput(last_hidden_state=enc), decoder_input_ids=torch.tensor([FREE_HEAD]),
                    generation_config=gc, logits_processor=LogitsProcessorList(procs))[0].numpy()
            rec[f"out_b{nb}_ts{int(ts)}"] = o
            print("free language", nb, ts, o[L:].tolist())
    np.savez_compressed(os.path.join(HERE, "free_language_micro.npz"), **rec)


GEN_CONTROLS = {   # name -> (num_beams, GenerationConfig fields): caller-supplied generate controls
    "b5_length_penalty_nrs3": (5, dict(length_penalty=0.6, num_return_sequences=3)),
    "b5_repetition_penalty": (5, dict(repetition_penalty=1.5)),
    "b5_no_repeat_ngram": (5, dict(no_repeat_ngram_size=2)),
    "b1_repetition_penalty": (1, dict(repetition_penalty=1.5)),
    "b1_no_repeat_ngram": (1, dict(no_repeat_ngram_size=2)),
    "b4_max_length": (4, dict(max_length=len(BEAM_PREFIX) + 10)),
}


def make_gen_controls():
    """GenerationMixin greedy / beam search (transformers 5.15 on the micro model, the decoder_micro encoder output)
    from BEAM_PREFIX with the suppression processors and, per case, a caller's length_penalty / num_return_sequences
    / repetition_penalty / no_repeat_ngram_size / max_length (the generation controls the reference forwards to
    transformers through **kwargs, pba_whisper.py:320-331).  24 new tokens unless max_length is given.  transformers
    5.15 semantics for decoder_prompt_len (= len(BEAM_PREFIX))."""
    from transformers import GenerationConfig
    from transformers.modeling_outputs import BaseModelOutput
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin
    model = longform_hf_model()
    g = np.load(os.path.join(HERE, "decoder_micro.npz"))
    enc = torch.from_numpy(g["enc_out"])[None]
    rec = {"prefix": np.array(BEAM_PREFIX), "suppress": np.array(SUPPRESS)}
    from transformers import LogitsProcessor, LogitsProcessorList

    class EosAt(LogitsProcessor):   # +30 on EOS at one position: a hypothesis that ends before max_length
        def __call__(self, ids, scores):
            if ids.shape[-1] == len(BEAM_PREFIX) + 5:
                scores = scores.clone()
                scores[:, 50257] += 30.0
            return scores

    for nb in (1, 3):   # HF writes the EOS that ended the hypothesis back into the output
        gc = GenerationConfig(decoder_start_token_id=BEAM_PREFIX[0], eos_token_id=50257, pad_token_id=50257,
                              num_beams=nb, do_sample=False, max_new_tokens=12, suppress_tokens=SUPPRESS,
                              length_penalty=1.0, early_stopping=False)
        with torch.inference_mode():
            o = super(WhisperGenerationMixin, model).generate(
                encoder_outputs=BaseModelOutput(last_hidden_state=enc), decoder_input_ids=torch.tensor([BEAM_PREFIX]),
                generation_config=gc, logits_processor=LogitsProcessorList([EosAt()])).numpy()
        rec[f"b{nb}_eos_at_5"] = o
        print("gen controls eos", nb, o[0][len(BEAM_PREFIX):].tolist())
    for name, (nb, extra) in GEN_CONTROLS.items():
        kw = dict(decoder_start_token_id=BEAM_PREFIX[0], eos_token_id=50257, pad_token_id=50257, num_beams=nb,
                  do_sample=False, suppress_tokens=SUPPRESS, begin_suppress_tokens=[220, 50257], early_stopping=False)
        if "max_length" not in extra:
            kw["max_new_tokens"] = 24
        kw.update(extra)
        with torch.inference_mode():
            o = super(WhisperGenerationMixin, model).generate(
                encoder_outputs=BaseModelOutput(last_hidden_state=enc.expand(1, -1, -1)),
                decoder_input_ids=torch.tensor([BEAM_PREFIX]), generation_config=GenerationConfig(**kw)).numpy()
        rec[name] = o
        print("gen controls", name, [r[len(BEAM_PREFIX):].tolist() for r in o])
    np.savez_compressed(os.path.join(HERE, "gen_controls_micro.npz"), **rec)


def make_scorer():
    """Entity recall + tokenizer (src/scorer.py, src/priberam_tokenizer.py): the reference modules
    themselves, loaded from /root/reference/src.  string2string (absent) is replaced by the build's
    restatement cbw.alignment.NeedlemanWunsch, so these fixtures pin the scorer and tokenizer logic
    and the aligner stays "parity unpinned" against the library."""
    import importlib.util
    import json

    from cbw.alignment import NeedlemanWunsch
    from scorer_cases import NER_TAG_SETS, RECALL_CASES, TOKENIZER_TEXTS

    def load(name):
        spec = importlib.util.spec_from_file_location(name, os.path.join(REF_SRC, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    s2s = types.ModuleType("string2string")
    s2s_al = types.ModuleType("string2string.alignment")
    s2s_al.NeedlemanWunsch = NeedlemanWunsch
    s2s.alignment = s2s_al
    sys.modules["string2string"] = s2s
    sys.modules["string2string.alignment"] = s2s_al
    for n in ("priberam_tokenizer", "scorer"):
        sys.modules.pop(n, None)
    ptok = load("priberam_tokenizer")
    sc = load("scorer")
    tk = ptok.PriberamTokenizer()
    out = {"tokenize": [[[list(t) for t in sent] for sent in tk.tokenize(s)] for s in TOKENIZER_TEXTS],
           "just_split_sentences": [[[list(t) for t in sent] for sent in tk.just_split_sentences(s)]
                                    for s in TOKENIZER_TEXTS if s.strip()],
           "recall": []}
    preds = [c[0] for c in RECALL_CASES]
    refs = [c[1] for c in RECALL_CASES]
    ments = [c[2] for c in RECALL_CASES]
    for tags in NER_TAG_SETS:
        for cs in (False, True):
            r_all = sc.entity_recall(preds, refs, ments, tags, char_split=cs)
            per = [sc.entity_recall([p], [r], [m], tags, char_split=cs) for p, r, m in RECALL_CASES]
            out["recall"].append({"ner_tags": tags, "char_split": cs, "all": r_all, "per_case": per})
    with open(os.path.join(HERE, "scorer.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=0, sort_keys=True)
    print("scorer.json:", len(out["tokenize"]), "texts,", len(out["recall"]), "recall settings")


if __name__ == "__main__":
    what = sys.argv[1:] or ["kws", "mel", "encoder", "decoder", "kwdb", "cnn12", "scorer", "longform",
                            "longform_batched", "padded_beams", "beam_sample", "language", "free_language",
                            "gen_controls", "longform_keywords"]
    if "language" in what:
        make_language()
    if "free_language" in what:
        make_free_language()
    if "gen_controls" in what:
        make_gen_controls()
    if "longform_keywords" in what:
        make_longform_keywords()
    if "longform" in what:
        make_longform()
    if "longform_batched" in what:
        make_longform_batched()
    if "padded_beams" in what:
        make_padded_beams()
    if "beam_sample" in what:
        make_beam_sample()
    if "scorer" in what:
        make_scorer()
    if "cnn12" in what:
        make_cnn12()
    if "kwdb" in what:
        make_kwdb()
    if "decoder" in what:
        make_decoder()
    if "mel" in what:
        make_mel()
    if "encoder" in what:
        make_encoder()
    if "kws" in what:
        make_kws()
