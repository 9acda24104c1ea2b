"""Seeded synthetic parameters and inputs for the CB-Whisper hot path.

No pretrained checkpoint exists offline (SURVEY.md §8c "Pretrained weights"), so
every test, the golden-fixture generator and ``bench.py`` draw parameters from
this module: a numpy PCG64 stream keyed by (seed, parameter name), so the same
state dict is regenerated bit-for-bit on the GPU box without the reference.

Parameter *names and shapes* follow the reference checkpoint layout exactly
(SURVEY.md §8b "On-disk formats"): the KWS names come from
``src/efficient_kws/model.py:71-124`` + ``src/efficient_kws/resnet.py:22-47``
(HF ``ResNetModel`` submodule names), the Whisper encoder names from the HF
``WhisperEncoder`` module used at ``src/model/cb_whisper.py:72``.
``tests/golden/make_golden.py`` loads these dicts into the reference modules
with ``strict=True``, which pins the naming.
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# ResNet topology (HF ResNetConfig defaults; efficient_kws/resnet.py:23-30)
# ---------------------------------------------------------------------------
RESNET_VERSIONS = {
    "resnet-50": ("bottleneck", [256, 512, 1024, 2048], [3, 4, 6, 3]),
    "resnet-34": ("basic", [64, 128, 256, 512], [3, 4, 6, 3]),
    "resnet-18": ("basic", [64, 128, 256, 512], [2, 2, 2, 2]),
}
EMBEDDING_SIZE = 64  # HF ResNetConfig.embedding_size


def _rng(seed: int, name: str) -> np.random.Generator:
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return np.random.Generator(np.random.PCG64(int.from_bytes(h[:8], "little")))


@dataclass
class ConvSpec:
    """One ResNetConvLayer / ResNetShortCut (conv without bias + BatchNorm2d)."""
    prefix: str          # e.g. model.feature_extractor.encoder.stages.0.layers.0.layer.0
    cin: int
    cout: int
    k: int
    stride: int
    relu: bool
    role: str = "main"   # stem | reduce | mid | expand | shortcut | basic1 | basic2


@dataclass
class BlockSpec:
    convs: List[ConvSpec]
    shortcut: ConvSpec | None


@dataclass
class ResNetSpec:
    version: str
    num_channels: int
    stem: ConvSpec
    blocks: List[BlockSpec] = field(default_factory=list)
    hidden: int = 2048


def resnet_spec(num_channels: int, version: str = "resnet-50",
                root: str = "model.feature_extractor") -> ResNetSpec:
    """Layer list of HF ResNetModel (modeling_resnet.py ResNetEmbeddings /
    ResNetStage / ResNetBottleNeckLayer, downsample_in_bottleneck=False ->
    stride sits in the 3x3), as instantiated by efficient_kws/resnet.py:22-38."""
    if version not in RESNET_VERSIONS:
        raise ValueError(f"unsupported resnet version {version}")
    layer_type, hidden, depths = RESNET_VERSIONS[version]
    stem = ConvSpec(f"{root}.embedder.embedder", num_channels, EMBEDDING_SIZE, 7, 2, True, "stem")
    spec = ResNetSpec(version, num_channels, stem, hidden=hidden[-1])
    cin = EMBEDDING_SIZE
    for s, (cout, depth) in enumerate(zip(hidden, depths)):
        for li in range(depth):
            stride = (1 if s == 0 else 2) if li == 0 else 1
            p = f"{root}.encoder.stages.{s}.layers.{li}"
            sc = None
            if cin != cout or stride != 1:
                sc = ConvSpec(f"{p}.shortcut", cin, cout, 1, stride, False, "shortcut")
            if layer_type == "bottleneck":
                mid = cout // 4
                convs = [
                    ConvSpec(f"{p}.layer.0", cin, mid, 1, 1, True, "reduce"),
                    ConvSpec(f"{p}.layer.1", mid, mid, 3, stride, True, "mid"),
                    ConvSpec(f"{p}.layer.2", mid, cout, 1, 1, False, "expand"),
                ]
            else:
                convs = [
                    ConvSpec(f"{p}.layer.0", cin, cout, 3, stride, True, "basic1"),
                    ConvSpec(f"{p}.layer.1", cout, cout, 3, 1, False, "basic2"),
                ]
            spec.blocks.append(BlockSpec(convs, sc))
            cin = cout
    return spec


def _conv_params(c: ConvSpec, conv_name: str) -> List[Tuple[str, Tuple[int, ...], str]]:
    base = c.prefix
    out = [(f"{base}.{conv_name}.weight", (c.cout, c.cin, c.k, c.k), f"conv:{c.role}")]
    for t in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
        out.append((f"{base}.normalization.{t}", (c.cout,) if t != "num_batches_tracked" else (), f"bn_{t}:{c.role}"))
    return out


def kws_param_shapes(n_layers: int, embedding_dim: int, learn_features: bool, proj_mlp: bool,
                     frames_conv: bool, proj_mlp_units: int = 64,
                     resnet_version: str = "resnet-50") -> List[Tuple[str, Tuple[int, ...], str]]:
    """(name, shape, kind) in reference state_dict order for
    efficient_kws.model.KWSModel (model.py:71-124)."""
    version = resnet_version if (learn_features and proj_mlp) else "resnet-50"
    spec = resnet_spec(n_layers, version)
    names: List[Tuple[str, Tuple[int, ...], str]] = []
    names += _conv_params(spec.stem, "convolution")
    for b in spec.blocks:
        if b.shortcut is not None:
            names += _conv_params(b.shortcut, "convolution")
        for c in b.convs:
            names += _conv_params(c, "convolution")
    names.append(("model.classifier.1.weight", (2, spec.hidden), "fc_w"))
    names.append(("model.classifier.1.bias", (2,), "fc_b"))
    if learn_features and proj_mlp:
        d = embedding_dim
        for i in range(n_layers):
            names.append((f"projector.{i}.0.weight", (d // 2, d), "lin_w"))
            names.append((f"projector.{i}.0.bias", (d // 2,), "lin_b"))
            names.append((f"projector.{i}.2.weight", (proj_mlp_units, d // 2), "lin_w"))
            names.append((f"projector.{i}.2.bias", (proj_mlp_units,), "lin_b"))
        if frames_conv:
            u = proj_mlp_units
            for i in range(n_layers):
                names.append((f"time_projector.{i}.0.weight", (u, u, 3), "lin_w"))
                names.append((f"time_projector.{i}.0.bias", (u,), "lin_b"))
                for t in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
                    names.append((f"time_projector.{i}.1.{t}", (u,) if t != "num_batches_tracked" else (),
                                  f"bn_{t}:tp"))
    return names


def _draw(kind: str, shape: Tuple[int, ...], g: np.random.Generator) -> np.ndarray:
    role = kind.split(":", 1)[1] if ":" in kind else ""
    if kind.startswith("conv"):
        # He fan-in scaling keeps activations O(1) through random layers (a
        # trained net's BN statistics do the same); the stem sees cosine
        # similarities of |x| <= 1, so it gets a larger gain.
        fan_in = int(np.prod(shape[1:]))
        std = math.sqrt(2.0 / fan_in) * (3.0 if role == "stem" else 1.0)
        return (g.standard_normal(shape) * std).astype(np.float32)
    if kind.startswith("bn_weight"):
        # keep the residual stream bounded through 16 blocks of random weights
        lo, hi = (0.3, 0.6) if role in ("expand", "basic2", "shortcut") else (0.8, 1.2)
        return g.uniform(lo, hi, shape).astype(np.float32)
    if kind.startswith("bn_bias"):
        return (g.standard_normal(shape) * 0.1).astype(np.float32)
    if kind.startswith("bn_running_mean"):
        return (g.standard_normal(shape) * 0.1).astype(np.float32)
    if kind.startswith("bn_running_var"):
        return g.uniform(0.8, 1.25, shape).astype(np.float32)
    if kind.startswith("bn_num_batches_tracked"):
        return np.array(1000, dtype=np.int64)
    if kind in ("lin_w", "fc_w"):
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / math.sqrt(fan_in)
        scale = 8.0 if kind == "fc_w" else 1.0
        return (g.uniform(-b, b, shape) * scale).astype(np.float32)
    if kind == "fc_b":  # shift class 1 so probabilities straddle 0.5 on random maps
        return (g.uniform(-0.1, 0.1, shape) + np.array([0.0, -1.5])).astype(np.float32)
    if kind == "lin_b":
        return (g.uniform(-0.1, 0.1, shape)).astype(np.float32)
    raise ValueError(kind)


def synth_kws_state_dict(seed: int = 0, **hp) -> Dict[str, np.ndarray]:
    """Seeded KWSModel state dict (numpy). ``hp`` = the KWSModel hparams in use."""
    shapes = kws_param_shapes(hp["n_layers"], hp["embedding_dim"], hp["learn_features"],
                              hp["proj_mlp"], hp.get("frames_conv", False),
                              hp.get("proj_mlp_units", 64), hp.get("resnet_version", "resnet-50"))
    return {n: _draw(k, s, _rng(seed, n)) for n, s, k in shapes}


# ---------------------------------------------------------------------------
# Whisper encoder (HF WhisperEncoder naming; cb_whisper.py:72, utils.py:150)
# ---------------------------------------------------------------------------
WHISPER_CONFIGS = {
    # name: (num_mel_bins, d_model, encoder_layers, encoder_attention_heads, encoder_ffn_dim)
    "micro": (80, 128, 3, 2, 256),
    "micro-deep": (80, 128, 21, 2, 256),   # 22 hidden states: hidden_states[10:22] selects 12 (CB-Whisper CNN)
    "tiny.en": (80, 384, 4, 6, 1536),
    "small": (80, 768, 12, 12, 3072),
    "medium": (80, 1024, 24, 16, 4096),
    "large-v3": (128, 1280, 32, 20, 5120),
}
MAX_SOURCE_POSITIONS = 1500


def whisper_sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Whisper's sinusoidal position table (sin | cos halves)."""
    log_inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-log_inc * np.arange(channels // 2, dtype=np.float64))
    t = np.arange(length, dtype=np.float64)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def whisper_encoder_param_shapes(name: str, n_layers: int | None = None) -> List[Tuple[str, Tuple[int, ...], str]]:
    """HF WhisperEncoder names; ``n_layers`` keeps only the first layers (a slice of a large encoder
    with the same per-name weights as the full one)."""
    n_mel, d, full_layers, _, ffn = WHISPER_CONFIGS[name]
    n_layers = full_layers if n_layers is None else min(n_layers, full_layers)
    out = [("conv1.weight", (d, n_mel, 3), "lin_w"), ("conv1.bias", (d,), "lin_b"),
           ("conv2.weight", (d, d, 3), "lin_w"), ("conv2.bias", (d,), "lin_b"),
           ("embed_positions.weight", (MAX_SOURCE_POSITIONS, d), "pos")]
    for i in range(n_layers):
        p = f"layers.{i}"
        out += [(f"{p}.self_attn.k_proj.weight", (d, d), "lin_w"),
                (f"{p}.self_attn.v_proj.weight", (d, d), "lin_w"), (f"{p}.self_attn.v_proj.bias", (d,), "lin_b"),
                (f"{p}.self_attn.q_proj.weight", (d, d), "lin_w"), (f"{p}.self_attn.q_proj.bias", (d,), "lin_b"),
                (f"{p}.self_attn.out_proj.weight", (d, d), "lin_w"), (f"{p}.self_attn.out_proj.bias", (d,), "lin_b"),
                (f"{p}.self_attn_layer_norm.weight", (d,), "ln_w"), (f"{p}.self_attn_layer_norm.bias", (d,), "ln_b"),
                (f"{p}.fc1.weight", (ffn, d), "lin_w"), (f"{p}.fc1.bias", (ffn,), "lin_b"),
                (f"{p}.fc2.weight", (d, ffn), "lin_w"), (f"{p}.fc2.bias", (d,), "lin_b"),
                (f"{p}.final_layer_norm.weight", (d,), "ln_w"), (f"{p}.final_layer_norm.bias", (d,), "ln_b")]
    out += [("layer_norm.weight", (d,), "ln_w"), ("layer_norm.bias", (d,), "ln_b")]
    return out


WHISPER_DECODERS = {
    # name: (vocab_size, d_model, decoder_layers, decoder_attention_heads, decoder_ffn_dim)
    "micro": (51865, 128, 2, 2, 256),
    "tiny.en": (51864, 384, 4, 6, 1536),
    "small": (51865, 768, 12, 12, 3072),
    "medium": (51865, 1024, 24, 16, 4096),
    "large-v3": (51866, 1280, 32, 20, 5120),
    "large-v3-2l": (51866, 1280, 2, 20, 5120),   # the first two layers of large-v3 (same seeded weights)
}
MAX_TARGET_POSITIONS = 448


def whisper_decoder_param_shapes(name: str) -> List[Tuple[str, Tuple[int, ...], str]]:
    """HF WhisperDecoder naming (the `model.decoder.` prefix stripped); proj_out is tied
    to embed_tokens in WhisperForConditionalGeneration."""
    V, d, n_layers, _, ffn = WHISPER_DECODERS[name]
    out = [("embed_tokens.weight", (V, d), "emb"), ("embed_positions.weight", (MAX_TARGET_POSITIONS, d), "pos_l")]
    for i in range(n_layers):
        p = f"layers.{i}"
        for att in ("self_attn", "encoder_attn"):
            out += [(f"{p}.{att}.k_proj.weight", (d, d), "lin_w"),
                    (f"{p}.{att}.v_proj.weight", (d, d), "lin_w"), (f"{p}.{att}.v_proj.bias", (d,), "lin_b"),
                    (f"{p}.{att}.q_proj.weight", (d, d), "lin_w"), (f"{p}.{att}.q_proj.bias", (d,), "lin_b"),
                    (f"{p}.{att}.out_proj.weight", (d, d), "lin_w"), (f"{p}.{att}.out_proj.bias", (d,), "lin_b"),
                    (f"{p}.{att}_layer_norm.weight", (d,), "ln_w"), (f"{p}.{att}_layer_norm.bias", (d,), "ln_b")]
        out += [(f"{p}.fc1.weight", (ffn, d), "lin_w"), (f"{p}.fc1.bias", (ffn,), "lin_b"),
                (f"{p}.fc2.weight", (d, ffn), "lin_w"), (f"{p}.fc2.bias", (d,), "lin_b"),
                (f"{p}.final_layer_norm.weight", (d,), "ln_w"), (f"{p}.final_layer_norm.bias", (d,), "ln_b")]
    out += [("layer_norm.weight", (d,), "ln_w"), ("layer_norm.bias", (d,), "ln_b")]
    return out


def synth_whisper_decoder_state_dict(name: str, seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded decoder weights; token embeddings get std 2/sqrt(d) so the tied output
    projection produces O(1)-spread logits (clear beam-search margins)."""
    sd = {}
    d = WHISPER_DECODERS[name][1]
    for n, shape, kind in whisper_decoder_param_shapes(name):
        g = _rng(seed, "whisper.decoder." + n)
        if kind == "emb":
            sd[n] = (g.standard_normal(shape) * (2.0 / math.sqrt(d))).astype(np.float32)
        elif kind == "pos_l":
            sd[n] = g.standard_normal(shape).astype(np.float32)   # position-dependent states: varied tokens
        elif kind == "ln_w":
            sd[n] = g.uniform(0.8, 1.2, shape).astype(np.float32)
        elif kind == "ln_b":
            sd[n] = (g.standard_normal(shape) * 0.02).astype(np.float32)
        elif kind == "lin_w":
            b = 1.0 / math.sqrt(int(np.prod(shape[1:])))
            sd[n] = g.uniform(-b, b, shape).astype(np.float32)
        else:
            sd[n] = g.uniform(-0.05, 0.05, shape).astype(np.float32)
    # make <|endoftext|> (50257) competitive with a frequently predicted token so that
    # beam hypotheses finish at different lengths (exercises the EOS path of the scorer)
    e = sd["embed_tokens.weight"]
    if e.shape[0] > 50257:
        e[50257] = 1.05 * e[44051]
    return sd


def synth_whisper_encoder_state_dict(name: str, seed: int = 0, n_layers: int | None = None) -> Dict[str, np.ndarray]:
    sd = {}
    d = WHISPER_CONFIGS[name][1]
    for n, shape, kind in whisper_encoder_param_shapes(name, n_layers):
        g = _rng(seed, "whisper." + n)
        if kind == "pos":
            sd[n] = whisper_sinusoids(MAX_SOURCE_POSITIONS, d)
        elif kind == "ln_w":
            sd[n] = g.uniform(0.8, 1.2, shape).astype(np.float32)
        elif kind == "ln_b":
            sd[n] = (g.standard_normal(shape) * 0.02).astype(np.float32)
        elif kind == "lin_w":
            fan_in = int(np.prod(shape[1:]))
            b = 1.0 / math.sqrt(fan_in)
            sd[n] = g.uniform(-b, b, shape).astype(np.float32)
        else:
            sd[n] = g.uniform(-0.05, 0.05, shape).astype(np.float32)
    return sd


# ---------------------------------------------------------------------------
# Synthetic inputs (SURVEY.md §8d "Synthetic inputs")
# ---------------------------------------------------------------------------
def synth_clip(idx: int, seconds: float = 30.0, sr: int = 16000) -> np.ndarray:
    """x = 0.1*N(0,1) + a few sinusoids, seeded PCG64(seed = clip index)."""
    g = np.random.Generator(np.random.PCG64(idx))
    n = int(seconds * sr)
    t = np.arange(n, dtype=np.float64) / sr
    x = 0.1 * g.standard_normal(n)
    for _ in range(3):
        f = g.uniform(80.0, 4000.0)
        x += g.uniform(0.05, 0.3) * np.sin(2 * np.pi * f * t + g.uniform(0, 2 * np.pi))
    return x.astype(np.float32)


def l2n(x: np.ndarray) -> np.ndarray:
    n = np.linalg.norm(x, axis=-1, keepdims=True)
    return (x / np.where(n == 0, 1, n)).astype(np.float32)


def synth_kws_batch(seed: int, K: int, n_layers: int, D: int, Tk: int = 150, Tu: int = 1500,
                    utt_len: int | None = None, ghost: Sequence[int] = (), plant: Sequence[int] = (),
                    min_len: int = 8):
    """Seeded keyword/utterance hs in the dataset contract
    (efficient_kws/dataset.py:1767-1796 keyword pad/mask, :2015-2044 utterance
    pad/mask): per-frame L2-normalised rows, zero padding, 0/1 masks.

    ``ghost`` keywords get zero features with the shortest keyword's mask
    (dataset.py:1711-1721); ``plant`` keywords are copied (with noise) into the
    utterance so the similarity maps carry a diagonal."""
    g = np.random.Generator(np.random.PCG64(seed))
    utt_len = Tu if utt_len is None else utt_len
    lens = g.integers(min_len, Tk + 1, size=K)
    if K > 0:
        lens[0] = Tk
    kwd = np.zeros((K, n_layers, Tk, D), np.float32)
    kwd_mask = np.zeros((K, n_layers, Tk), np.float32)
    for i in range(K):
        kwd[i, :, :lens[i]] = l2n(g.standard_normal((n_layers, lens[i], D)).astype(np.float32))
        kwd_mask[i, :, :lens[i]] = 1.0
    utt = np.zeros((1, n_layers, Tu, D), np.float32)
    utt[0, :, :utt_len] = l2n(g.standard_normal((n_layers, utt_len, D)).astype(np.float32))
    for i in plant:
        off = int(g.integers(0, max(1, utt_len - lens[i])))
        seg = kwd[i, :, :lens[i]] + 0.3 * g.standard_normal((n_layers, lens[i], D)).astype(np.float32)
        n = min(lens[i], utt_len - off)
        utt[0, :, off:off + n] = l2n(seg[:, :n])
    utt_mask = np.zeros((1, n_layers, Tu), np.float32)
    utt_mask[0, :, :utt_len] = 1.0
    ghost_mask = np.ones((K,), np.float32)
    if len(ghost):
        shortest = int(np.argmin(lens))
        for i in ghost:
            kwd[i] = 0.0
            kwd_mask[i] = 0.0
            kwd_mask[i, :, :lens[shortest]] = 1.0
            ghost_mask[i] = 0.0
    return dict(kwd=kwd, kwd_mask=kwd_mask, utt=utt, utt_mask=utt_mask, ghost_mask=ghost_mask)


# ---------------------------------------------------------------------------
# Local checkpoint directories (HF layout) for the drop-in constructors: no hub access exists
# offline, so tests and tools write small seeded stand-ins in the files the reference's
# from_pretrained calls read (config.json, generation_config.json, model.safetensors, tokenizer
# files).
# ---------------------------------------------------------------------------
TOKENIZER_WORDS = ["the", "topic", "of", "today", "speech", "is", "ah", "okay", "then", "continue", "alpha", "bravo",
                   "charlie", "delta", "echo", "foxtrot", "keyword", "spotting", "whisper", "neural", "machine",
                   "translation", "attention", "transformer", "model", "data", "and", "to", "in", "we", "I'll"]


def whisper_special_tokens(vocab_size: int) -> List[str]:
    """Added tokens of the multilingual Whisper tokenizers from <|endoftext|> (50257) on, in id order."""
    from .tokens import LANGUAGES
    n_lang = 100 if vocab_size >= 51866 else 99
    toks = ["<|endoftext|>", "<|startoftranscript|>"] + [f"<|{l}|>" for l in LANGUAGES[:n_lang]]
    toks += ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nospeech|>", "<|notimestamps|>"]
    toks += [f"<|{i * 0.02:.2f}|>" for i in range(1501)]
    return toks


def write_synth_tokenizer(path: str, vocab_size: int = 51865) -> None:
    """A byte-level BPE tokenizer in the Whisper file layout (vocab.json, merges.txt, added_tokens.json,
    special_tokens_map.json, tokenizer_config.json): the 256 byte symbols, merges spelling TOKENIZER_WORDS
    (with and without the leading-space marker), filler entries up to id 50256, <|endoftext|> = 50257 in
    vocab.json as well, then the Whisper added tokens at their real ids (<|endoftext|> = 50257 ...)."""
    import json
    import os
    from .tokenizer import bytes_to_unicode
    os.makedirs(path, exist_ok=True)
    b2u = bytes_to_unicode()
    vocab = {b2u[b]: i for i, b in enumerate(sorted(b2u))}
    merges = []
    sp = b2u[ord(" ")]
    for w in TOKENIZER_WORDS:
        for word in (w, sp + "".join(b2u[b] for b in w.encode())):
            syms = list(word) if word[0] == sp else ["".join(b2u[b] for b in c.encode()) for c in word]
            cur = syms[0]
            for s in syms[1:]:
                if (cur, s) not in merges:
                    merges.append((cur, s))
                cur = cur + s
                vocab.setdefault(cur, len(vocab))
    n = len(vocab)
    for i in range(n, 50257):
        vocab[f"☃fill{i}"] = i
    specials = whisper_special_tokens(vocab_size)
    added = {t: 50257 + i for i, t in enumerate(specials)}
    vocab["<|endoftext|>"] = 50257   # real Whisper vocab.json files list it too (as well as added_tokens.json)
    with open(os.path.join(path, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    with open(os.path.join(path, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    with open(os.path.join(path, "added_tokens.json"), "w", encoding="utf-8") as f:
        json.dump(added, f, ensure_ascii=False)
    with open(os.path.join(path, "special_tokens_map.json"), "w", encoding="utf-8") as f:
        json.dump({"bos_token": "<|endoftext|>", "eos_token": "<|endoftext|>", "unk_token": "<|endoftext|>",
                   "pad_token": "<|endoftext|>", "additional_special_tokens": specials[1:-1501]}, f)
    dec = {str(i): {"content": t, "lstrip": False, "normalized": False, "rstrip": False, "single_word": False,
                    "special": not t[2].isdigit()} for t, i in added.items()}
    with open(os.path.join(path, "tokenizer_config.json"), "w", encoding="utf-8") as f:
        json.dump({"tokenizer_class": "WhisperTokenizer", "model_max_length": 1024, "errors": "replace",
                   "add_prefix_space": False, "added_tokens_decoder": dec}, f)


def whisper_hf_config(enc_name: str, dec_name: str | None = None) -> dict:
    """config.json fields of WhisperConfig for a seeded encoder (+ decoder) size."""
    n_mel, d, el, eh, ef = WHISPER_CONFIGS[enc_name]
    cfg = {"model_type": "whisper", "architectures": ["WhisperForConditionalGeneration"], "num_mel_bins": n_mel,
           "d_model": d, "encoder_layers": el, "encoder_attention_heads": eh, "encoder_ffn_dim": ef,
           "max_source_positions": MAX_SOURCE_POSITIONS, "max_target_positions": MAX_TARGET_POSITIONS,
           "vocab_size": 51865, "decoder_layers": 0, "decoder_attention_heads": eh, "decoder_ffn_dim": ef}
    if dec_name is not None:
        V, dd, dl, dh, df = WHISPER_DECODERS[dec_name]
        cfg.update(vocab_size=V, decoder_layers=dl, decoder_attention_heads=dh, decoder_ffn_dim=df)
    return cfg


def write_cbwhisper_fixture(root: str, keywords: Sequence[str] = ("alpha", "bravo", "charlie", "delta", "echo",
                                                                   "foxtrot", "golf"),
                            ghosts: Sequence[int] = (5,), seed: int = 0, keyword_hs: Dict[int, np.ndarray] | None = None,
                            cnn_class1_shift: float = 0.0) -> Dict[str, str]:
    """Everything cb-whisper-acl.yaml's CBWhisper init_args point at, seeded and small:
    whisper_ckpt (micro WhisperForConditionalGeneration + tokenizer files), encoder_ckpt (micro-deep
    WhisperModel: 22 hidden states), kws_ckpt (the 12-channel CNN, model.model.KWSModel, as a Lightning
    .ckpt) and an ACL-layout root (root/2/acl_6060/eval: text/keywords.txt, keywords-hs/tts/<idx>.bin with
    12 L2-normalised [12, Tk, 128] hidden states per keyword -- ``keyword_hs[i]`` replaces keyword i's, e.g.
    slices of an utterance's own hidden states; ``ghosts`` have no file).  ``cnn_class1_shift`` is added to
    the CNN's class-1 bias (moves the argmax decision boundary)."""
    import os
    import torch
    from .checkpoint import save_whisper_dir
    paths = {k: os.path.join(root, k) for k in ("whisper", "encoder", "acl")}
    paths["kws_ckpt"] = os.path.join(root, "cnn12.ckpt")
    sd = {"model.encoder." + k: torch.from_numpy(np.asarray(v)) for k, v in
          synth_whisper_encoder_state_dict("micro", seed).items()}
    sd.update({"model.decoder." + k: torch.from_numpy(np.asarray(v)) for k, v in
               synth_whisper_decoder_state_dict("micro", seed).items()})
    gen = {"suppress_tokens": [1, 2, 7], "begin_suppress_tokens": [220, 50257], "max_length": 448,
           "max_initial_timestamp_index": 50, "decoder_start_token_id": 50258}
    save_whisper_dir(paths["whisper"], whisper_hf_config("micro", "micro"), sd, gen)
    write_synth_tokenizer(paths["whisper"])
    esd = {"encoder." + k: torch.from_numpy(np.asarray(v)) for k, v in
           synth_whisper_encoder_state_dict("micro-deep", seed).items()}
    save_whisper_dir(paths["encoder"], whisper_hf_config("micro-deep"), esd)
    ksd = {k: torch.from_numpy(np.asarray(v)) for k, v in
           synth_kws_state_dict(seed=seed + 3, n_layers=12, embedding_dim=128, learn_features=False,
                                proj_mlp=False).items()}
    ksd["model.classifier.1.bias"][1] += cnn_class1_shift
    torch.save({"state_dict": ksd, "hyper_parameters": {"num_domains": 72}}, paths["kws_ckpt"])
    split = os.path.join(paths["acl"], "2", "acl_6060", "eval")
    os.makedirs(os.path.join(split, "text"), exist_ok=True)
    os.makedirs(os.path.join(split, "keywords-hs", "tts"), exist_ok=True)
    with open(os.path.join(split, "text", "keywords.txt"), "w") as f:
        f.write("\n".join(keywords) + "\n")
    g = np.random.default_rng(seed + 11)
    width = len(str(len(keywords) - 1))
    for i in range(len(keywords)):
        if i in ghosts:
            continue
        T = int(g.integers(6, 60))
        x = g.standard_normal((12, T, 128)).astype(np.float32)
        x /= np.linalg.norm(x, axis=-1, keepdims=True)
        if keyword_hs is not None and i in keyword_hs:
            x = np.ascontiguousarray(keyword_hs[i], dtype=np.float32)
        with open(os.path.join(split, "keywords-hs", "tts", str(i).zfill(width) + ".bin"), "wb") as f:
            torch.save(torch.from_numpy(x), f)
    return paths
