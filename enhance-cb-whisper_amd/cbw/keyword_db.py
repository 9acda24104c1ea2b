"""Keyword database: hidden-state extraction to ``.bin`` files, database loading with ghost
keywords, grouping, pad/truncate + masks, and the pre-projected (LE/LEF) cache that
``KwsEngine.score`` consumes.

Reference (paths relative to the reference ``src/``):

* ``utils.py:130-205`` ``extract_hidden_states`` — log-mel (padding to 30 s), encoder
  ``hidden_states[10:22]`` stacked on dim 0, truncated to ``t_len = ceil(frames / 2)`` where
  ``frames`` is the unpadded feature length, per-frame L2 normalisation, ``torch.save`` of an
  fp32 ``[L, t_len, D]`` tensor to ``<stem>.bin`` (an ``audio-`` prefix is stripped);
* ``efficient_kws/dataset.py:1677-1765`` — ``text/keywords.txt`` + ``keywords-hs/<kw_type>/<idx>.bin``
  (index zero-filled to the width of ``len(keywords) - 1``); a missing file is a *ghost* keyword
  whose hs are zeros shaped like the shortest stored keyword; groups of ``keywords_per_group``
  with a 0/1 ghost mask;
* ``efficient_kws/dataset.py:1767-1796`` — each keyword padded with zeros (mask 0) or truncated
  to ``features_size[0]`` frames, mask ``[L, Tk]``;
* ``model/cb_whisper.py:298-367`` ``DatabaseLite`` — ``num_groups`` / ``group`` / ``__getitem__``.

On the GPU path the keyword side is projected once per database (keyword-side
projections are amortised) and kept resident: bf16 ``[K, L, Tk', E]`` + f32 masks, about 29 KB
per keyword at LEF.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

HOP = 160                 # WhisperFeatureExtractor hop length (16 kHz)
N_SAMPLES = 480000        # 30 s


def hs_frames(n_samples: int) -> int:
    """t_len of utils.py:187: the unpadded log-mel has n_samples // 160 frames (HF drops the last
    STFT frame), the encoder halves it (conv2 stride 2), rounded up; capped at the 30 s window."""
    n = min(int(n_samples), N_SAMPLES)
    return int(math.ceil((n // HOP) / 2.0))


def extract_hidden_states(pcm, encoder, layer_ids: Sequence[int] = tuple(range(10, 22))) -> torch.Tensor:
    """utils.py:182-195 on the GPU: 16 kHz mono pcm -> f32 [len(layer_ids), t_len, D], per-frame
    L2-normalised (cbw_mel + cbw_encoder_hs)."""
    from .whisper import log_mel
    pcm = torch.as_tensor(np.asarray(pcm, dtype=np.float32)).to(encoder.device)
    _, pk = log_mel(pcm, encoder.n_mel, packed=True)
    hs = encoder.hidden_states(pk, list(layer_ids), normalize=True)[0]
    return hs[:, : hs_frames(pcm.numel())].contiguous()


def bin_name(audio_stem: str) -> str:
    """utils.py:197: ``<stem>.bin``, with a leading ``audio-`` removed."""
    return (audio_stem[6:] if "audio-" in audio_stem else audio_stem) + ".bin"


def write_bin(path: str, hs: torch.Tensor) -> None:
    """utils.py:199-201: torch.save of the fp32 tensor."""
    with open(path, "wb") as f:
        torch.save(hs.detach().to("cpu", torch.float32).clone(), f)


def read_bin(path: str) -> torch.Tensor:
    """Load a reference ``.bin`` (a pickled tensor) without executing code from the file."""
    with open(path, "rb") as f:
        return torch.load(f, map_location="cpu", weights_only=True).detach().to(torch.float32)


def pad_keyword(hs: torch.Tensor, frames: int):
    """efficient_kws/dataset.py:1767-1796: [L, T, D] -> ([L, frames, D], mask [L, frames])."""
    L, T, D = hs.shape
    if frames - T >= 0:
        mask = torch.cat((torch.ones(L, T), torch.zeros(L, frames - T)), dim=1)
        out = torch.cat((hs, torch.zeros(L, frames - T, D, dtype=hs.dtype)), dim=1)
    else:
        out = hs[:, :frames, :]
        mask = torch.ones(L, frames)
    return out, mask


class KeywordDatabase:
    """Keywords + per-keyword hs; ghosts (missing hs) get zeros shaped like the shortest stored
    keyword and a 0 in ``ghost_mask`` (efficient_kws/dataset.py:1711-1725)."""

    def __init__(self, keywords: Sequence[str], hidden_states: Sequence[Optional[torch.Tensor]],
                 keywords_per_group: int = 100):
        if len(keywords) != len(hidden_states):
            raise ValueError("one hs entry (or None for a ghost) per keyword")
        self.keywords = list(keywords)
        hs = [None if h is None else torch.as_tensor(h, dtype=torch.float32) for h in hidden_states]
        present = [(i, h.shape) for i, h in enumerate(hs) if h is not None]
        if not present and hs:
            raise ValueError("every keyword is a ghost")
        ghosts = [i for i, h in enumerate(hs) if h is None]
        if ghosts:
            smallest = min(present, key=lambda x: x[1][1])[0]
            for i in ghosts:
                hs[i] = torch.zeros_like(hs[smallest])
        self.hidden_states: List[torch.Tensor] = hs
        self.ghost_mask = torch.tensor([0.0 if i in set(ghosts) else 1.0 for i in range(len(hs))])
        self.keywords_per_group = len(self.keywords) if keywords_per_group == -1 else keywords_per_group
        self._projected: Dict[tuple, tuple] = {}

    # ---------------------------------------------------------------- loading
    @classmethod
    def from_split_folder(cls, split_folder: str, kw_type: str = "tts", keywords_per_group: int = 100,
                          keywords_file: str = os.path.join("text", "keywords.txt")):
        """efficient_kws/dataset.py:1677-1708 / data/dataset.py:386-407 layout: text/keywords.txt (Aishell:
        hotword.txt, data/dataset.py:243-251), keywords-hs/<kw_type>/<idx>.bin."""
        with open(os.path.join(split_folder, keywords_file)) as f:
            keywords = [line.strip() for line in f.readlines()]
        width = len(str(len(keywords) - 1))
        hs = []
        for i in range(len(keywords)):
            p = os.path.join(split_folder, "keywords-hs", kw_type, str(i).zfill(width) + ".bin")
            hs.append(read_bin(p) if os.path.exists(p) else None)
        return cls(keywords, hs, keywords_per_group)

    # ---------------------------------------------------------------- DatabaseLite surface
    def __len__(self) -> int:
        return len(self.keywords)

    def __getitem__(self, idx: int) -> dict:
        return {"keyword": self.keywords[idx], "hidden_states": self.hidden_states[idx]}

    def num_groups(self) -> int:
        return (len(self.keywords) + self.keywords_per_group - 1) // self.keywords_per_group

    def group(self, idx: int, device: str = "cpu", load_hs: bool = True) -> dict:
        lo = idx * self.keywords_per_group
        hi = min(lo + self.keywords_per_group, len(self.keywords))
        return {"keywords": self.keywords[lo:hi],
                "hidden_states": [h.to(device) for h in self.hidden_states[lo:hi]] if load_hs else None,
                "mask": self.ghost_mask[lo:hi].clone()}

    # ---------------------------------------------------------------- model inputs
    def padded(self, frames: int = 150, n_layers: Optional[int] = None):
        """All keywords padded/truncated to ``frames``: (f32 [K, L, frames, D], mask [K, L, frames],
        ghost mask [K]).  ``n_layers`` keeps the last n stored layers (efficient_kws/dataset.py:
        570-573 ``[-n_layers:]``)."""
        feats, masks = [], []
        for h in self.hidden_states:
            if n_layers is not None:
                h = h[-n_layers:]
            f, m = pad_keyword(h, frames)
            feats.append(f)
            masks.append(m)
        return torch.stack(feats), torch.stack(masks), self.ghost_mask.clone()

    def projected(self, engine, frames: int = 150, chunk: int = 256):
        """The keyword side through ``engine.project`` once, cached on the device:
        (bf16 [K, L, Tk', E], f32 [K, L, Tk'], ghost f32 [K])."""
        key = (id(engine), frames)
        if key not in self._projected:
            feats, masks, ghost = self.padded(frames, engine.n_layers)
            outs, oms = [], []
            for k0 in range(0, feats.shape[0], chunk):
                pk, pm = engine.project(feats[k0:k0 + chunk].to(engine.device), masks[k0:k0 + chunk].to(engine.device))
                outs.append(pk)
                oms.append(pm)
            self._projected[key] = (torch.cat(outs), torch.cat(oms), ghost.to(engine.device))
        return self._projected[key]

    def projected_f32(self, engine, frames: int = 150, chunk: int = 256) -> torch.Tensor:
        """The fp32 projections of the keyword side (KwsEngine.project_f32), cached on the device: the
        re-scoring tiers read them (f32 [K, L, Tk', E], 57.6 KB per keyword at LEF)."""
        key = ("f32", id(engine), frames)
        if key not in self._projected:
            feats, masks, _ = self.padded(frames, engine.n_layers)
            outs = [engine.project_f32(feats[k0:k0 + chunk].to(engine.device), masks[k0:k0 + chunk].to(engine.device))[0]
                    for k0 in range(0, feats.shape[0], chunk)]
            self._projected[key] = torch.cat(outs)
        return self._projected[key]

    def save_projected(self, path: str, engine, frames: int = 150) -> None:
        """Persist the projected cache (safetensors: no code in the file)."""
        from safetensors.torch import save_file
        pk, pm, g = self.projected(engine, frames)
        save_file({"features": pk.contiguous().cpu(), "mask": pm.contiguous().cpu(), "ghost": g.cpu()}, path)

    @staticmethod
    def load_projected(path: str, device) -> tuple:
        from safetensors.torch import load_file
        d = load_file(path, device=str(device))
        return d["features"], d["mask"], d["ghost"]


def build_split_folder(split_folder: str, keywords: Sequence[str], audios: Dict[int, np.ndarray], encoder,
                       kw_type: str = "tts", layer_ids: Sequence[int] = tuple(range(10, 22))) -> None:
    """Write the layout efficient_kws/dataset.py reads: text/keywords.txt and
    keywords-hs/<kw_type>/<idx>.bin for every keyword index that has audio (others stay ghosts)."""
    os.makedirs(os.path.join(split_folder, "text"), exist_ok=True)
    out = os.path.join(split_folder, "keywords-hs", kw_type)
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(split_folder, "text", "keywords.txt"), "w") as f:
        f.write("\n".join(keywords) + "\n")
    width = len(str(len(keywords) - 1))
    for i, pcm in audios.items():
        write_bin(os.path.join(out, str(i).zfill(width) + ".bin"), extract_hidden_states(pcm, encoder, layer_ids))
