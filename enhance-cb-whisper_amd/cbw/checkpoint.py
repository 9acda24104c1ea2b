"""Local HF-format checkpoint directories (what the reference's ``from_pretrained`` calls read), offline.

The reference loads every model by hub name (``PBAWhisper.from_pretrained(whisper_ckpt)``,
src/model/cb_whisper.py:57; ``WhisperModel.from_pretrained(encoder_ckpt).encoder``, :72;
``WhisperProcessor.from_pretrained``, :46-54).  There is no network here, so the drop-in takes a local
directory in the same layout -- ``config.json`` (WhisperConfig fields), optional ``generation_config.json``,
weights as ``model.safetensors`` / sharded ``model.safetensors.index.json`` / ``pytorch_model.bin``
(loaded with ``torch.load(weights_only=True)``: nothing in the file executes), tokenizer files -- and
hands the host tensors to the engines.  A hub name that is not a local directory raises.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Tuple

import torch


def _require_dir(path: str) -> str:
    if not os.path.isdir(path):
        raise FileNotFoundError(f"{path!r} is not a local checkpoint directory (hub downloads are not available "
                                f"offline: point the config at a directory holding config.json + model weights)")
    return path


def read_json(path: str, name: str) -> dict:
    p = os.path.join(path, name)
    if not os.path.exists(p):
        return {}
    with open(p, encoding="utf-8") as f:
        return json.load(f)


def load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    """All weights of a checkpoint directory as CPU tensors (safetensors first, then pytorch_model.bin)."""
    _require_dir(path)
    st = os.path.join(path, "model.safetensors")
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(st) or os.path.exists(idx):
        from safetensors.torch import load_file
        if os.path.exists(st):
            return dict(load_file(st))
        with open(idx) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        out: Dict[str, torch.Tensor] = {}
        for fn in files:
            out.update(load_file(os.path.join(path, fn)))
        return out
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.exists(pt):
        return dict(torch.load(pt, map_location="cpu", weights_only=True))
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin in {path}")


def whisper_configs(cfg: dict) -> Tuple[tuple, tuple, int]:
    """WhisperConfig fields -> (encoder (n_mel, d_model, layers, heads, ffn), decoder (vocab, d_model, layers,
    heads, ffn), max_target_positions)."""
    enc = (int(cfg["num_mel_bins"]), int(cfg["d_model"]), int(cfg["encoder_layers"]),
           int(cfg["encoder_attention_heads"]), int(cfg["encoder_ffn_dim"]))
    dec = (int(cfg["vocab_size"]), int(cfg["d_model"]), int(cfg.get("decoder_layers", 0)),
           int(cfg.get("decoder_attention_heads", 1)), int(cfg.get("decoder_ffn_dim", 0)))
    return enc, dec, int(cfg.get("max_target_positions", 448))


def encoder_state(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """The WhisperEncoder entries of a WhisperModel ('encoder.*') or WhisperForConditionalGeneration
    ('model.encoder.*') state dict, prefix stripped."""
    for pre in ("model.encoder.", "encoder."):
        sub = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        if sub:
            return sub
    raise KeyError("no encoder weights (model.encoder.* / encoder.*) in the checkpoint")


def save_whisper_dir(path: str, config: dict, state_dict: Dict[str, torch.Tensor],
                     generation_config: Optional[dict] = None) -> None:
    """Write config.json (+ generation_config.json) and model.safetensors (tests / tools)."""
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(config, f, indent=1)
    if generation_config is not None:
        with open(os.path.join(path, "generation_config.json"), "w") as f:
            json.dump(generation_config, f, indent=1)
    save_file({k: (v if torch.is_tensor(v) else torch.as_tensor(v)).contiguous() for k, v in state_dict.items()},
              os.path.join(path, "model.safetensors"))
