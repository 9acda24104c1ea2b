"""Whisper front end + encoder engines over libcbw.

* ``log_mel`` replaces HF ``WhisperFeatureExtractor(padding='max_length')``
  (src/utils.py:186-187; src/data/dataset.py:332-339).
* ``EncoderEngine.hidden_states`` replaces ``WhisperModel.encoder(...,
  output_hidden_states=True)['hidden_states'][ids]`` + the per-frame L2
  normalisation (src/model/cb_whisper.py:100-106, src/utils.py:188-195).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

N_SAMPLES, N_FRAMES, N_CTX = 480000, 3000, 1500


def cpad_for(n_mel: int) -> int:
    return (n_mel + 63) // 64 * 64


def log_mel(pcm: torch.Tensor, n_mel: int, packed: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """pcm f32 [n] (device) -> (mel f32 [n_mel, 3000], time-major bf16 [3000, cpad] or None)."""
    _lib.require_gpu()
    lib = _lib.load()
    pcm = pcm.to(torch.float32).contiguous()
    dev = pcm.device
    out = torch.empty((n_mel, N_FRAMES), dtype=torch.float32, device=dev)
    cp = cpad_for(n_mel)
    pk = torch.empty((N_FRAMES, cp), dtype=torch.bfloat16, device=dev) if packed else None
    ws = torch.empty(64, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.cbw_mel(pcm.data_ptr(), pcm.numel(), n_mel, out.data_ptr(), _lib.ptr(pk), cp, ws.data_ptr(),
                               _lib.stream_handle()), "cbw_mel")
    return out, pk


def log_mel_long(pcm: torch.Tensor, n_mel: int) -> torch.Tensor:
    """Long-form features of a whole audio (cbw_mel_long; WhisperFeatureExtractor(padding='longest',
    truncation=False)): pcm f32 [n] (device) -> f32 [n_mel, n // 160]."""
    _lib.require_gpu()
    lib = _lib.load()
    pcm = pcm.to(torch.float32).contiguous()
    out = torch.empty((n_mel, pcm.numel() // 160), dtype=torch.float32, device=pcm.device)
    ws = torch.empty(1024, dtype=torch.uint8, device=pcm.device)
    with torch.cuda.device(pcm.device):
        _lib.check(lib.cbw_mel_long(pcm.data_ptr(), pcm.numel(), n_mel, out.data_ptr(), ws.data_ptr(),
                                    _lib.stream_handle()), "cbw_mel_long")
    return out


def default_layer_ids(n_layers: int, n_select: int = 3):
    """hidden_states[10:22][-n:] (cb_whisper.py:100-104, efficient_kws/dataset.py:570-573);
    encoders with < 11 hidden states (tiny: 5) use hidden_states[-n:]."""
    ids = list(range(n_layers + 1))[10:22][-n_select:]
    return ids if len(ids) == n_select else list(range(n_layers + 1))[-n_select:]


class EncoderEngine:
    def __init__(self, config: Tuple[int, int, int, int, int], state_dict: Dict[str, object],
                 device: Optional[torch.device] = None):
        """config = (n_mel, d_model, n_layers, n_heads, ffn_dim); state_dict in HF WhisperEncoder naming."""
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.n_mel, self.d_model, self.n_layers, self.n_heads, self.ffn = config
        self.cpad = cpad_for(self.n_mel)
        cfg = _lib.EncoderConfig(*config)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_encoder_create(ctypes.byref(cfg), ctypes.byref(h)), "cbw_encoder_create")
            self.h = h
            for name, v in state_dict.items():
                name = name[len("encoder."):] if name.startswith("encoder.") else name
                a = np.ascontiguousarray(v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v),
                                         dtype=np.float32)
                _lib.check(self.lib.cbw_encoder_set_param(self.h, name.encode(), a.ctypes.data, a.size),
                           f"cbw_encoder_set_param({name})")
            _lib.check(self.lib.cbw_encoder_finalize(self.h), "cbw_encoder_finalize")
        self._ws = _lib.Workspace()

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.cbw_encoder_destroy(h)
            except Exception:
                pass

    def hidden_states(self, mel_packed: torch.Tensor, layer_ids: Sequence[int], normalize: bool = True,
                      early_exit: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """mel_packed bf16 [B, 3000, cpad] (or [3000, cpad]) -> f32 [B, n_ids, 1500, D]."""
        if mel_packed.dim() == 2:
            mel_packed = mel_packed.unsqueeze(0)
        B = mel_packed.shape[0]
        if tuple(mel_packed.shape[1:]) != (N_FRAMES, self.cpad) or mel_packed.dtype != torch.bfloat16:
            raise ValueError(f"expected bf16 [B, {N_FRAMES}, {self.cpad}] mel, got {tuple(mel_packed.shape)} "
                             f"{mel_packed.dtype}")
        mel_packed = mel_packed.contiguous()
        ids = torch.tensor(list(layer_ids), dtype=torch.int32)
        hs = out if out is not None else torch.empty((B, len(ids), N_CTX, self.d_model), dtype=torch.float32,
                                                     device=self.device)
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_encoder_workspace_bytes(self.h, B)
            ws = self._ws.get(nb, self.device)
            flags = (1 if normalize else 0) | (2 if early_exit else 0)
            _lib.check(self.lib.cbw_encoder_hs(self.h, mel_packed.data_ptr(), B, ids.numpy().ctypes.data, len(ids),
                                               flags, hs.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle()),
                       "cbw_encoder_hs")
        return hs
