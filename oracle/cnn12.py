"""ORACLE (test infrastructure only) — numpy restatement of CB-Whisper's own keyword spotter:
similarity matrices, bilinear resize, the 12-channel ResNet-50 classifier, argmax rule.

Only ``tests/`` may import this module, as the checker.  Pinned by ``tests/golden/cnn12.npz``
(the reference's ``model.model.KWSModel`` forward, made by ``make_golden.py cnn12``); the resize
is pinned against torch's ``F.interpolate(bilinear, align_corners=False, antialias=False)``,
the kernel torchvision's tensor ``resize`` dispatches to (torchvision is not installed here).
"""
from __future__ import annotations

import numpy as np

from oracle.kws import resnet_forward


def sim_matrices(kwd_hs, utt_hs: np.ndarray):
    """model/cb_whisper.py:196: matmul(kwd_hs_, utt_hs.transpose(2, 3)) — inputs already
    L2-normalised (utils.py:195, cb_whisper.py:106), no masks.  kwd_hs: list of [L, Tk, D];
    utt_hs [L, Tu, D] -> list of [L, Tk, Tu]."""
    u = utt_hs.astype(np.float64)
    return [np.matmul(k.astype(np.float64), np.swapaxes(u, -1, -2)) for k in kwd_hs]


def _axis(n_in: int, n_out: int):
    """PyTorch upsample_bilinear2d, align_corners=False, no scale factor: scale = in / out,
    src = max(scale * (dst + 0.5) - 0.5, 0); i1 = i0 + 1 unless i0 is the last index."""
    scale = np.float32(n_in) / np.float32(n_out)
    src = np.maximum(scale * (np.arange(n_out, dtype=np.float32) + np.float32(0.5)) - np.float32(0.5), 0)
    i0 = src.astype(np.int64)
    i1 = np.where(i0 < n_in - 1, i0 + 1, i0)
    l1 = (src - i0).astype(np.float32)
    return i0, i1, np.float32(1) - l1, l1


def resize_bilinear(x: np.ndarray, size) -> np.ndarray:
    """cb_whisper.py:206 torchvision resize(antialias=False) of [C, H, W] to (Ho, Wo), fp32 math."""
    x = x.astype(np.float32)
    y0, y1, ly0, ly1 = _axis(x.shape[-2], size[0])
    x0, x1, lx0, lx1 = _axis(x.shape[-1], size[1])
    top = x[:, y0][:, :, x0] * lx0 + x[:, y0][:, :, x1] * lx1
    bot = x[:, y1][:, :, x0] * lx0 + x[:, y1][:, :, x1] * lx1
    return top * ly0[:, None] + bot * ly1[:, None]


def cnn_forward(sd: dict, maps: np.ndarray) -> np.ndarray:
    """model/model.py:78-93: logits = classifier(flatten(ResNetModel(pixel_values).pooler_output))."""
    return resnet_forward(sd, maps, "resnet-50")


def keyword_spotting_logits(sd: dict, kwd_hs, utt_hs: np.ndarray, size=(150, 750)) -> np.ndarray:
    """cb_whisper.py:110-126 for one segment: sims -> resize -> CNN -> logits [K, 2]."""
    maps = np.stack([resize_bilinear(m, size) for m in sim_matrices(kwd_hs, utt_hs)])
    return cnn_forward(sd, maps)
