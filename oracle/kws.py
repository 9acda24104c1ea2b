"""ORACLE (test infrastructure only) — CPU restatement of the efficient_kws
classifier path in numpy.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``enhance-cb-whisper_amd``) never calls it and fails loudly when its HIP
library is missing.

Parity pinning: ``tests/test_oracle_golden.py`` checks every function here
against fixtures produced by the *reference's own code* (imported with
host-only stubs by ``tests/golden/make_golden.py``).

Each function cites the reference file:line it restates (paths relative to
the reference ``src/``).  Third-party code on the path (HF transformers
``ResNetModel`` — pinned transformers==4.37.2 in ``requirements.txt:21``,
installed copy 5.15.0) is restated from its published module structure.
"""
from __future__ import annotations

import numpy as np

from oracle.common import (conv2d_nchw, batchnorm_eval, maxpool2d_nchw, relu,
                           conv1d_ncl, maxpool1d_ncl, softmax)

__all__ = ["sim_matrix", "project", "pool_mask", "kws_forward", "resnet_forward",
           "decide", "spot_argmax"]


def sim_matrix(a: np.ndarray, b: np.ndarray, eps: float = 1e-6) -> np.ndarray:
    """efficient_kws/model.py:210-218 — cosine similarity with norms clamped at eps.
    a: [B, Ta, E], b: [B, Tb, E] -> [B, Ta, Tb]."""
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    an = np.maximum(np.linalg.norm(a, axis=-1, keepdims=True), eps)
    bn = np.maximum(np.linalg.norm(b, axis=-1, keepdims=True), eps)
    return np.matmul(a / an, np.swapaxes(b / bn, -1, -2))


def project(x: np.ndarray, sd: dict, n_layers: int, frames_conv: bool) -> np.ndarray:
    """efficient_kws/model.py:143-166 — per-layer projector MLP
    (Linear·ReLU·Linear, :87-104) and optional time projector
    (Conv1d k3 p1 -> BatchNorm1d (eval) -> MaxPool1d(3,2,1), :106-124).
    x: [B, L, T, D] -> [B, L, T', U]."""
    outs = []
    for i in range(n_layers):
        h = x[:, i].astype(np.float64)
        h = h @ sd[f"projector.{i}.0.weight"].T.astype(np.float64) + sd[f"projector.{i}.0.bias"]
        h = relu(h)
        h = h @ sd[f"projector.{i}.2.weight"].T.astype(np.float64) + sd[f"projector.{i}.2.bias"]
        if frames_conv:
            p = f"time_projector.{i}"
            t = np.swapaxes(h, 1, 2)                                   # [B, U, T]
            t = conv1d_ncl(t, sd[f"{p}.0.weight"], sd[f"{p}.0.bias"], stride=1, pad=1)
            t = batchnorm_eval(t, sd[f"{p}.1.weight"], sd[f"{p}.1.bias"],
                               sd[f"{p}.1.running_mean"], sd[f"{p}.1.running_var"], axis=1)
            t = maxpool1d_ncl(t, 3, 2, 1)
            h = np.swapaxes(t, 1, 2)
        outs.append(h)
    return np.stack(outs, axis=1)


def pool_mask(mask: np.ndarray) -> np.ndarray:
    """LEF mask semantics (build decision): the
    reference LEF path crashes at model.py:186-191 because MaxPool1d halves the
    frame axis but not the masks; the masks go through the same MaxPool1d(3,2,1).
    mask: [B, L, T] -> [B, L, T']."""
    return maxpool1d_ncl(mask.astype(np.float64), 3, 2, 1)


def resnet_forward(sd: dict, x: np.ndarray, version: str = "resnet-50",
                   root: str = "model.feature_extractor") -> np.ndarray:
    """efficient_kws/resnet.py:51-58 over HF ResNetModel (embedder conv7x7 s2 p3
    ·BN·ReLU·MaxPool(3,2,1); stages of bottleneck layers with the stride in the
    3x3; shortcut = conv1x1(stride)·BN when shape changes; residual add then
    ReLU; AdaptiveAvgPool(1,1)) + classifier Linear(hidden[-1] -> 2).
    x: [K, C, H, W] -> logits [K, 2] (float64)."""
    from cbw.synth import resnet_spec  # topology table only (names/shapes)

    spec = resnet_spec(x.shape[1], version, root)

    def conv_bn(h, c):
        w = sd[f"{c.prefix}.convolution.weight"]
        h = conv2d_nchw(h, w, c.stride, c.k // 2)
        h = batchnorm_eval(h, sd[f"{c.prefix}.normalization.weight"], sd[f"{c.prefix}.normalization.bias"],
                           sd[f"{c.prefix}.normalization.running_mean"],
                           sd[f"{c.prefix}.normalization.running_var"], axis=1)
        return relu(h) if c.relu else h

    if x.shape[1] != spec.num_channels:
        raise ValueError("Make sure that the channel dimension of the pixel values match with the one set in the configuration.")
    h = conv_bn(x.astype(np.float32), spec.stem)
    h = maxpool2d_nchw(h, 3, 2, 1)
    for b in spec.blocks:
        r = h
        for c in b.convs:
            h = conv_bn(h, c)
        if b.shortcut is not None:
            r = conv_bn(r, b.shortcut)
        h = relu(h + r)
    feat = h.astype(np.float64).mean(axis=(2, 3))
    return feat @ sd["model.classifier.1.weight"].T.astype(np.float64) + sd["model.classifier.1.bias"]


def kws_forward(sd: dict, hp: dict, kwd: np.ndarray, utt: np.ndarray,
                kwd_mask: np.ndarray, utt_mask: np.ndarray, return_features: bool = True):
    """efficient_kws/model.py:129-208 (KWSModel.forward), eval mode.
    kwd: [K, L, Tk, D]; utt: [1 or K, L, Tu, D]; masks [K|1, L, T].
    Returns (logits [K,2] f64, features [K, L, Tk', Tu'] f32 or None)."""
    L = hp["n_layers"]
    learned = hp.get("learn_features", False) and hp.get("proj_mlp", False)
    frames_conv = learned and hp.get("frames_conv", False)
    if learned:
        pk = project(kwd, sd, L, frames_conv)
        pu = project(utt, sd, L, frames_conv)
        if frames_conv:
            kwd_mask = pool_mask(kwd_mask)
            utt_mask = pool_mask(utt_mask)
    else:
        pk, pu = kwd, utt
    K = pk.shape[0]
    feats = np.stack([
        np.swapaxes(sim_matrix(np.broadcast_to(pu[:, l], (K,) + pu.shape[2:]), pk[:, l]), 1, 2)
        for l in range(pk.shape[1])], axis=1)                        # [K, L, Tk, Tu]
    feats = feats * utt_mask[:, :, None, :] * kwd_mask[..., None]
    feats = feats.astype(np.float32)
    logits = resnet_forward(sd, feats, hp.get("resnet_version", "resnet-50") if learned else "resnet-50")
    return logits, (feats if return_features else None)


def decide(logits: np.ndarray, ghost_mask: np.ndarray | None, threshold: float):
    """efficient_kws/model.py:782-799 (prob = softmax(logits)[:,1] * ghost mask)
    and the operating point of :804-813 (positive iff prob >= threshold: the
    PR-curve index counts thresholds strictly below it).
    Returns (probs [K] f64, sorted int64 indices)."""
    p = softmax(np.asarray(logits, np.float64), axis=-1)[:, 1]
    if ghost_mask is not None:
        p = p * ghost_mask
    return p, np.nonzero(p >= threshold)[0].astype(np.int64)


def spot_argmax(logits: np.ndarray) -> np.ndarray:
    """model/cb_whisper.py:128 — CB-Whisper keeps keywords with argmax(logits)==1
    (torch.argmax returns the first index on ties)."""
    lg = np.asarray(logits)
    return np.nonzero(lg[:, 1] > lg[:, 0])[0].astype(np.int64)
