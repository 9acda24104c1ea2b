"""ORACLE (test infrastructure only) — numpy primitives shared by the
restatements in this directory: NCHW conv via im2col, eval BatchNorm, pooling,
GELU, LayerNorm.  Semantics are those of torch.nn.{Conv1d,Conv2d,BatchNorm*d,
MaxPool*d,LayerNorm,GELU} as used by the reference path; never imported by the
product."""
from __future__ import annotations

import math

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view


def relu(x):
    return np.maximum(x, 0)


def softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / np.sum(e, axis=axis, keepdims=True)


def gelu_erf(x):
    """torch.nn.GELU() / ACT2FN['gelu'] (exact erf form)."""
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def conv2d_nchw(x: np.ndarray, w: np.ndarray, stride: int, pad: int, bias=None) -> np.ndarray:
    """torch.nn.functional.conv2d (zero padding, groups=1) via im2col + float32
    BLAS, batched over N to bound memory."""
    N, C, H, W = x.shape
    O, Ci, kh, kw = w.shape
    assert Ci == C
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    wm = w.reshape(O, -1).astype(np.float32).T                      # [C*kh*kw, O]
    out = np.empty((N, O, Ho, Wo), np.float32)
    xp = np.pad(x.astype(np.float32), ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    per = max(1, int(2e8 // max(1, C * kh * kw * Ho * Wo * 4)))
    for n0 in range(0, N, per):
        xs = xp[n0:n0 + per]
        v = sliding_window_view(xs, (kh, kw), axis=(2, 3))[:, :, ::stride, ::stride][:, :, :Ho, :Wo]
        # v: [n, C, Ho, Wo, kh, kw] -> [n, Ho, Wo, C, kh, kw]
        cols = np.ascontiguousarray(v.transpose(0, 2, 3, 1, 4, 5)).reshape(-1, C * kh * kw)
        r = (cols @ wm).reshape(xs.shape[0], Ho, Wo, O).transpose(0, 3, 1, 2)
        out[n0:n0 + per] = r
    if bias is not None:
        out += bias.reshape(1, -1, 1, 1)
    return out


def conv1d_ncl(x: np.ndarray, w: np.ndarray, b, stride: int, pad: int) -> np.ndarray:
    """torch.nn.Conv1d on [N, C, L] (float64)."""
    N, C, L = x.shape
    O, Ci, k = w.shape
    xp = np.pad(x.astype(np.float64), ((0, 0), (0, 0), (pad, pad)))
    Lo = (L + 2 * pad - k) // stride + 1
    v = sliding_window_view(xp, k, axis=2)[:, :, ::stride][:, :, :Lo]    # [N, C, Lo, k]
    cols = v.transpose(0, 2, 1, 3).reshape(N, Lo, C * k)
    out = cols @ w.reshape(O, -1).T.astype(np.float64)                   # [N, Lo, O]
    if b is not None:
        out = out + b
    return out.transpose(0, 2, 1)


def batchnorm_eval(x, weight, bias, mean, var, axis=1, eps=1e-5):
    """torch BatchNorm (eval): (x - running_mean) / sqrt(running_var + eps) * w + b."""
    shape = [1] * x.ndim
    shape[axis] = -1
    inv = 1.0 / np.sqrt(var.astype(np.float64) + eps)
    return ((x - mean.reshape(shape)) * (inv * weight).reshape(shape) + bias.reshape(shape)).astype(x.dtype)


def maxpool2d_nchw(x, k, s, p):
    """torch.nn.MaxPool2d(k, s, p): padding is -inf."""
    N, C, H, W = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (p, p), (p, p)), constant_values=-np.inf)
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    v = sliding_window_view(xp, (k, k), axis=(2, 3))[:, :, ::s, ::s][:, :, :Ho, :Wo]
    return v.max(axis=(4, 5))


def maxpool1d_ncl(x, k, s, p):
    """torch.nn.MaxPool1d(k, s, p) on [..., L]: padding is -inf."""
    pads = [(0, 0)] * (x.ndim - 1) + [(p, p)]
    xp = np.pad(x, pads, constant_values=-np.inf)
    L = x.shape[-1]
    Lo = (L + 2 * p - k) // s + 1
    v = sliding_window_view(xp, k, axis=-1)[..., ::s, :][..., :Lo, :]
    return v.max(axis=-1)


def layernorm(x, w, b, eps=1e-5):
    x = x.astype(np.float64)
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + eps) * w + b
