"""ORACLE (test infrastructure only) — numpy restatement of the Whisper encoder
as the reference calls it: ``WhisperModel.from_pretrained(ckpt).encoder(
input_features, output_hidden_states=True)`` (src/model/cb_whisper.py:100-104,
src/utils.py:188-192) followed by the hs selection/normalisation of
cb_whisper.py:104-106 / utils.py:187-195.

Third-party algorithm restated: transformers==4.37.2 ``WhisperEncoder``
(installed 5.15.0, drift-checked in SURVEY.md §8c): conv1(k3,p1)·GELU,
conv2(k3,s2,p1)·GELU, + embed_positions, N pre-LN layers (self-attention with
q·d^-1/2 scaling, k without bias; GELU MLP), final LayerNorm.  hidden_states has
N+1 entries: [0] = embeddings, [i] = raw output of layer i, [N] = post-LN.
Pinned by tests/golden/encoder_micro.npz.
"""
from __future__ import annotations

import numpy as np

from oracle.common import conv1d_ncl, gelu_erf, layernorm, softmax


def encoder_hidden_states(sd: dict, mel: np.ndarray, n_heads: int) -> list:
    """mel [n_mel, 3000] -> list of N+1 arrays [1500, D] (float64)."""
    x = mel[None].astype(np.float64)
    x = gelu_erf(conv1d_ncl(x, sd["conv1.weight"], sd["conv1.bias"], 1, 1))
    x = gelu_erf(conv1d_ncl(x, sd["conv2.weight"], sd["conv2.bias"], 2, 1))
    h = x[0].T + sd["embed_positions.weight"][: x.shape[2]]
    T, D = h.shape
    hd = D // n_heads
    n_layers = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    states = [h]
    for i in range(n_layers):
        p = f"layers.{i}"
        r = h
        a = layernorm(h, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"])
        q = (a @ sd[f"{p}.self_attn.q_proj.weight"].T + sd[f"{p}.self_attn.q_proj.bias"]) * hd ** -0.5
        k = a @ sd[f"{p}.self_attn.k_proj.weight"].T
        v = a @ sd[f"{p}.self_attn.v_proj.weight"].T + sd[f"{p}.self_attn.v_proj.bias"]
        q = q.reshape(T, n_heads, hd).transpose(1, 0, 2)
        k = k.reshape(T, n_heads, hd).transpose(1, 0, 2)
        v = v.reshape(T, n_heads, hd).transpose(1, 0, 2)
        att = softmax(q @ k.transpose(0, 2, 1), axis=-1) @ v          # [H, T, hd]
        att = att.transpose(1, 0, 2).reshape(T, D)
        h = r + att @ sd[f"{p}.self_attn.out_proj.weight"].T + sd[f"{p}.self_attn.out_proj.bias"]
        r = h
        a = layernorm(h, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"])
        a = gelu_erf(a @ sd[f"{p}.fc1.weight"].T + sd[f"{p}.fc1.bias"])
        h = r + a @ sd[f"{p}.fc2.weight"].T + sd[f"{p}.fc2.bias"]
        states.append(h)
    states[-1] = layernorm(h, sd["layer_norm.weight"], sd["layer_norm.bias"])
    return states


def select_and_normalise(states: list, layer_ids) -> np.ndarray:
    """cb_whisper.py:100-106: stack(hidden_states[ids]) / ||.||_2 over D (no eps)
    -> [L, 1500, D]."""
    hs = np.stack([states[i] for i in layer_ids], 0)
    return hs / np.linalg.norm(hs, axis=-1, keepdims=True)


def default_layer_ids(n_layers: int, n_select: int = 3):
    """hidden_states[10:22][-n_select:] (cb_whisper.py:100-104 + dataset.py:570-573);
    for encoders with < 11 entries (tiny: 5) the slice is empty and the build
    uses hidden_states[-n_select:]."""
    ids = list(range(n_layers + 1))[10:22][-n_select:]
    if len(ids) < n_select:
        ids = list(range(n_layers + 1))[-n_select:]
    return ids
