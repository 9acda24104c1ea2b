"""ORACLE (test infrastructure only) — numpy restatement of the keyword-database preparation:
hs frame count, ghost keywords, grouping, pad/truncate + masks.

Only ``tests/`` may import this module, as the checker.  Pinned by
``tests/golden/kwdb_acl.npz`` (the reference's own ``ACL6060KeywordDataset`` run on a synthetic
split folder by ``tests/golden/make_golden.py kwdb``).
"""
from __future__ import annotations

import math

import numpy as np


def hs_frames(n_samples: int, hop: int = 160, n_max: int = 480000) -> int:
    """src/utils.py:187 — ceil(unpadded log-mel frames / 2); HF's fbank has n // hop frames
    (its last STFT frame is dropped), the feature extractor truncates to 30 s."""
    return int(math.ceil((min(n_samples, n_max) // hop) / 2.0))


def build_groups(keywords, hs, keywords_per_group: int, frames: int):
    """efficient_kws/dataset.py:1693-1796.  hs: list of [L, T, D] arrays or None (ghost)."""
    hs = list(hs)
    ghosts = [i for i, h in enumerate(hs) if h is None]
    present = [(i, h.shape) for i, h in enumerate(hs) if h is not None]
    smallest = min(present, key=lambda x: x[1][1])[0]          # :1716-1723, first of the shortest
    for i in ghosts:
        hs[i] = np.zeros_like(hs[smallest])
    kpg = len(keywords) if keywords_per_group == -1 else keywords_per_group
    groups = []
    for i in range(0, len(keywords), kpg):
        sl = hs[i:i + kpg]
        g = {"keywords": list(keywords[i:i + kpg]),
             "max_length": max(max(h.shape[1] for h in sl), 32),
             "mask": np.array([0 if j in ghosts else 1 for j in range(i, min(i + kpg, len(keywords)))]),
             "hs_lengths": np.array([h.shape[1] for h in sl]),
             "kwd": [], "kwd_mask": []}
        for h in sl:
            L, T, D = h.shape
            if frames - T >= 0:
                g["kwd"].append(np.concatenate([h, np.zeros((L, frames - T, D), h.dtype)], axis=1))
                g["kwd_mask"].append(np.concatenate([np.ones((L, T)), np.zeros((L, frames - T))], axis=1))
            else:
                g["kwd"].append(h[:, :frames])
                g["kwd_mask"].append(np.ones((L, frames)))
        g["kwd"] = np.stack(g["kwd"])
        g["kwd_mask"] = np.stack(g["kwd_mask"])
        groups.append(g)
    return groups
