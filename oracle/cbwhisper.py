"""ORACLE (test infrastructure only) — numpy restatement of ``CBWhisper.keyword_spotting``
(src/model/cb_whisper.py:82-149) with the reference's own spotter: only ``tests/`` may import it.

Per segment of ``input_features`` [S, n_mel, 3000]:
  1. encoder ``hidden_states[10:22]`` stacked and L2-normalised per frame (:98-106; oracle/encoder.py);
  2. per keyword group of the database (:110-129): similarity matrices ``matmul(kwd_hs, utt_hs^T)`` and the
     bilinear resize to ``kws_features_size`` -- or to (longest keyword of the group, utterance frames) when
     it is None (:189-210; oracle/cnn12.py) -- the 12-channel ResNet-50 (model/model.py:78-93) and
     ``argwhere(argmax(logits) == 1)`` (:128);
  3. duplicates removed (:132); the prompt ``prepend + sep.join(keywords) + append`` through
     ``get_prompt_ids``, with ``<|startofprev|>`` kept only when ``start_of_prev`` (:140-147).
The reference's ``set`` (:132) leaves the keyword order undefined; the restatement keeps database order,
as the build does, so prompts compare exactly.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from oracle.cnn12 import cnn_forward, resize_bilinear, sim_matrices
from oracle.encoder import encoder_hidden_states


def utterance_hs(enc_sd: dict, mel: np.ndarray, n_heads: int, layer_ids: Optional[Sequence[int]] = None) -> np.ndarray:
    """cb_whisper.py:100-106 for one segment: [n_mel, 3000] -> [12, 1500, D] (float64, unit rows)."""
    states = encoder_hidden_states({k: np.asarray(v, np.float64) for k, v in enc_sd.items()}, mel, n_heads)
    sel = states[10:22] if layer_ids is None else [states[i] for i in layer_ids]
    hs = np.stack(sel, 0)
    return hs / np.linalg.norm(hs, axis=-1, keepdims=True)


def spot_segment(cnn_sd: dict, utt_hs: np.ndarray, kwd_hs: Sequence[np.ndarray], keywords: Sequence[str],
                 keywords_per_group: int, kws_features_size=(150, 750)) -> Tuple[List[str], np.ndarray]:
    """(deduplicated spotted keywords in database order, logits [K, 2])."""
    K = len(keywords)
    g = keywords_per_group if keywords_per_group > 0 else K
    logits = []
    for lo in range(0, K, g):
        hs = kwd_hs[lo:lo + g]
        size = tuple(kws_features_size) if kws_features_size is not None else \
            (max(h.shape[1] for h in hs), utt_hs.shape[1])
        maps = np.stack([resize_bilinear(m, size) for m in sim_matrices(hs, utt_hs)])
        logits.append(cnn_forward(cnn_sd, maps))
    logits = np.concatenate(logits, 0)
    hit = np.nonzero(np.argmax(logits, axis=1) == 1)[0]
    return [keywords[i] for i in sorted(set(hit.tolist()))], logits


def keyword_spotting(enc_sd: dict, n_heads: int, input_features: np.ndarray, cnn_sd: dict,
                     kwd_hs: Sequence[np.ndarray], keywords: Sequence[str], get_prompt_ids: Callable[[str], List[int]],
                     keywords_per_group: int = 100, kws_features_size=(150, 750), prepend: str = "(",
                     append: str = ")", sep: str = " ", start_of_prev: bool = False):
    """-> (keyword lists per segment, prompt ids per segment, logits per segment)."""
    kws, ids, lgs = [], [], []
    for mel in input_features:
        words, lg = spot_segment(cnn_sd, utterance_hs(enc_sd, mel, n_heads), kwd_hs, keywords, keywords_per_group,
                                 kws_features_size)
        kws.append(words)
        lgs.append(lg)
        if not words:
            ids.append([])
            continue
        p = get_prompt_ids(prepend + sep.join(words) + append)
        ids.append(list(p) if start_of_prev else list(p)[1:])
    return kws, ids, lgs
