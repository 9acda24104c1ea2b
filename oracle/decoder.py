"""ORACLE (test infrastructure only) — numpy restatement of the Whisper decoder
forward that PBAWhisper's generation runs every step (HF WhisperDecoder behind
``WhisperForConditionalGeneration.generate``, src/model/pba_whisper.py:323-331,
:425-442; transformers==4.37.2 pinned, 5.15.0 installed): token + learned
position embeddings; per layer pre-LN causal self-attention, pre-LN cross-attention
over the (post-LN) encoder output, pre-LN GELU MLP; final LayerNorm; logits =
h · embed_tokensᵀ (proj_out tied).  Teacher-forced: all positions at once.
Pinned by tests/golden/decoder_micro.npz.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from oracle.common import gelu_erf, layernorm, softmax


def _mha(xq, xkv, sd, p, n_heads, causal):
    T, D = xq.shape
    S = xkv.shape[0]
    hd = D // n_heads
    q = (xq @ sd[f"{p}.q_proj.weight"].T + sd[f"{p}.q_proj.bias"]) * hd ** -0.5
    k = xkv @ sd[f"{p}.k_proj.weight"].T
    v = xkv @ sd[f"{p}.v_proj.weight"].T + sd[f"{p}.v_proj.bias"]
    q = q.reshape(T, n_heads, hd).transpose(1, 0, 2)
    k = k.reshape(S, n_heads, hd).transpose(1, 0, 2)
    v = v.reshape(S, n_heads, hd).transpose(1, 0, 2)
    s = q @ k.transpose(0, 2, 1)
    if causal:
        s = s + np.triu(np.full((T, S), -np.inf), 1)[None]
    o = (softmax(s, axis=-1) @ v).transpose(1, 0, 2).reshape(T, D)
    return o @ sd[f"{p}.out_proj.weight"].T + sd[f"{p}.out_proj.bias"]


def decoder_logits(sd: dict, tokens, enc_out: np.ndarray, n_heads: int, last_only: bool = False) -> np.ndarray:
    """tokens [T] int, enc_out [1500, D] (post-LN encoder output) -> logits [T, V] (float64)."""
    tokens = np.asarray(tokens)
    T = tokens.shape[0]
    h = sd["embed_tokens.weight"][tokens].astype(np.float64) + sd["embed_positions.weight"][:T]
    enc = enc_out.astype(np.float64)
    n_layers = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    for i in range(n_layers):
        p = f"layers.{i}"
        a = layernorm(h, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"])
        h = h + _mha(a, a, sd, f"{p}.self_attn", n_heads, True)
        a = layernorm(h, sd[f"{p}.encoder_attn_layer_norm.weight"], sd[f"{p}.encoder_attn_layer_norm.bias"])
        h = h + _mha(a, enc, sd, f"{p}.encoder_attn", n_heads, False)
        a = layernorm(h, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"])
        h = h + gelu_erf(a @ sd[f"{p}.fc1.weight"].T + sd[f"{p}.fc1.bias"]) @ sd[f"{p}.fc2.weight"].T + sd[f"{p}.fc2.bias"]
    h = layernorm(h, sd["layer_norm.weight"], sd["layer_norm.bias"])
    if last_only:
        h = h[-1:]
    return h @ sd["embed_tokens.weight"].T.astype(np.float64)


def cross_attn_probs(sd: dict, tokens, enc_out: np.ndarray, n_heads: int, heads) -> np.ndarray:
    """The cross-attention probabilities softmax(q k^T) of the (layer, head) pairs ``heads`` along the teacher-forced
    ``tokens`` (what HF's output_attentions=True cross_attentions hold, the token-level timestamps' input) ->
    float64 [len(heads), T, 1500].  Pinned by tests/test_oracle_golden.py against HF's cross_attentions."""
    tokens = np.asarray(tokens)
    T = tokens.shape[0]
    h = sd["embed_tokens.weight"][tokens].astype(np.float64) + sd["embed_positions.weight"][:T]
    enc = enc_out.astype(np.float64)
    want = {}
    last = max(l for l, _ in heads)
    for i in range(last + 1):
        p = f"layers.{i}"
        a = layernorm(h, sd[f"{p}.self_attn_layer_norm.weight"], sd[f"{p}.self_attn_layer_norm.bias"])
        h = h + _mha(a, a, sd, f"{p}.self_attn", n_heads, True)
        a = layernorm(h, sd[f"{p}.encoder_attn_layer_norm.weight"], sd[f"{p}.encoder_attn_layer_norm.bias"])
        c = f"{p}.encoder_attn"
        D = a.shape[1]
        hd = D // n_heads
        q = ((a @ sd[f"{c}.q_proj.weight"].T + sd[f"{c}.q_proj.bias"]) * hd ** -0.5).reshape(T, n_heads, hd)
        k = (enc @ sd[f"{c}.k_proj.weight"].T).reshape(enc.shape[0], n_heads, hd)
        for hh in range(n_heads):
            want[(i, hh)] = softmax(q[:, hh] @ k[:, hh].T, axis=-1)
        h = h + _mha(a, enc, sd, c, n_heads, False)
        a = layernorm(h, sd[f"{p}.final_layer_norm.weight"], sd[f"{p}.final_layer_norm.bias"])
        h = h + gelu_erf(a @ sd[f"{p}.fc1.weight"].T + sd[f"{p}.fc1.bias"]) @ sd[f"{p}.fc2.weight"].T + sd[f"{p}.fc2.bias"]
    return np.stack([want[(int(l), int(hh))] for l, hh in heads])


def _logsumexp(x: np.ndarray) -> float:
    m = x.max()
    return float(m + np.log(np.exp(x - m).sum())) if np.isfinite(m) else float(m)


def _pre_mass_mask(scores: np.ndarray, sampled, tb: int, no_timestamps: int, eos: int,
                   max_initial_timestamp_index, at_begin: Optional[bool] = None) -> np.ndarray:
    """The rules of WhisperTimeStampLogitsProcessor.__call__ before its probability-mass test.  ``at_begin``
    (input_ids.shape[1] == begin_index) defaults to len(sampled) == 0; it is False at a position before begin_index
    (the free language position of short-form language=None), where ``sampled`` is empty too."""
    if at_begin is None:
        at_begin = len(sampled) == 0
    m = np.zeros_like(scores, dtype=np.float64)
    m[no_timestamps] = -np.inf
    last = len(sampled) >= 1 and sampled[-1] >= tb
    penult = len(sampled) < 2 or sampled[-2] >= tb
    if last:
        if penult:
            m[tb:] = -np.inf
        else:
            m[:eos] = -np.inf
    ts = [t for t in sampled if t >= tb]
    if ts:
        m[tb:(ts[-1] if (last and not penult) else ts[-1] + 1)] = -np.inf
    if at_begin:
        m[:tb] = -np.inf
        if max_initial_timestamp_index is not None:
            m[tb + max_initial_timestamp_index + 1:] = -np.inf
    return m


def timestamp_mass_margin(scores: np.ndarray, sampled, timestamp_begin: int, no_timestamps: int, eos: int,
                          max_initial_timestamp_index, at_begin: Optional[bool] = None) -> float:
    """The quantity the processor's probability-mass rule thresholds at 0: logsumexp of the timestamp
    log-probs minus the best text log-prob (> 0: every text token is masked)."""
    x = scores + _pre_mass_mask(scores, sampled, timestamp_begin, no_timestamps, eos, max_initial_timestamp_index,
                                at_begin)
    lp = x - _logsumexp(x)
    return _logsumexp(lp[timestamp_begin:]) - float(lp[:timestamp_begin].max())


def timestamp_mask(scores: np.ndarray, sampled, timestamp_begin: int, no_timestamps: int, eos: int,
                   max_initial_timestamp_index, at_begin: Optional[bool] = None) -> np.ndarray:
    """WhisperTimeStampLogitsProcessor.__call__ (transformers 4.37.2 / 5.15.0
    generation/logits_process.py, identical) for one row as an additive 0 / -inf mask over
    ``scores`` (the row's scores after the earlier processors); ``sampled`` = input_ids[begin_index:]."""
    m = _pre_mass_mask(scores, sampled, timestamp_begin, no_timestamps, eos, max_initial_timestamp_index, at_begin)
    if timestamp_mass_margin(scores, sampled, timestamp_begin, no_timestamps, eos, max_initial_timestamp_index,
                             at_begin) > 0:
        m[:timestamp_begin] = -np.inf
    return m


def oracle_step_fn(sd: dict, enc_out: np.ndarray, n_heads: int, k: int, bias_at, timestamps=None, begin_index: int = 0,
                   free_pos: Optional[int] = None):
    """cbw.generate StepFn over the oracle: re-runs the teacher-forced decoder on each
    row's full prefix (rows tracked here, reorder applied to the row histories).  Scores as
    HF beam search forms them: log_softmax(logits) + the processors' masks (suppression
    bias, then the timestamp rules when ``timestamps`` = (timestamp_begin, no_timestamps,
    eos, max_initial_timestamp_index)); ``free_pos``: a position before ``begin_index`` the
    timestamp processor still runs at (4.37.2 short-form language=None: nothing sampled yet,
    not at its begin)."""
    hist = {}

    def fn(tokens, pos, reorder_rows):
        nonlocal hist
        rows = len(tokens)
        if pos == 0:
            hist = {r: [] for r in range(rows)}
        if reorder_rows is not None:
            hist = {r: list(hist[src]) for r, src in enumerate(reorder_rows)}
        lps, ids = [], []
        for r, t in enumerate(tokens):
            hist[r].append(int(t))
            lg = decoder_logits(sd, hist[r], enc_out, n_heads, last_only=True)[0]
            b = bias_at(pos + 1)
            b = np.zeros_like(lg) if b is None else np.asarray(b, dtype=np.float64)
            if timestamps is not None and pos + 1 == free_pos:
                b = b + timestamp_mask(lg + b, [], *timestamps, at_begin=False)
            elif timestamps is not None and pos + 1 >= begin_index:
                b = b + timestamp_mask(lg + b, hist[r][begin_index:], *timestamps)
            lp = lg - _logsumexp(lg) + b
            order = np.lexsort((np.arange(lp.size), -lp))[:k]
            lps.append(lp[order])
            ids.append(order)
        return np.array(lps), np.array(ids)
    return fn


def oracle_processed_step_fn(sd: dict, enc_out: np.ndarray, n_heads: int, k: int, bias_at,
                             repetition_penalty=None, no_repeat_ngram_size: int = 0, greedy: bool = False):
    """cbw.generate StepFn over the oracle with a caller's transformers processors, in 4.37.2's order
    (generation/utils.py _get_logits_processor: RepetitionPenaltyLogitsProcessor, NoRepeatNGramLogitsProcessor, then
    SuppressTokens / SuppressTokensAtBegin = ``bias_at``) on log_softmax(logits) (beam search) or the raw logits
    (greedy).  RepetitionPenalty (logits_process.py): score = score * p where score < 0 else score / p, for every
    token of the row so far; NoRepeatNGram: -inf on each token that would complete an n-gram already in the row."""
    hist = {}

    def fn(tokens, pos, reorder_rows):
        nonlocal hist
        if pos == 0:
            hist = {r: [] for r in range(len(tokens))}
        if reorder_rows is not None:
            hist = {r: list(hist[src]) for r, src in enumerate(reorder_rows)}
        lps, ids = [], []
        for r, t in enumerate(tokens):
            hist[r].append(int(t))
            lg = decoder_logits(sd, hist[r], enc_out, n_heads, last_only=True)[0]
            x = lg.copy() if greedy else lg - _logsumexp(lg)
            if repetition_penalty is not None and repetition_penalty != 1.0:
                for tok in set(hist[r]):
                    x[tok] = x[tok] * repetition_penalty if x[tok] < 0 else x[tok] / repetition_penalty
            n = no_repeat_ngram_size
            if n > 0 and len(hist[r]) + 1 >= n:
                seq = hist[r]
                prev = tuple(seq[len(seq) - n + 1:]) if n > 1 else ()
                for i in range(len(seq) - n + 1):
                    if tuple(seq[i:i + n - 1]) == prev:
                        x[seq[i + n - 1]] = -np.inf
            b = bias_at(pos + 1)
            if b is not None:
                x = x + np.asarray(b, dtype=np.float64)
            order = np.lexsort((np.arange(x.size), -x))[:k]
            lps.append(x[order])
            ids.append(order)
        return np.array(lps), np.array(ids)
    return fn


def oracle_scores_fn(sd: dict, enc_out: np.ndarray, n_heads: int, bias_at):
    """cbw.generate.beam_sample scores function over the oracle: every row's processed log-probs for the next
    position, log_softmax(logits) + the suppression bias (HF's processors), as a float32 torch tensor [rows, V] (the
    dtype transformers samples in); the rows' histories tracked and reordered here."""
    import torch
    hist = {}

    def fn(tokens, pos, reorder_rows):
        nonlocal hist
        if pos == 0:
            hist = {r: [] for r in range(len(tokens))}
        if reorder_rows is not None:
            hist = {r: list(hist[src]) for r, src in enumerate(reorder_rows)}
        out = []
        for r, t in enumerate(tokens):
            hist[r].append(int(t))
            lg = decoder_logits(sd, hist[r], enc_out, n_heads, last_only=True)[0]
            b = bias_at(pos + 1)
            b = np.zeros_like(lg) if b is None else np.asarray(b, dtype=np.float64)
            out.append(lg - _logsumexp(lg) + b)
        return torch.from_numpy(np.array(out)).float()
    return fn
