"""Temperature fallback of PBAWhisper's long-form generation (src/model/pba_whisper.py:31-34 arguments, :349-351
temperature list, :425-442 ``generate_with_fallback``), restated from the transformers==4.37.2 code the reference
calls (requirements.txt:21; not vendored -- the installed 5.15.0 copy, generation_whisper.py:970-1110 and
:1243-1290, :1949-1975, was read for the parts that did not change, and its drifts are named below):

* ``compression_ratio`` -- WhisperGenerationMixin._retrieve_compression_ratio: the window's tokens as
  little-endian ``int(log2(vocab) / 8) + 1``-byte integers, raw length / zlib-compressed length (identical in
  4.37.2 and 5.15.0).
* ``avg_logprob`` -- _retrieve_avg_logprobs (4.37.2): the per-step scores HF records (processed logits; for
  sampling also temperature-scaled and top-k-masked), rescaled by the temperature, log-softmaxed; the selected
  tokens' log-probs summed with EOS excluded and divided by (number of non-EOS tokens + 1).  5.15.0 counts the
  EOS and divides by the token count (``hf5=True``).
* ``need_fallback`` -- _need_fallback: compression ratio above its threshold, or log-prob (beam search: the
  best hypothesis' ``sequences_scores``; greedy / sampling: ``avg_logprob``) below its threshold, asks for the
  next temperature; a log-prob below its threshold together with a no-speech probability above its threshold
  skips the window instead (``should_skip``: the seek moves by the window, no segment).
* ``generate_with_fallback`` -- the temperature loop for one window: temperature 0 decodes deterministically
  (greedy or beam search with the caller's num_beams), a positive temperature samples with num_beams 1; the
  window's tokens are post-processed as 4.37.2 does before the checks (EOS of a non-final window, then trailing
  pads, cbw.timestamps.strip_window); the last temperature's result stands whatever its checks say; the
  next window conditions on this one's tokens only if the temperature used was < 0.5 (``conditions_next_window``; its
  None-temperature case is parity-unpinned against 4.37.2).

The no-speech probability (WhisperNoSpeechDetection with ``no_speech_token = no_timestamps - 1``) is the
softmax probability of that token in the logits at the <|startoftranscript|> position of the window's decoder
input (``begin_index - start_of_trans_offset``); ``scores_is_logprobs`` does not change it.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def compression_ratio(tokens: Sequence[int], vocab_size: int) -> float:
    length = int(math.log2(vocab_size) / 8) + 1
    raw = b"".join(int(t).to_bytes(length, "little") for t in tokens)
    return len(raw) / len(zlib.compress(raw))


def avg_logprob(token_logprobs: Sequence[float], tokens: Sequence[int], eos: Optional[int], hf5: bool = False) -> float:
    """token_logprobs[i] = log_softmax(scores_i * rescale_temperature)[token] of the i-th recorded step, aligned as
    HF aligns them: with more steps than tokens the first len(tokens) steps, otherwise the last len(steps)
    tokens."""
    lp = list(token_logprobs)
    toks = list(tokens)
    if len(lp) > len(toks):
        lp = lp[:len(toks)]
    else:
        toks = toks[len(toks) - len(lp):]
    if hf5:
        return float(sum(lp) / len(toks))
    keep = [t != eos for t in toks] if eos is not None else [True] * len(toks)
    s = sum(v for v, k in zip(lp, keep) if k)
    return float(s / (sum(keep) + 1))


def need_fallback(tokens: Sequence[int], logprob: Optional[float], no_speech_prob: Optional[float], vocab_size: int,
                  compression_ratio_threshold: Optional[float], logprob_threshold: Optional[float],
                  no_speech_threshold: Optional[float]) -> Tuple[bool, bool]:
    """-> (needs_fallback, should_skip)."""
    needs, skip = False, False
    if compression_ratio_threshold is not None and compression_ratio(tokens, vocab_size) > compression_ratio_threshold:
        needs = True
    if logprob_threshold is not None and logprob < logprob_threshold:
        needs = True
    if no_speech_threshold is not None:
        if logprob_threshold is None:
            raise ValueError("no_speech_threshold needs logprob_threshold (transformers' _need_fallback reads both)")
        if logprob < logprob_threshold and no_speech_prob > no_speech_threshold:
            needs, skip = False, True
    return needs, skip


@dataclass
class WindowDecode:
    """One decoding attempt of a window: the generated tokens (after the decoder prefix, before any stripping),
    the log-prob the checks read (beam: the best hypothesis' score; greedy / sampling: per-step log-probs of the
    selected tokens, as ``avg_logprob`` takes them) and the no-speech probability (None when not asked for)."""
    tokens: List[int]
    sequence_score: Optional[float] = None
    token_logprobs: List[float] = field(default_factory=list)
    no_speech_prob: Optional[float] = None


@dataclass
class FallbackResult:
    tokens: List[int]           # the window's tokens after 4.37.2's post-processing
    should_skip: bool
    condition_on_prev: bool     # condition the next window on this one (temperature < 0.5)
    temperature: float          # the temperature whose result stands
    attempts: int
    raw: List[int] = field(default_factory=list)   # that attempt's generated tokens before the post-processing


def conditions_next_window(temperature: Optional[float]) -> bool:
    """Whether the window decoded at ``temperature`` lets the next window condition on its tokens: temperature < 0.5,
    and None (deterministic decoding) counted as low.  The installed transformers 5.15.0 reads, verbatim
    (generation_whisper.py:1090): ``is_low_temperature = temperature is None or temperature < 0.5``.  What 4.37.2
    (the pinned version) does for a None temperature is not restated from its source here -- PARITY UNPINNED: no
    fixture or reference run covers a None temperature in the fallback loop (the reference configs pass
    temperature=0, which both versions treat as low).  Kept in this one helper so a 4.37.2 difference is a one-line
    change."""
    return temperature is None or temperature < 0.5


def generate_with_fallback(decode: Callable[[float], WindowDecode], temperatures: Sequence[Optional[float]],
                           eos: int, pad: int, is_final: bool, vocab_size: int,
                           compression_ratio_threshold: Optional[float] = None,
                           logprob_threshold: Optional[float] = None, no_speech_threshold: Optional[float] = None,
                           condition_on_prev_tokens: bool = False) -> FallbackResult:
    """decode(temperature) runs one attempt (temperature None / 0: deterministic)."""
    from .timestamps import strip_window
    temps = list(temperatures) if temperatures else [None]
    res = None
    for i, t in enumerate(temps):
        out = decode(t)
        seq = strip_window(out.tokens, eos, pad, is_final)
        if out.sequence_score is not None:
            lp = out.sequence_score
        elif logprob_threshold is not None:
            lp = avg_logprob(out.token_logprobs, seq, eos)
        else:
            lp = None
        needs, skip = need_fallback(seq, lp, out.no_speech_prob, vocab_size, compression_ratio_threshold,
                                    logprob_threshold, no_speech_threshold)
        res = FallbackResult(seq, skip, bool(condition_on_prev_tokens and conditions_next_window(t)),
                             0.0 if t is None else float(t), i + 1, list(out.tokens))
        if not needs:
            break
    return res


def sample_step_logprob(scores: np.ndarray, token: int, temperature: float, top_k: int = 50) -> float:
    """log_softmax(scores * T)[token] over HF's recorded sampling scores (processed logits / T, all but the top_k
    set to -inf) -- the quantity ``avg_logprob`` sums for a sampled step (reference for tests; the GPU sampler
    computes the same on the device)."""
    x = np.asarray(scores, np.float64)
    kth = np.sort(x)[-top_k] if x.size > top_k else -np.inf
    w = np.where(x >= kth, x / temperature, -np.inf)
    w = w * temperature
    m = w.max()
    return float(w[token] - (m + np.log(np.exp(w - m).sum())))
