"""Temperature fallback of PBAWhisper long-form generation (cbw.fallback; reference pba_whisper.py:31-34, :349-351,
:425-442 -> transformers 4.37.2 generate_with_fallback / _need_fallback / _retrieve_compression_ratio /
_retrieve_avg_logprobs).

Pinned to the installed transformers (5.15.0) where the function did not change (the compression ratio; the
5.x form of the average log-prob, ``hf5=True``, incl. HF's step/token alignment); the 4.37.2 form and the
fallback loop are checked against an independent restatement of the 4.37.2 loop written out in this file, on
recorded window outputs (token sequences + per-step log-probs + no-speech probabilities per temperature).
"""
import math
import zlib

import numpy as np
import pytest
import torch

from cbw import fallback as fb
from cbw.timestamps import longform_generate

EOS = 50257


def _hf():
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin
    return WhisperGenerationMixin


def test_compression_ratio_matches_transformers():
    rng = np.random.default_rng(0)
    cases = [rng.integers(0, 51865, 60).tolist(), [50364, 440, 50370] * 40, list(range(300)), [7] * 200, [220]]
    for toks in cases:
        want = _hf()._retrieve_compression_ratio(torch.tensor(toks), 51865)
        assert fb.compression_ratio(toks, 51865) == pytest.approx(want, rel=0, abs=0)
    # the byte width follows the vocabulary: 2 bytes below 65 536 tokens
    raw = b"".join(int(t).to_bytes(2, "little") for t in cases[1])
    assert fb.compression_ratio(cases[1], 51865) == len(raw) / len(zlib.compress(raw))
    assert fb.compression_ratio(cases[1], 51865) > 2.4 > fb.compression_ratio(cases[0], 51865)


@pytest.mark.parametrize("n_steps,n_tokens,temp", [(10, 10, 0.0), (12, 9, 0.2), (7, 11, 0.6), (5, 5, 1.0)])
def test_avg_logprob_alignment_and_forms(n_steps, n_tokens, temp):
    rng = np.random.default_rng(n_steps * 31 + n_tokens)
    V = 300
    scores = [torch.from_numpy(rng.standard_normal((1, V)).astype(np.float32))[0] * 3 for _ in range(n_steps)]
    toks = rng.integers(0, V, n_tokens)
    toks[-1] = 17   # an "EOS" inside the vocabulary of this test
    rescale = temp if temp > 0 else 1
    # per-step log-probs of the tokens as HF aligns them (first len(tokens) steps, or the last len(steps) tokens)
    steps = scores[:n_tokens] if n_steps > n_tokens else scores
    tk = toks if n_steps > n_tokens else toks[n_tokens - n_steps:]
    lps = [float(torch.log_softmax(s * rescale, -1)[t]) for s, t in zip(steps, tk)]
    pad = [0.0] * (max(0, n_steps - n_tokens))
    # 5.x form == the installed transformers
    want5 = float(_hf()._retrieve_avg_logprobs(scores, torch.from_numpy(toks), temp))
    assert fb.avg_logprob(lps + pad, toks.tolist(), 17, hf5=True) == pytest.approx(want5, abs=1e-5)
    # 4.37.2 form: EOS excluded from the sum, divided by (non-EOS count + 1)
    keep = [t != 17 for t in tk]
    want4 = sum(v for v, k in zip(lps, keep) if k) / (sum(keep) + 1)
    assert fb.avg_logprob(lps + pad, toks.tolist(), 17) == pytest.approx(want4, abs=1e-12)


def test_sample_step_logprob_is_top_k_log_softmax():
    rng = np.random.default_rng(5)
    x = rng.standard_normal(200) * 2
    tok = int(np.argsort(-x)[3])
    top = np.sort(x)[-50:]
    want = x[tok] - (top.max() + np.log(np.exp(top - top.max()).sum()))
    assert fb.sample_step_logprob(x, tok, 0.4) == pytest.approx(want, abs=1e-12)
    assert fb.sample_step_logprob(x, int(np.argmin(x)), 0.4) == -np.inf   # outside the top 50


def test_need_fallback_truth_table():
    rep = [50364, 440, 50370] * 40          # compression ratio ~ 40
    ok = list(range(1000, 1060))              # ratio < 1
    V = 51865
    assert fb.need_fallback(ok, -0.2, 0.1, V, compression_ratio_threshold=2.4, logprob_threshold=-1.0,
                            no_speech_threshold=0.6) == (False, False)
    assert fb.need_fallback(rep, -0.2, 0.1, V, 2.4, -1.0, 0.6)[0]
    assert fb.need_fallback(ok, -1.5, 0.1, V, 2.4, -1.0, 0.6) == (True, False)
    assert fb.need_fallback(ok, -1.5, 0.9, V, 2.4, -1.0, 0.6) == (False, True)    # silence: skip
    assert fb.need_fallback(rep, -1.5, 0.9, V, 2.4, -1.0, 0.6) == (False, True)   # skip overrides
    assert fb.need_fallback(ok, -0.5, 0.9, V, 2.4, -1.0, 0.6) == (False, False)   # confident speech
    assert fb.need_fallback(rep, None, None, V, None, None, None) == (False, False)
    with pytest.raises(ValueError):
        fb.need_fallback(ok, None, 0.9, V, None, None, 0.6)


def _reference_loop_437(recorded, temperatures, is_final, cr, lp_thr, ns_thr, cond_flag, num_beams):
    """generate_with_fallback of transformers 4.37.2 for one window, written out independently over recorded
    outputs: recorded[t] = (generated tokens, per-step token log-probs or a beam sequence score, no-speech prob)."""
    for idx, t in enumerate(temperatures):
        toks, lp_src, nsp = recorded[t]
        seq = list(toks)
        if not is_final and seq[-1] == EOS:      # make sure we cut a predicted EOS token if not final
            seq = seq[:-1]
        if seq and seq[-1] == EOS:               # remove all padding tokens (pad == eos)
            n = sum(1 for x in seq if x == EOS)
            seq = seq[:-n]
        needs, skip = False, False
        if cr is not None:
            b = b"".join(x.to_bytes(2, "little") for x in seq)
            if len(b) / len(zlib.compress(b)) > cr:
                needs = True
        if lp_thr is not None:
            if num_beams > 1 and (t is None or t == 0):
                logprob = lp_src
            else:
                lps = list(lp_src)
                tk = list(seq)
                if len(lps) > len(tk):
                    lps = lps[:len(tk)]
                else:
                    tk = tk[len(tk) - len(lps):]
                s = sum(v for v, x in zip(lps, tk) if x != EOS)
                logprob = s / (sum(1 for x in tk if x != EOS) + 1)
            if logprob < lp_thr:
                needs = True
        if ns_thr is not None and logprob < lp_thr and nsp > ns_thr:
            needs, skip = False, True
        # (the None case restates cbw.fallback.conditions_next_window, read from transformers 5.15: parity-unpinned
        # against 4.37.2, so this oracle cannot catch a difference there -- the temperatures below are never None)
        cond = cond_flag and (t is None or t < 0.5)
        if not needs or idx == len(temperatures) - 1:
            return seq, skip, cond, t


def _recorded_windows(rng):
    """Recorded outputs of one window per temperature: (tokens incl. a final EOS, per-step log-probs, no-speech p)."""
    out = []
    for case in range(40):
        rec = {}
        for t in (0.0, 0.2, 0.4, 0.6, 0.8, 1.0):
            n = int(rng.integers(3, 40))
            if rng.random() < 0.3:   # a repetition loop: high compression ratio
                toks = ([int(rng.integers(220, 5000))] * 3 + [50364 + int(rng.integers(0, 30))]) * (n // 4 + 1)
            else:
                toks = rng.integers(220, 50000, n).tolist()
            toks = toks + [EOS]
            lps = (-np.abs(rng.standard_normal(len(toks))) * rng.uniform(0.1, 2.5)).tolist()
            rec[t] = (toks, lps, float(rng.uniform(0, 1)))
        out.append(rec)
    return out


@pytest.mark.parametrize("thresholds", [(2.4, -1.0, 0.6), (2.4, -1.0, None), (None, -0.8, None), (1.8, None, None)])
@pytest.mark.parametrize("is_final", [False, True])
def test_generate_with_fallback_matches_437_loop_on_recorded_windows(thresholds, is_final):
    rng = np.random.default_rng(hash((thresholds, is_final)) % 2 ** 32)
    temps = [0.0, 0.2, 0.4, 0.6, 0.8, 1.0]
    cr, lp_thr, ns_thr = thresholds
    seen = set()
    for rec in _recorded_windows(rng):
        calls = []

        def decode(t):
            calls.append(t)
            toks, lps, nsp = rec[t]
            return fb.WindowDecode(list(toks), None, list(lps), nsp)
        got = fb.generate_with_fallback(decode, temps, EOS, EOS, is_final, 51865, cr, lp_thr, ns_thr, True)
        seq, skip, cond, t_used = _reference_loop_437(rec, temps, is_final, cr, lp_thr, ns_thr, True, 1)
        assert (got.tokens, got.should_skip, got.condition_on_prev, got.temperature) == (seq, skip, cond, t_used)
        assert calls == temps[:got.attempts]
        seen.add((got.attempts, got.should_skip))
    assert len(seen) >= 2   # the cases exercise first-try and fallback outcomes (and skips with no_speech)
    if ns_thr is not None:
        assert any(skip for _, skip in seen)


def test_beam_attempt_uses_the_sequence_score():
    """Temperature 0 with beams: the logprob check reads HF's sequences_scores (the best hypothesis' length-
    normalised score) instead of averaging per-step log-probs."""
    toks = list(range(1000, 1020)) + [EOS]
    rec = {0.0: (toks, -1.2, 0.1), 0.2: (toks[:5] + [EOS], [-0.1] * 6, 0.1)}

    def decode(t):
        tk, lp, nsp = rec[t]
        return fb.WindowDecode(list(tk), lp if t == 0.0 else None, [] if t == 0.0 else lp, nsp)
    got = fb.generate_with_fallback(decode, [0.0, 0.2], EOS, EOS, False, 51865, None, -1.0, None, True)
    assert got.temperature == 0.2 and got.attempts == 2 and got.tokens == toks[:5]
    assert not got.condition_on_prev or 0.2 < 0.5
    want = _reference_loop_437(rec, [0.0, 0.2], False, None, -1.0, None, True, 5)
    assert (got.tokens, got.should_skip, got.condition_on_prev, got.temperature) == want


def test_longform_loop_skips_and_drops_conditioning():
    """The seek loop with a fallback hook: a skipped window moves the seek by the window and adds no segment;
    a window decoded at temperature >= 0.5 stops the next window from conditioning on previous tokens."""
    TB, SOP, INIT = 50365, 50362, [50258, 50259, 50360]
    prefixes = []
    results = iter([
        fb.FallbackResult([TB, 400, 401, TB + 100, TB + 100], False, True, 0.0, 1),   # closed segment -> seek 200
        fb.FallbackResult([1, 2], True, True, 0.0, 6),                                # silence: skipped
        fb.FallbackResult([TB, 500, 501, TB + 50, TB + 50], False, False, 0.6, 4),    # hot: next not conditioned
        fb.FallbackResult([TB, 600, TB + 10], False, True, 0.0, 1),                   # single ending
    ])

    def fallback(seg, prefix, begin, is_final):
        prefixes.append(list(prefix))
        return next(results)
    toks, segs = longform_generate(6300, lambda s, n: (s, n), lambda seg: [], None, INIT, SOP, EOS, TB, True,
                                   fallback=fallback)
    assert [p[0] for p in prefixes] == [INIT[0], SOP, SOP, INIT[0]]
    assert prefixes[1] == [SOP, TB, 400, 401, TB + 100] + INIT   # the closed segment's tokens
    assert prefixes[3] == INIT   # the previous window ran at 0.6: no conditioning
    starts = [round(s["start"], 2) for s in segs]
    # window 1 seeks to its closed segment's end (200 frames); window 2 is skipped (200 -> 3200); window 3 seeks
    # 100 frames (-> 3300); window 4 ends on a single timestamp and takes the rest (3300 -> 6300)
    assert starts == [0.0, 32.0, 33.0]
    assert toks == [TB, 400, 401, TB + 100, TB, 500, 501, TB + 50, TB, 600, TB + 10]
