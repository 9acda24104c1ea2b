"""Long-form Whisper generation pieces of the reference's PBAWhisper.generate (src/model/pba_whisper.py:343-475),
restated from the transformers==4.37.2 code it calls (requirements.txt:21; the installed 5.15.0 copies of the
same functions are cited where they were read):

* ``TimestampRules`` — the per-row state WhisperTimeStampLogitsProcessor derives from a row's sampled tokens
  (generation/logits_process.py, class WhisperTimeStampLogitsProcessor.__call__): last / penultimate token a
  timestamp, the lowest timestamp still allowed (non-decreasing; the same value again only to close a pair),
  and "nothing sampled yet" (forces a timestamp <= max_initial_timestamp_index).  The masks themselves are
  applied on the GPU (cbw_timestamp_rules) or by the oracle (oracle/decoder.py:timestamp_mask).
* ``retrieve_segment`` — WhisperGenerationMixin._retrieve_segment (4.37.2; 5.15.0 generation_whisper.py:1977):
  split a window's tokens at consecutive timestamp pairs; seek to the last closed segment's end timestamp
  (x input_stride mel frames) unless the window ends on a single timestamp (no speech after it: seek the
  whole window).
* ``strip_window`` — generate_with_fallback's post-processing of one window's tokens: the EOS of a
  non-final window is dropped, then trailing pad tokens (pad == eos for Whisper).
* ``longform_generate`` — the seek loop of pba_whisper.py:364-465 for one audio; with a ``fallback`` the
  temperature fallback of generate_with_fallback (cbw.fallback) decodes each window.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

N_FRAMES = 3000          # num_segment_frames (30 s of 10 ms mel frames)
TIME_PRECISION = 0.02    # seconds per timestamp step
INPUT_STRIDE = 2         # encoder conv stride: mel frames per timestamp step


class TimestampRules:
    def __init__(self, timestamp_begin: int, no_timestamps: int, eos: int, max_initial_timestamp_index: Optional[int]):
        self.timestamp_begin = timestamp_begin
        self.no_timestamps = no_timestamps
        self.eos = eos
        self.max_initial = -1 if max_initial_timestamp_index is None else int(max_initial_timestamp_index)

    def state(self, sampled: Sequence[int]) -> Tuple[int, int, int, int]:
        """sampled = input_ids[k, begin_index:] -> (last_was_ts, penultimate_was_ts, lowest allowed ts id,
        at_begin)."""
        tb = self.timestamp_begin
        last = len(sampled) >= 1 and sampled[-1] >= tb
        penult = len(sampled) < 2 or sampled[-2] >= tb
        floor = tb
        ts = [t for t in sampled if t >= tb]
        if ts:
            floor = ts[-1] if (last and not penult) else ts[-1] + 1
        return int(last), int(penult), int(floor), int(len(sampled) == 0)


def retrieve_segment(seq: Sequence[int], time_offset: float, timestamp_begin: int, seek_num_frames: int,
                     time_precision: float = TIME_PRECISION, input_stride: int = INPUT_STRIDE
                     ) -> Tuple[List[Dict], int]:
    is_ts = [t >= timestamp_begin for t in seq]
    single_ending = is_ts[-2:] == [False, True]
    cuts = [i + 1 for i in range(len(seq) - 1) if is_ts[i] and is_ts[i + 1]]
    segments: List[Dict] = []
    if cuts:
        if single_ending:
            cuts.append(len(seq))
        last = 0
        for c in cuts:
            toks = list(seq[last:c])
            segments.append({"start": time_offset + (toks[0] - timestamp_begin) * time_precision,
                             "end": time_offset + (toks[-1] - timestamp_begin) * time_precision,
                             "tokens": toks})
            last = c
        if single_ending:
            offset = seek_num_frames
        else:
            offset = (seq[last - 1] - timestamp_begin) * input_stride
    else:
        ts = [t for t in seq if t >= timestamp_begin]
        end_pos = seek_num_frames
        if ts and ts[-1] != timestamp_begin:
            end_pos = ts[-1] - timestamp_begin
        segments.append({"start": time_offset, "end": time_offset + end_pos * time_precision, "tokens": list(seq)})
        offset = seek_num_frames
    return segments, offset


def strip_window(seq: Sequence[int], eos: int, pad: int, is_final: bool) -> List[int]:
    seq = list(seq)
    if not is_final and seq and seq[-1] == eos:
        seq = seq[:-1]
    if seq and seq[-1] == pad:
        n = sum(1 for t in seq if t == pad)   # HF removes as many trailing tokens as there are pads
        seq = seq[:-n] if n else seq
    return seq


def prompt_prefix(keywords: Sequence[int], prev_tokens: Sequence[int], init_tokens: Sequence[int], startofprev: int,
                  condition_on_prev_tokens: bool, max_target_positions: int = 448) -> List[int]:
    """pba_whisper.py:478-548 for one audio: <|startofprev|> + last keyword tokens + last previous-window
    tokens + init tokens (the keyword share shrinks to 3/4 of the half context when conditioning)."""
    cut = max_target_positions // 2 - 1
    kw = list(keywords)
    if kw:
        kw = kw[-((cut * 3) // 4 - 1):] if condition_on_prev_tokens else kw[-(cut - 1):]
    prev: List[int] = []
    if condition_on_prev_tokens and prev_tokens:
        prev = list(prev_tokens)[-(cut - len(kw) - 1):]
    if kw or prev:
        return [startofprev] + kw + prev + list(init_tokens)
    return list(init_tokens)


def longform_generate(features_total: int, window: Callable[[int, int], object],
                      keyword_spotting: Callable[[object], List[int]],
                      decode: Callable[[object, List[int], int], List[int]], init_tokens: Sequence[int],
                      startofprev: int, eos: int, timestamp_begin: int, condition_on_prev_tokens: bool,
                      max_target_positions: int = 448, fallback: Optional[Callable] = None,
                      result_fn: Optional[Callable[[int, List[int], object], object]] = None) -> Tuple[List[int], List[Dict]]:
    """The seek loop for one audio of ``features_total`` mel frames.  window(seek, n) -> the zero-padded
    30 s segment input; keyword_spotting(segment) -> prompt token ids (no <|startofprev|>);
    decode(segment, prefix, begin_index) -> the full decoded sequence (prefix included).
    ``fallback`` (temperature fallback, cbw.fallback): fallback(segment, prefix, begin_index, is_final) ->
    cbw.fallback.FallbackResult replaces decode + strip_window: a skipped window moves the seek by the window
    without segments, and whether the next window conditions on the previous tokens follows the temperature
    that decoded this one (pba_whisper.py:425-465).
    ``result_fn(0, row, segment)`` (optional): the object each of the window's segments carries as "result" (4.37.2
    _retrieve_segment: seek_outputs[idx], the window's generate output row, decoder input ids included).
    Returns (sequence = concatenated segment tokens, segments)."""
    seek = 0
    segments: List[Dict] = []
    cond = condition_on_prev_tokens
    while seek < features_total:
        time_offset = seek * TIME_PRECISION / INPUT_STRIDE
        n = min(features_total - seek, N_FRAMES)
        seg_in = window(seek, n)
        kw = keyword_spotting(seg_in)
        prev = [t for s in segments for t in s["tokens"]]
        prefix = prompt_prefix(kw, prev, init_tokens, startofprev, cond, max_target_positions)
        is_final = seek + N_FRAMES >= features_total
        if fallback is not None:
            res = fallback(seg_in, prefix, len(prefix), is_final)
            cond = res.condition_on_prev
            if res.should_skip:
                seek += n
                continue
            seq = res.tokens
            row = list(prefix) + list(res.raw)
        else:
            out = decode(seg_in, prefix, len(prefix))
            seq = strip_window(out[len(prefix):], eos, eos, is_final=is_final)
            row = list(out)
        if not seq:   # nothing decoded (an EOS-only window): HF's slicing of an empty tensor ends the window
            seek += n
            continue
        segs, offset = retrieve_segment(seq, time_offset, timestamp_begin, n)
        if result_fn is not None:
            r = result_fn(0, row, seg_in)
            for s_ in segs:
                s_["result"] = r
        segments += segs
        seek += offset
    return [t for s in segments for t in s["tokens"]], segments


def _pad_left(rows: Sequence[Optional[Sequence[int]]], pad: int, cut_off_length: Optional[int] = None) -> List[List[int]]:
    """transformers 4.37.2 ``_pad_to_max_length(..., padding="left", bos_token_tensor=None, cut_off_length)`` over
    one token list per row (None or empty: no tokens): each row cut to its last ``cut_off_length`` tokens, then left-
    padded with ``pad`` to the longest row."""
    seqs = []
    for r in rows:
        s = list(r) if r else []
        if cut_off_length is not None:
            s = s[-cut_off_length:]   # torch slicing as the reference's: a cut of 0 keeps the whole row
        seqs.append(s)
    width = max((len(s) for s in seqs), default=0)
    return [[pad] * (width - len(s)) + s for s in seqs]


def batched_prompt_prefixes(keywords: Sequence[Sequence[int]], active_prev: Sequence[Optional[Sequence[int]]],
                            init_tokens: Sequence[int], startofprev: int, pad: int,
                            any_condition: bool, condition_prev: bool, max_target_positions: int = 448) -> List[List[int]]:
    """pba_whisper.py:478-548 (``_prepare_decoder_input_ids``) for the ``cur_bsz`` windows of one iteration of the
    batched seek loop -> one decoder input row per window, all of one length:

    * keyword tokens (one list per window) left-padded with ``pad`` to the longest, each cut to its last
      (cut * 3) // 4 - 1 (166) tokens when any audio conditions on its previous tokens (``any_condition`` =
      any(do_condition_on_prev_tokens) over the whole batch), else cut - 1 (222), cut = max_target_positions // 2 - 1;
    * with ``condition_prev`` (any_condition and audio 0 of the batch has segments, :520) the previous tokens:
      ``active_prev`` per window (the concatenated segment tokens, None when that audio does not condition),
      left-padded, each cut to its last cut - (padded keyword width) - 1 tokens;
    * [<|startofprev|>] + keywords + previous tokens + init tokens when either part is non-empty, else the init tokens.

    The rows keep their pads: transformers 4.37.2's WhisperForConditionalGeneration.prepare_inputs_for_generation
    passes ``decoder_attention_mask=None`` to the decoder, so the pads are attended as tokens at their positions and
    every window of a batch decodes as its padded row alone would."""
    cut = max_target_positions // 2 - 1
    n = len(keywords)
    if any(len(k) > 0 for k in keywords):
        kw = _pad_left(keywords, pad, (cut * 3) // 4 - 1 if any_condition else cut - 1)
    else:
        kw = [[] for _ in range(n)]
    kw_width = len(kw[0]) if n else 0
    if condition_prev:
        prev = _pad_left(active_prev, pad, cut - kw_width - 1)
    else:
        prev = [[] for _ in range(n)]
    if kw_width > 0 or (n and len(prev[0]) > 0):
        return [[startofprev] + kw[i] + prev[i] + list(init_tokens) for i in range(n)]
    return [list(init_tokens) for _ in range(n)]


def longform_generate_batched(max_frames: Sequence[int], window: Callable[[int, int, int], object],
                              keyword_spotting: Callable[[List[object]], List[List[int]]],
                              decode: Callable[[List[object], List[List[int]], int], List[List[int]]],
                              init_tokens: Sequence[int], startofprev: int, eos: int, timestamp_begin: int,
                              condition_on_prev_tokens: bool, max_target_positions: int = 448,
                              fallback: Optional[Callable] = None, pad: Optional[int] = None,
                              result_fn: Optional[Callable[[int, List[int], object], object]] = None
                              ) -> Tuple[List[List[int]], List[List[Dict]]]:
    """The seek loop of pba_whisper.py:351-465 over a batch of audios (``max_frames[b]`` mel frames each, from the
    attention mask, :353-355): per iteration the audios not yet at their end (``_maybe_reduce_batch``, :370-376,
    keeping batch order), each one's next window (window(b, seek, n) -> the zero-padded 30 s segment input,
    ``_get_input_segment``, :381-388), ONE keyword_spotting call over all of them (:391), their decoder inputs
    (batched_prompt_prefixes), their decodes (decode(segments, prefixes, begin_index) -> the full decoded sequences,
    prefixes included), then per window the post-processing, segments and seek (:444-465).  ``fallback``
    (temperature fallback): fallback(segment, prefix, begin_index, is_final) -> cbw.fallback.FallbackResult per
    window, as longform_generate.  ``result_fn(i, row, segment)`` (optional): the "result" of the segments of the iteration's
    i-th window, row = its decoder output right-padded with ``pad`` to the longest of the iteration (generate's
    batched sequences; with the fallback, the attempt that stood, padded the same way -- 4.37.2 pads per fallback
    round, a difference this restatement does not model).  Returns (per audio: concatenated segment tokens, segments)."""
    B = len(max_frames)
    pad = eos if pad is None else pad
    seek = [0] * B
    segments: List[List[Dict]] = [[] for _ in range(B)]
    cond = [bool(condition_on_prev_tokens)] * B
    while any(seek[b] < max_frames[b] for b in range(B)):
        active = [b for b in range(B) if seek[b] < max_frames[b]]
        nfr = {b: min(max_frames[b] - seek[b], N_FRAMES) for b in active}
        segs = [window(b, seek[b], nfr[b]) for b in active]
        kws = keyword_spotting(segs)
        any_cond = any(cond)
        prev = [[t for s in segments[b] for t in s["tokens"]] if cond[b] else None for b in active]
        prefixes = batched_prompt_prefixes(kws, prev, init_tokens, startofprev, pad, any_cond,
                                           any_cond and len(segments[0]) > 0, max_target_positions)
        begin = len(prefixes[0])
        finals = [seek[b] + N_FRAMES >= max_frames[b] for b in active]
        if fallback is not None:
            seqs, rows = [], []
            for i, b in enumerate(active):
                res = fallback(segs[i], prefixes[i], begin, finals[i])
                cond[b] = res.condition_on_prev
                seqs.append(None if res.should_skip else res.tokens)
                rows.append(list(prefixes[i]) + list(res.raw))
        else:
            outs = decode(segs, prefixes, begin)
            seqs = [strip_window(o[begin:], eos, pad, is_final=f) for o, f in zip(outs, finals)]
            rows = [list(o) for o in outs]
        width = max(len(r) for r in rows)
        rows = [r + [pad] * (width - len(r)) for r in rows]
        for i, b in enumerate(active):
            seq = seqs[i]
            if seq is None or not seq:   # skipped, or nothing decoded (an EOS-only window): the seek moves by the window
                seek[b] += nfr[b]
                continue
            segs_b, offset = retrieve_segment(seq, seek[b] * TIME_PRECISION / INPUT_STRIDE, timestamp_begin, nfr[b])
            if result_fn is not None:
                r = result_fn(i, rows[i], segs[i])
                for s_ in segs_b:
                    s_["result"] = r
            segments[b] += segs_b
            seek[b] += offset
    return [[t for s in segments[b] for t in s["tokens"]] for b in range(B)], segments
