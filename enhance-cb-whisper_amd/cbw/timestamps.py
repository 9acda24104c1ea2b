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
                      max_target_positions: int = 448, fallback: Optional[Callable] = None) -> Tuple[List[int], List[Dict]]:
    """The seek loop for one audio of ``features_total`` mel frames.  window(seek, n) -> the zero-padded
    30 s segment input; keyword_spotting(segment) -> prompt token ids (no <|startofprev|>);
    decode(segment, prefix, begin_index) -> the full decoded sequence (prefix included).
    ``fallback`` (temperature fallback, cbw.fallback): fallback(segment, prefix, begin_index, is_final) ->
    cbw.fallback.FallbackResult replaces decode + strip_window: a skipped window moves the seek by the window
    without segments, and whether the next window conditions on the previous tokens follows the temperature
    that decoded this one (pba_whisper.py:425-465).
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
        else:
            out = decode(seg_in, prefix, len(prefix))
            seq = strip_window(out[len(prefix):], eos, eos, is_final=is_final)
        if not seq:   # nothing decoded (an EOS-only window): HF's slicing of an empty tensor ends the window
            seek += n
            continue
        segs, offset = retrieve_segment(seq, time_offset, timestamp_begin, n)
        segments += segs
        seek += offset
    return [t for s in segments for t in s["tokens"]], segments
