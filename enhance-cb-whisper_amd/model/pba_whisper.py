"""model.pba_whisper.PBAWhisper — MI355X drop-in for src/model/pba_whisper.py:15-548.

``generate(input_features, ..., keyword_spotting=callable)`` keeps the reference's
contract: the keyword-spotting callback is called per 30 s window and its token ids
become a ``<|startofprev|>`` prompt; ``prompt_ids`` is rejected (:281-282); a
short-form batch must be 1 (:284-285); the short-form output drops the prompt
(:338).  Encoder (cbw_encoder_hs), cross-KV, every decode step and the
log-softmax/top-k run in libcbw; the beam scorer (cbw.generate) restates HF
4.37.2 beam search on the host.

Long-form (> 3000 mel frames, :343-475) is the reference's seek loop (cbw.timestamps, restated
from the transformers 4.37.2 functions it calls): per window the keyword prompt
(keyword_spotting(segment)) and, with condition_on_prev_tokens, the previous segments' tokens
form the <|startofprev|> prefix (_prepare_decoder_input_ids, :478-548); with
timestamps (long-form always predicts them: return_timestamps None -> True, False -> ValueError, 4.37.2's
_set_return_timestamps called at :273) the decoder runs under WhisperTimeStampLogitsProcessor
(cbw_timestamp_rules on the GPU) and the window is split into segments at timestamp pairs, the seek
moving to the last closed segment (_retrieve_segment, :445-465).  Short-form with return_timestamps
runs the same processor from the first free position.  A temperature list or any of compression_ratio_threshold /
logprob_threshold / no_speech_threshold runs each window through generate_with_fallback (:425-442,
cbw.fallback; positive temperatures sample on the device with a seeded RNG); the reference configs use
temperature 0 and no thresholds, the deterministic path.
"""
from __future__ import annotations

import os
import warnings

from typing import Callable, Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from cbw.decoder import DecoderEngine
from cbw.fallback import WindowDecode, generate_with_fallback
from cbw.generate import beam_sample, beam_search, greedy
from cbw.timestamps import TimestampRules, longform_generate, longform_generate_batched
from cbw.tokens import SpecialTokens
from cbw.whisper import EncoderEngine

N_FRAMES = 3000


def shortform_prefix(prompt: Sequence[int], init: Sequence[int], max_target_positions: int = 448) -> List[int]:
    """The forced decoder prefix of a short-form window with a keyword prompt, as transformers 4.37.2
    (requirements.txt:21) WhisperGenerationMixin._set_forced_decoder_ids builds it for pba_whisper.py:287-296: the
    decoder starts at prompt[0] (<|startofprev|>), then the LAST ``-max_target_positions // 2 - 1`` (225) text prompt
    tokens (OpenAI decoding.py's cut), then the init tokens (sot, language, task, notimestamps).  pba_whisper.py:338
    still slices the output by the untruncated prompt length."""
    if not prompt:
        return list(init)
    return list(prompt[:1]) + list(prompt[1:])[-max_target_positions // 2 - 1:] + list(init)


def free_language_positions(prefix: Sequence[int], init: Sequence[int]) -> Dict:
    """Short-form ``language=None`` on a multilingual checkpoint, as transformers 4.37.2 runs it for
    pba_whisper.py:287-296: _set_forced_decoder_ids appends ``(1, None)`` when the generation config has no language
    ("automatically detect the language"), so ForceTokensLogitsProcessor leaves the position after
    <|startoftranscript|> free -- the search picks it over the whole vocabulary, conditioned on the keyword prompt --
    and forces the task (and <|notimestamps|>) tokens after it.  ``prefix`` is the forced prefix built with a
    placeholder language token (``init`` = sot, language, task[, notimestamps]).  -> {"pos": the free position (the
    forced head is prefix[:pos]), "forced": position -> token after it, "begin": the first position after the forced
    ids (begin suppression, the timestamp processor's begin_index)}."""
    pos = len(prefix) - len(init) + 1
    return {"pos": pos, "forced": {pos + 1 + i: int(t) for i, t in enumerate(init[2:])}, "begin": len(prefix)}


class PBAWhisper:
    def __init__(self, encoder_config, decoder_config, state_dict: Dict[str, object],
                 suppress_tokens: Sequence[int] = (), begin_suppress_tokens: Optional[Sequence[int]] = None,
                 max_length: int = 448, device: Optional[torch.device] = None,
                 max_initial_timestamp_index: Optional[int] = 50, tokenizer=None,
                 alignment_heads: Optional[Sequence[Sequence[int]]] = None, median_filter_width: int = 7):
        """encoder_config = (n_mel, d_model, n_layers, n_heads, ffn); decoder_config =
        (vocab, d_model, n_layers, n_heads, ffn); state_dict in HF
        WhisperForConditionalGeneration naming (model.encoder.*, model.decoder.*).  alignment_heads
        (generation_config.json) / median_filter_width (config.json): the token-level timestamps' cross-attention
        heads and smoothing.  The GPU engines are built on first use (construction itself is host-only)."""
        self._enc_sd = {k[len("model.encoder."):]: v for k, v in state_dict.items() if k.startswith("model.encoder.")}
        self._dec_sd = {k[len("model.decoder."):]: v for k, v in state_dict.items() if k.startswith("model.decoder.")}
        if not self._enc_sd or not self._dec_sd:
            raise KeyError("state_dict needs model.encoder.* and model.decoder.* entries "
                           "(WhisperForConditionalGeneration naming)")
        self.encoder_config, self.decoder_config = tuple(encoder_config), tuple(decoder_config)
        self._device = device
        self._encoder = self._decoder = None
        self._bias = self._bias_begin = None
        self.tokens = SpecialTokens(decoder_config[0])
        self.tokenizer = tokenizer
        self.max_length = max_length
        self.suppress_tokens = list(suppress_tokens)
        self.begin_suppress_tokens = [220, self.tokens.eot] if begin_suppress_tokens is None else list(begin_suppress_tokens)
        self.rules = TimestampRules(self.tokens.timestamp_begin, self.tokens.notimestamps, self.tokens.eot,
                                    max_initial_timestamp_index)
        self.alignment_heads = [list(map(int, p)) for p in alignment_heads] if alignment_heads else None
        self.median_filter_width = int(median_filter_width)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, device: Optional[torch.device] = None,
                        **overrides) -> "PBAWhisper":
        """WhisperForConditionalGeneration.from_pretrained (cb_whisper.py:57) from a local HF-format
        directory: config.json (WhisperConfig), generation_config.json (suppress_tokens,
        begin_suppress_tokens, max_initial_timestamp_index; config.json as the older fallback),
        model.safetensors / pytorch_model.bin, and the tokenizer files when present."""
        from cbw.checkpoint import load_state_dict, read_json, whisper_configs
        from cbw.tokenizer import WhisperTokenizerLite
        path = pretrained_model_name_or_path
        sd = load_state_dict(path)
        cfg = read_json(path, "config.json")
        gen = read_json(path, "generation_config.json")
        enc, dec, max_pos = whisper_configs(cfg)
        pick = lambda k, d=None: gen.get(k, cfg.get(k, d))   # noqa: E731
        tok = None
        try:
            tok = WhisperTokenizerLite.from_dir(path)
        except FileNotFoundError:
            pass
        kw = dict(suppress_tokens=pick("suppress_tokens") or (), begin_suppress_tokens=pick("begin_suppress_tokens"),
                  max_length=int(pick("max_length", max_pos) or max_pos), device=device,
                  max_initial_timestamp_index=pick("max_initial_timestamp_index", 50), tokenizer=tok,
                  alignment_heads=gen.get("alignment_heads"), median_filter_width=cfg.get("median_filter_width", 7))
        kw.update(overrides)
        return cls(enc, dec, sd, **kw)

    @property
    def encoder(self) -> EncoderEngine:
        if self._encoder is None:
            self._encoder = EncoderEngine(self.encoder_config, self._enc_sd, self._device)
        return self._encoder

    @property
    def decoder(self) -> DecoderEngine:
        if self._decoder is None:
            self._decoder = DecoderEngine(self.decoder_config, self._dec_sd, self.encoder.device, max_len=self.max_length)
        return self._decoder

    @property
    def device(self) -> torch.device:
        return self.encoder.device

    def _biases(self):
        if self._bias is None:
            base = torch.zeros(self.decoder_config[0], device=self.device)
            if self.suppress_tokens:
                base[self.suppress_tokens] = float("-inf")
            begin = base.clone()
            begin[self.begin_suppress_tokens] = float("-inf")
            self._bias, self._bias_begin = base, begin
        return self._bias, self._bias_begin

    # ------------------------------------------------------------------ pieces
    _controls: Dict = {}   # the generation controls of the generate call in progress (set / reset by generate)

    def _window_max_length(self, n_prefix: int, max_new_tokens: Optional[int]) -> int:
        """A window's max_length: the prefix + max_new_tokens, else a caller's max_length (transformers: max_new_tokens
        takes precedence when both are given), else the checkpoint's; never past the decoder's positions."""
        if max_new_tokens is not None:
            return min(self.max_length, n_prefix + max_new_tokens)
        ml = self._controls.get("max_length")
        return self.max_length if ml is None else min(self.max_length, int(ml))

    def encode(self, mel_packed: torch.Tensor) -> torch.Tensor:
        """post-LN encoder output f32 [B, 1500, D] (hidden_states[-1])."""
        return self.encoder.hidden_states(mel_packed, [self.encoder.n_layers], normalize=False)[:, 0]

    def _pack(self, input_features: torch.Tensor) -> torch.Tensor:
        """[B, n_mel, 3000] f32 -> [B, 3000, cpad] bf16 (layout of cbw_encoder_hs)."""
        B, n_mel, T = input_features.shape
        pk = torch.zeros((B, T, self.encoder.cpad), dtype=torch.bfloat16, device=self.device)
        pk[:, :, :n_mel] = input_features.to(self.device).transpose(1, 2).to(torch.bfloat16)
        return pk

    def decode_window(self, enc_out: torch.Tensor, prefix: List[int], num_beams: int,
                      max_new_tokens: Optional[int] = None, timestamps: bool = False,
                      decoder_prompt_len: int = 1, return_score: bool = False, free: Optional[Dict] = None):
        """One 30 s window from ``prefix``: greedy or HF 4.37 beam search under the suppression
        processors (begin suppression at the first free position) and, with ``timestamps``, the
        timestamp rules.  decoder_prompt_len: 1 when the prefix is forced (short-form), the prefix
        length when it is passed as decoder_input_ids (long-form, HF _beam_search).  ``return_score`` (beam
        search): (sequence, HF's sequences_scores of it).  ``free`` (``_free_language``): ``prefix`` ends at
        <|startoftranscript|>, the next position is the search's, then ``free["forced"]``; begin suppression and the
        timestamp rules start at ``free["begin"]`` (short-form ``language=None``, host bookkeeping)."""
        n_forced = 1 + len(free["forced"]) if free else 0
        max_length = self._window_max_length(len(prefix) + n_forced, max_new_tokens)
        begin_pos = free["begin"] if free else len(prefix)
        bias, bias_begin = self._biases()
        bias_at = lambda pos: bias_begin if pos == begin_pos else bias   # noqa: E731
        rows = max(1, num_beams)
        rules = self.rules if timestamps else None
        self.decoder.start(enc_out, rows)
        c = self._controls
        lp, nrs = c.get("length_penalty", 1.0), c.get("num_return_sequences", 1)
        if c.get("repetition_penalty") is not None or c.get("no_repeat_ngram_size"):
            # a caller's multiplicative / n-gram processors: scores formed with torch ops on the device logits
            step = self.decoder.processed_step_fn(2 * rows, bias_at, c.get("repetition_penalty"),
                                                  c.get("no_repeat_ngram_size") or 0, greedy=num_beams <= 1)
            if num_beams <= 1:
                return greedy(step, prefix, self.tokens.eot, max_length)
            return beam_search(step, prefix, num_beams, self.tokens.eot, max_length, length_penalty=lp,
                               decoder_prompt_len=decoder_prompt_len, return_score=return_score,
                               num_return_sequences=nrs)
        if free:
            step = self.decoder.step_fn(min(16, 2 * rows), bias_at, rules, begin_pos, free_pos=len(prefix))
            if num_beams <= 1:
                return greedy(step, prefix, self.tokens.eot, max_length, forced=free["forced"])
            return beam_search(step, prefix, num_beams, self.tokens.eot, max_length, length_penalty=lp,
                               decoder_prompt_len=decoder_prompt_len, return_score=return_score, forced=free["forced"],
                               num_return_sequences=nrs)
        if num_beams > 1 and nrs > 1:
            step = self.decoder.step_fn(min(16, 2 * rows), bias_at, rules, begin_pos)
            return beam_search(step, prefix, num_beams, self.tokens.eot, max_length, length_penalty=lp,
                               decoder_prompt_len=decoder_prompt_len, return_score=return_score,
                               num_return_sequences=nrs)
        if num_beams > 1 and os.environ.get("CBW_DEV_BEAM", "1") != "0":
            # the bookkeeping on the GPU, no host round trip per token (cbw_beam_select; same result as below)
            out = self.decoder.beam_search_dev(prefix, num_beams, self.tokens.eot, max_length, min(16, 2 * rows),
                                               bias_at, rules, begin_pos, decoder_prompt_len, length_penalty=lp,
                                               return_score=return_score)
            if out is not None:
                return out
        step = self.decoder.step_fn(min(16, 2 * rows), bias_at, rules, begin_pos)
        if num_beams <= 1:
            return greedy(step, prefix, self.tokens.eot, max_length)
        return beam_search(step, prefix, num_beams, self.tokens.eot, max_length, length_penalty=lp,
                           decoder_prompt_len=decoder_prompt_len, return_score=return_score)

    def sample_window(self, enc_out: torch.Tensor, prefix: List[int], temperature: float,
                      generator: Optional[torch.Generator], max_new_tokens: Optional[int] = None,
                      timestamps: bool = False, free: Optional[Dict] = None):
        """One window decoded token by token with the per-step log-probs of the fallback checks: temperature > 0
        samples (HF's sample loop: processors, then temperature + top-k 50 warpers, a seeded device RNG),
        temperature 0 is greedy.  -> (sequence incl. the prefix, per-step log-probs)."""
        n_forced = 1 + len(free["forced"]) if free else 0
        max_length = self._window_max_length(len(prefix) + n_forced, max_new_tokens)
        begin_pos = free["begin"] if free else len(prefix)
        bias, bias_begin = self._biases()
        bias_at = lambda pos: bias_begin if pos == begin_pos else bias   # noqa: E731
        self.decoder.start(enc_out, 1)
        return self.decoder.sample_search(prefix, self.tokens.eot, max_length, bias_at,
                                          self.rules if timestamps else None, begin_pos, temperature or 0.0,
                                          generator=generator, forced=free["forced"] if free else None,
                                          free_pos=len(prefix) if free else None)

    def beam_sample_window(self, enc_out: torch.Tensor, prefix: List[int], num_beams: int, temperature: float,
                           generator: Optional[torch.Generator], max_new_tokens: Optional[int] = None,
                           timestamps: bool = False, decoder_prompt_len: int = 1):
        """One window by beam-sample decoding (do_sample with num_beams > 1, HF 4.37.2 _beam_sample through the
        reference's short-form GenerationMixin.generate call, pba_whisper.py:318-329): the decoder step and the
        processors' masks in libcbw, the warpers (temperature, top-k 50), the draw (torch.multinomial with
        ``generator``) and BeamSearchScorer's bookkeeping in cbw.generate.beam_sample."""
        max_length = self._window_max_length(len(prefix), max_new_tokens)
        begin_pos = len(prefix)
        bias, bias_begin = self._biases()
        bias_at = lambda pos: bias_begin if pos == begin_pos else bias   # noqa: E731
        self.decoder.start(enc_out, num_beams)
        fn = self.decoder.scores_fn(bias_at, self.rules if timestamps else None, begin_pos)
        return beam_sample(fn, prefix, num_beams, self.tokens.eot, max_length, temperature, generator=generator,
                           decoder_prompt_len=decoder_prompt_len,
                           length_penalty=self._controls.get("length_penalty", 1.0))

    def _fallback_window(self, temps, num_beams, max_new_tokens, timestamps, init, generator, thresholds, cond):
        """pba_whisper.py:425-442 generate_with_fallback for one window (cbw.fallback)."""
        cr_thr, lp_thr, ns_thr = thresholds

        def run(seg, prefix, begin_index, is_final):
            enc = self.encode(self._pack(seg))
            nsp = None
            if ns_thr is not None:
                self.decoder.start(enc, 1)
                nsp = self.decoder.no_speech_prob(prefix, len(prefix) - len(init), self.tokens.nospeech)

            def attempt(t):
                if t is not None and t > 0:
                    seq, lps = self.sample_window(enc, prefix, t, generator, max_new_tokens, timestamps)
                    return WindowDecode(seq[len(prefix):], None, lps, nsp)
                if num_beams > 1:
                    seq, score = self.decode_window(enc, prefix, num_beams, max_new_tokens, timestamps=timestamps,
                                                    decoder_prompt_len=begin_index, return_score=True)
                    return WindowDecode(seq[len(prefix):], score, [], nsp)
                seq, lps = self.sample_window(enc, prefix, 0.0, generator, max_new_tokens, timestamps)
                return WindowDecode(seq[len(prefix):], None, lps, nsp)

            return generate_with_fallback(attempt, temps, self.tokens.eot, self.tokens.eot, is_final,
                                          self.decoder_config[0], cr_thr, lp_thr, ns_thr, cond)
        return run

    def detect_language(self, input_features: torch.Tensor) -> torch.Tensor:
        """The language token id of every audio's first 30 s window: the decoder's logits after
        <|startoftranscript|> restricted to the language tokens, argmax (transformers'
        WhisperGenerationMixin.detect_language; 4.37.2 leaves that position unforced inside the search instead, see
        ``generate``).  input_features [B, n_mel, T] -> LongTensor [B] on the host."""
        if self.tokens.english_only:
            raise ValueError("detect_language needs a multilingual checkpoint")
        feats = input_features[..., :N_FRAMES]
        if feats.shape[-1] < N_FRAMES:
            feats = torch.nn.functional.pad(feats, (0, N_FRAMES - feats.shape[-1]))
        lang = torch.arange(self.tokens.lang0, self.tokens.lang0 + self.tokens.n_lang, device=self.device)
        out = []
        for b in range(feats.shape[0]):
            enc = self.encode(self._pack(feats[b:b + 1]))
            self.decoder.start(enc, 1)
            self.decoder.step([self.tokens.sot], 0)
            out.append(int(lang[int(torch.argmax(self.decoder.logits_row(0)[lang]))]))
        return torch.tensor(out, dtype=torch.long)

    def _language_or_detect(self, language: Optional[str], input_features: torch.Tensor) -> Optional[str]:
        if language is not None or self.tokens.english_only:
            return language
        ids = self.detect_language(input_features).tolist()
        if any(i != ids[0] for i in ids):
            raise ValueError("Multiple languages detected when trying to predict the most likely target language for "
                             "transcription. It is currently not supported to transcribe to different languages in a "
                             "single batch. Please make sure to either force a single language by passing "
                             "`language='...'` or make sure all input audio is of the same language.")
        from cbw.tokens import LANGUAGES
        return LANGUAGES[ids[0] - self.tokens.lang0]

    # ------------------------------------------------------------------ reference API
    # generation controls of pba_whisper.py:17-43 that this build accepts only at their no-op value: passing anything
    # else raises NotImplementedError instead of being dropped (a caller's processor must not vanish silently)
    _UNSUPPORTED = {"generation_config": (None,), "logits_processor": (None,), "stopping_criteria": (None,),
                    "prefix_allowed_tokens_fn": (None,), "num_segment_frames": (None, N_FRAMES),
                    "time_precision": (0.02,)}
    _KWARGS = ("num_beams", "do_sample", "max_new_tokens", "inputs", "seed", "synced_gpus", "is_multilingual",
               "return_dict_in_generate", "num_frames")

    def generate(self, input_features: Optional[torch.Tensor] = None, generation_config=None, logits_processor=None,
                 stopping_criteria=None, prefix_allowed_tokens_fn=None, synced_gpus: bool = False,
                 return_timestamps: Optional[bool] = None, task: Optional[str] = None, language: Optional[str] = None,
                 is_multilingual: Optional[bool] = None, prompt_ids: Optional[torch.Tensor] = None,
                 condition_on_prev_tokens: Optional[bool] = None,
                 temperature: Optional[Union[float, Sequence[float]]] = None,
                 compression_ratio_threshold: Optional[float] = None, logprob_threshold: Optional[float] = None,
                 no_speech_threshold: Optional[float] = None, num_segment_frames: Optional[int] = None,
                 attention_mask: Optional[torch.Tensor] = None, time_precision: float = 0.02,
                 return_token_timestamps: Optional[bool] = None, return_segments: bool = False,
                 return_dict_in_generate: Optional[bool] = None, keyword_spotting: Optional[Callable] = None,
                 num_beams: int = 1, do_sample: bool = False, max_new_tokens: Optional[int] = None, seed: int = 0,
                 **kwargs):
        """pba_whisper.py:17-475, same parameters in the same order (:17-43).  Short-form: the keyword prompt, then HF
        generate (greedy / beam search; with do_sample, sampling at ``temperature`` with top-k 50: num_beams 1
        samples, num_beams > 1 is beam-sample; return_timestamps applies the timestamp rules).  Long-form (timestamps
        always on): the seek loop; a temperature list or any of the thresholds runs each window through
        generate_with_fallback (cbw.fallback; sampling draws from a device RNG seeded with ``seed``).

        ``language=None`` on a multilingual checkpoint: short-form leaves the language position free inside the search
        (4.37.2 forced_decoder_ids ``(1, None)``, ``free_language_positions``: greedy, beam search and sampling; a
        beam-sample call raises NotImplementedError); long-form, where 4.37.2 has no defined path (its init tokens
        would hold the None), detects the language per call from the first window (``detect_language``: the
        decoder's logits after <|startoftranscript|> restricted to the language tokens, transformers 5.x
        WhisperGenerationMixin.detect_language) -- parity unpinned against 4.37.2 there.  ``is_multilingual=False``
        with a language or task raises as 4.37.2's _set_language_and_task does.  ``synced_gpus`` has no effect (one device decodes).
        ``return_dict_in_generate`` changes nothing in long-form (4.37.2 returns sequences / segments either way);
        in short-form the reference slices the ModelOutput it then gets with ``outputs[:, len(prompt_ids):]``
        (:338), which raises TypeError -- so does this build.

        ``return_token_timestamps`` (4.37.2 _set_return_outputs / _set_num_frames / _extract_token_timestamps): a
        checkpoint without ``alignment_heads`` raises ValueError; short-form computes them on a ModelOutput that
        :338 then slices -- the TypeError above; long-form returns the same sequences, and with ``return_segments``
        every segment's "result" is {"sequences": the window's decoder output row, "token_timestamps": its token
        timestamps} (cbw.token_timestamps: the alignment heads' cross-attention weights from libcbw, DTW) -- the
        other ModelOutput fields 4.37.2 puts there (scores, attentions, beam indices) are not restated.  Without it
        "result" is the row itself (return_dict_in_generate False).  ``num_frames`` (keyword, as 4.37.2 pops it)
        crops the weights to num_frames // 2 encoder frames.

        A caller's transformers generation controls (keyword arguments the reference forwards to
        GenerationMixin.generate, :320-331): ``length_penalty`` (beam search, beam-sample, long-form windows),
        ``max_length`` (per window; ``max_new_tokens`` takes precedence), ``num_return_sequences`` (short-form beam
        search: the best that many, rows padded with EOS), ``repetition_penalty`` and ``no_repeat_ngram_size``
        (short-form greedy / beam search without timestamps, DecoderEngine.processed_step_fn), with 4.37.2's argument
        checks; pinned by tests/golden/gen_controls_micro.npz.  Other combinations of them raise NotImplementedError.

        Not restated, raising NotImplementedError when set: a caller's generation_config / logits_processor /
        stopping_criteria / prefix_allowed_tokens_fn, num_segment_frames other than 3000, time_precision other than
        0.02; any other keyword argument raises TypeError."""
        if "inputs" in kwargs:   # pba_whisper.py:232-237: the deprecated input name
            input_features = kwargs.pop("inputs")
            warnings.warn("The input name `inputs` is deprecated. Please make sure to use `input_features` instead.",
                          FutureWarning)
        num_frames = kwargs.pop("num_frames", None)
        controls = {k: kwargs.pop(k) for k in self._CONTROLS if k in kwargs and kwargs[k] is not None}
        if kwargs:
            raise TypeError(f"PBAWhisper.generate got unsupported keyword argument(s) {sorted(kwargs)}")
        self._check_controls(controls, num_beams, do_sample, input_features, return_timestamps)
        self._controls = controls
        try:
            return self._generate(input_features, generation_config, logits_processor, stopping_criteria,
                                  prefix_allowed_tokens_fn, return_timestamps, task, language, is_multilingual,
                                  prompt_ids, condition_on_prev_tokens, temperature, compression_ratio_threshold,
                                  logprob_threshold, no_speech_threshold, num_segment_frames, attention_mask,
                                  time_precision, return_token_timestamps, return_segments, return_dict_in_generate,
                                  keyword_spotting, num_beams, do_sample, max_new_tokens, seed, num_frames)
        finally:
            self._controls = {}

    # a caller's transformers generation controls this build restates (the reference forwards
    # **kwargs into GenerationMixin.generate, pba_whisper.py:320-331), pinned by tests/golden/gen_controls_micro.npz
    _CONTROLS = ("length_penalty", "num_return_sequences", "max_length", "repetition_penalty", "no_repeat_ngram_size")

    def _check_controls(self, c: Dict, num_beams: int, do_sample: bool, input_features, return_timestamps):
        """transformers 4.37.2's argument checks for the restated controls (GenerationConfig.validate /
        GenerationMixin.generate), and NotImplementedError where a combination is not restated."""
        longform = input_features is not None and input_features.shape[-1] > N_FRAMES
        nrs = c.get("num_return_sequences", 1)
        if not isinstance(nrs, int) or nrs < 1:
            raise ValueError(f"`num_return_sequences` has to be a positive integer, but is {nrs}")
        if nrs > 1:
            if num_beams <= 1 and not do_sample:
                raise ValueError(f"num_return_sequences has to be 1 when doing greedy search, but is {nrs}.")
            if nrs > num_beams:
                raise ValueError("`num_return_sequences` has to be smaller or equal to `num_beams`.")
            if longform or do_sample:
                raise NotImplementedError("PBAWhisper.generate: num_return_sequences > 1 is restated for short-form "
                                          "beam search only")
        rp = c.get("repetition_penalty")
        if rp is not None and not (isinstance(rp, (int, float)) and rp > 0):
            raise ValueError(f"`penalty` has to be a strictly positive float, but is {rp}")
        ng = c.get("no_repeat_ngram_size")
        if ng is not None and (not isinstance(ng, int) or ng < 0):
            raise ValueError(f"`ngram_size` has to be a strictly positive integer, but is {ng}")
        if (rp not in (None, 1.0) or ng) and (longform or do_sample or return_timestamps):
            raise NotImplementedError("PBAWhisper.generate: repetition_penalty / no_repeat_ngram_size are restated for "
                                      "short-form greedy and beam search without timestamps only")
        ml = c.get("max_length")
        if ml is not None and (not isinstance(ml, int) or ml < 1):
            raise ValueError(f"`max_length` has to be a positive integer, but is {ml}")

    def _generate(self, input_features, generation_config, logits_processor, stopping_criteria,
                  prefix_allowed_tokens_fn, return_timestamps, task, language, is_multilingual, prompt_ids,
                  condition_on_prev_tokens, temperature, compression_ratio_threshold, logprob_threshold,
                  no_speech_threshold, num_segment_frames, attention_mask, time_precision, return_token_timestamps,
                  return_segments, return_dict_in_generate, keyword_spotting, num_beams, do_sample, max_new_tokens,
                  seed, num_frames):
        given = dict(generation_config=generation_config, logits_processor=logits_processor,
                     stopping_criteria=stopping_criteria, prefix_allowed_tokens_fn=prefix_allowed_tokens_fn,
                     num_segment_frames=num_segment_frames, time_precision=time_precision)
        for name, allowed in self._UNSUPPORTED.items():
            v = given[name]
            if isinstance(v, (list, tuple)) and len(v) == 0:   # an empty LogitsProcessorList / StoppingCriteriaList
                v = None
            if not any(v is a or (v is not None and a is not None and isinstance(v, (int, float)) and v == a)
                       for a in allowed):
                raise NotImplementedError(f"PBAWhisper.generate({name}={v!r}) is not supported by this build "
                                          f"(accepted: {', '.join(repr(a) for a in allowed)})")
        if input_features is None:
            raise ValueError("PBAWhisper.generate needs input_features")
        if is_multilingual is not None and not is_multilingual and (task is not None or language is not None):
            raise ValueError("Cannot specify `task` or `language` for an English-only model. If the model is intended "
                             "to be multilingual, pass `is_multilingual=True` to generate, or update the generation "
                             "config.")
        if is_multilingual and self.tokens.english_only:
            raise ValueError("is_multilingual=True for an English-only checkpoint (no language / task tokens)")
        if prompt_ids is not None:
            raise ValueError("PBAWhisper: you can not provide prompt_ids to the generate method.")
        if input_features.shape[-1] <= N_FRAMES and input_features.size(0) != 1:
            raise ValueError("PBAWhisper: you can not pass audios with duration of at most 30 seconds in-batch.")
        if return_token_timestamps and not self.alignment_heads:   # 4.37.2 _set_num_frames
            raise ValueError("Model generation config has no `alignment_heads`, token-level timestamps not available. "
                             "See https://gist.github.com/hollance/42e32852f24243b748ae6bc1f985b13a on how to add this "
                             "property to the generation config.")
        if (return_dict_in_generate or return_token_timestamps) and input_features.shape[-1] <= N_FRAMES:
            # the reference's short-form return, outputs[:, len(prompt_ids):] (:338), on the ModelOutput that
            # return_dict_in_generate (or return_token_timestamps, which forces it: 4.37.2 _set_return_outputs) gives
            raise TypeError("tuple indices must be integers or slices, not tuple (short-form generate with "
                            "return_dict_in_generate=True: pba_whisper.py:338 slices the ModelOutput)")
        # language=None on a multilingual checkpoint: short-form leaves the language position to the search (4.37.2
        # forced_decoder_ids (1, None)); long-form detects it first (transformers 5.x; 4.37.2 has no such path)
        free_language = language is None and not self.tokens.english_only
        if input_features.shape[-1] > N_FRAMES:
            language = self._language_or_detect(language, input_features)
        temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature]
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(seed))
        spot = keyword_spotting or (lambda input_features, start_of_prev=False: [[] for _ in range(input_features.size(0))])
        T = input_features.shape[-1]
        if T > N_FRAMES:   # _set_return_timestamps (called at pba_whisper.py:273): long-form predicts timestamps
            if return_timestamps is False:
                raise ValueError("You have passed more than 3000 mel input features (> 30 seconds) which automatically "
                                 "enables long-form generation which requires the model to predict timestamp tokens. "
                                 "Please either pass `return_timestamps=True` or make sure to pass no more than 3000 "
                                 "mel input features.")
            return_timestamps = True
        if T <= N_FRAMES:
            if input_features.size(0) != 1:
                raise ValueError("PBAWhisper: you can not pass audios with duration of at most 30 seconds in-batch.")
            prompt = list(spot(input_features=input_features, start_of_prev=True)[0])
            init = self.tokens.init_tokens(language, task, bool(return_timestamps))
            prefix = shortform_prefix(prompt, init, self.max_length)   # the returned slice drops len(prompt)
            free = None
            if free_language:   # <|startoftranscript|> ends the forced head; the language token is the search's
                free = free_language_positions(prefix, init)
                prefix = prefix[:free["pos"]]
            feats = torch.nn.functional.pad(input_features, (0, N_FRAMES - T)) if T < N_FRAMES else input_features
            enc = self.encode(self._pack(feats))
            # return_timestamps: WhisperTimeStampLogitsProcessor with begin_index = the forced ids + 1 = len(prefix)
            # (4.37.2 _retrieve_logit_processors, called at pba_whisper.py:310-316)
            ts = bool(return_timestamps)
            t = temps[0] if temps[0] is not None else 1.0
            if do_sample and not t > 0:   # 4.37.2 TemperatureLogitsWarper.__init__ (via _get_logits_warper)
                raise ValueError(f"`temperature` (={t}) has to be a strictly positive float, otherwise your next token "
                                 "scores will be invalid. If you're looking for greedy decoding strategies, set "
                                 "`do_sample=False`.")
            if do_sample and num_beams > 1:   # beam-sample (GenerationMixin._beam_sample)
                if free:
                    raise NotImplementedError("PBAWhisper.generate: beam-sample (do_sample=True, num_beams > 1) with "
                                              "language=None is not restated; pass a language")
                seq = self.beam_sample_window(enc, prefix, num_beams, t, gen, max_new_tokens, timestamps=ts)
            elif do_sample:   # HF short-form: kwargs temperature (default 1.0), the sampling warpers
                seq, _ = self.sample_window(enc, prefix, t, gen, max_new_tokens, timestamps=ts, free=free)
            else:
                seq = self.decode_window(enc, prefix, num_beams, max_new_tokens, timestamps=ts, free=free)
            if self._controls.get("num_return_sequences", 1) > 1:   # rows of equal length (BeamProcess.result)
                return torch.tensor([r[len(prompt):] for r in seq], dtype=torch.long)
            return torch.tensor([seq[len(prompt):]], dtype=torch.long)
        # long-form: the seek loop (pba_whisper.py:343-475)
        B = input_features.size(0)
        if B > 1 and attention_mask is None:   # _retrieve_max_frames_and_seek (4.37.2)
            raise ValueError("When doing batched long-form audio transcription, make sure to pass an `attention_mask`. "
                             "You can retrieve the `attention_mask` by doing `processor(audio, ..., "
                             "return_attention_mask=True)` ")
        init = self.tokens.init_tokens(language, task, bool(return_timestamps))
        thresholds = (compression_ratio_threshold, logprob_threshold, no_speech_threshold)
        use_fallback = len(temps) > 1 or any(t is not None and t > 0 for t in temps) or \
            any(x is not None for x in thresholds)

        def window(seek, n):
            seg = input_features[..., seek:seek + n]
            return torch.nn.functional.pad(seg, (0, N_FRAMES - seg.shape[-1])) if seg.shape[-1] < N_FRAMES else seg

        def decode(seg, prefix, begin_index):
            enc = self.encode(self._pack(seg))
            return self.decode_window(enc, prefix, num_beams, max_new_tokens, timestamps=bool(return_timestamps),
                                      decoder_prompt_len=begin_index)

        fb = self._fallback_window(temps, num_beams, max_new_tokens, bool(return_timestamps), init, gen, thresholds,
                                   bool(condition_on_prev_tokens)) if use_fallback else None
        if B > 1:
            return self._generate_batched(input_features, attention_mask, spot, init, num_beams, max_new_tokens,
                                          bool(return_timestamps), bool(condition_on_prev_tokens), fb, return_segments,
                                          bool(return_token_timestamps), num_frames)
        total = int(attention_mask[0].sum()) if attention_mask is not None else T
        result_fn = self._segment_result(bool(return_token_timestamps), num_frames) if return_segments else None
        all_tokens, segs = longform_generate(
            total, window, lambda seg: list(spot(input_features=seg)[0]), decode, init, self.tokens.startofprev,
            self.tokens.eot, self.tokens.timestamp_begin, bool(condition_on_prev_tokens), self.max_length, fallback=fb,
            result_fn=result_fn)
        segments = [self._segment_out(s_) for s_ in segs]
        sequences = torch.tensor([all_tokens], dtype=torch.long)
        if return_segments:
            return {"sequences": sequences, "segments": [segments]}
        return sequences

    def _segment_result(self, token_timestamps: bool, num_frames: Optional[int]):
        """A segment's "result" (4.37.2 _retrieve_segment: seek_outputs[idx]): the window's decoder output row as a
        LongTensor, or with return_token_timestamps {"sequences": row, "token_timestamps": float32 [len(row)]} --
        the alignment heads' cross-attention weights along the row (teacher-forced in libcbw against the window's
        encoder output) through cbw.token_timestamps (variant 4.37)."""
        def fn(i, row, seg):
            seq = torch.tensor(row, dtype=torch.long)
            if not token_timestamps:
                return seq
            return {"sequences": seq, "token_timestamps": self.token_timestamps(seg, row, num_frames)}
        return fn

    def token_timestamps(self, segment: torch.Tensor, row: Sequence[int], num_frames: Optional[int] = None,
                         variant: str = "4.37", num_input_ids: Optional[int] = None) -> torch.Tensor:
        """Token-level timestamps of a decoded row (decoder input ids included) of the 30 s window ``segment``
        [1, n_mel, 3000]: float32 [len(row)] (cbw.token_timestamps.extract_token_timestamps)."""
        from cbw.token_timestamps import alignment_pairs, extract_token_timestamps
        if not self.alignment_heads:
            raise ValueError("token-level timestamps need the checkpoint's alignment_heads")
        row = [int(t) for t in row]
        if len(row) < 2:
            return torch.zeros(len(row), dtype=torch.float32)
        enc = self.encode(self._pack(segment))
        self.decoder.start(enc, 1)
        w = self.decoder.cross_attn_probs(row[:-1], alignment_pairs(self.alignment_heads))
        return extract_token_timestamps(w, self.median_filter_width, 0.02, num_frames, variant, num_input_ids)

    @staticmethod
    def _segment_out(s_):
        out = {"start": s_["start"], "end": s_["end"], "tokens": torch.tensor(s_["tokens"], dtype=torch.long)}
        if "result" in s_:
            out["result"] = s_["result"]
        return out

    def _generate_batched(self, input_features, attention_mask, spot, init, num_beams, max_new_tokens, timestamps,
                          condition_on_prev_tokens, fallback, return_segments, token_timestamps=False, num_frames=None):
        """Long-form over a batch of audios (pba_whisper.py:351-475 with batch_size > 1): per-audio lengths from the
        attention mask, one keyword_spotting call per iteration over every unfinished audio's window, the windows'
        left-padded decoder inputs (cbw.timestamps.batched_prompt_prefixes), their beam searches decoded together on
        one decoder state (DecoderEngine.beam_search_windows), per-audio segments and seeks
        (cbw.timestamps.longform_generate_batched).  Returns sequences right-padded with the pad token (eos) as
        _pad_to_max_length(current_segments, pad, padding="right") (:468-475)."""
        max_frames = [int(v) for v in attention_mask.sum(-1).tolist()]
        bias, bias_begin = self._biases()

        def window(b, seek, n):
            seg = input_features[b:b + 1, :, seek:seek + n]
            return torch.nn.functional.pad(seg, (0, N_FRAMES - seg.shape[-1])) if seg.shape[-1] < N_FRAMES else seg

        def spot_all(segs):
            kw = spot(input_features=torch.cat(segs, 0))
            return [list(k) for k in kw]

        def decode(segs, prefixes, begin):
            enc = self.encode(self._pack(torch.cat(segs, 0)))
            if num_beams > 1 and len(segs) > 1 and os.environ.get("CBW_DEV_BEAM", "1") != "0":
                max_length = self._window_max_length(len(prefixes[0]), max_new_tokens)
                bias_at = lambda pos: bias_begin if pos == begin else bias   # noqa: E731
                return self.decoder.beam_search_windows([(enc[i], prefixes[i]) for i in range(len(segs))], num_beams,
                                                        self.tokens.eot, max_length, bias_at,
                                                        self.rules if timestamps else None, begin, begin,
                                                        length_penalty=self._controls.get("length_penalty", 1.0))
            return [self.decode_window(enc[i:i + 1], prefixes[i], num_beams, max_new_tokens, timestamps=timestamps,
                                       decoder_prompt_len=begin) for i in range(len(segs))]

        seqs, segs = longform_generate_batched(
            max_frames, window, spot_all, decode, init, self.tokens.startofprev, self.tokens.eot,
            self.tokens.timestamp_begin, condition_on_prev_tokens, self.max_length, fallback=fallback,
            pad=self.tokens.eot, result_fn=self._segment_result(token_timestamps, num_frames) if return_segments else None)
        width = max((len(q) for q in seqs), default=0)
        sequences = torch.full((len(seqs), width), self.tokens.eot, dtype=torch.long)
        for b, q in enumerate(seqs):
            sequences[b, :len(q)] = torch.tensor(q, dtype=torch.long)
        if return_segments:
            segments = [[self._segment_out(s_) for s_ in sb] for sb in segs]
            return {"sequences": sequences, "segments": segments}
        return sequences
