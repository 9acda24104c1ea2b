"""Whisper decoder engine over libcbw (cbw_decoder_*): cross-KV precompute once per
30 s window, one decode step per token with a self-attention KV cache, beam reorder,
log-softmax + top-k with additive suppression bias.  Drives cbw.generate."""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


class DecoderEngine:
    def __init__(self, config: Tuple[int, int, int, int, int], state_dict: Dict[str, object],
                 device: Optional[torch.device] = None, max_len: int = 448):
        """config = (vocab, d_model, n_layers, n_heads, ffn_dim); HF WhisperDecoder names
        (a leading `model.decoder.` is stripped)."""
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.vocab, self.d_model, self.n_layers, self.n_heads, self.ffn = config
        self.max_len = max_len
        cfg = _lib.DecoderConfig(self.vocab, self.d_model, self.n_layers, self.n_heads, self.ffn, max_len)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_create(ctypes.byref(cfg), ctypes.byref(h)), "cbw_decoder_create")
            self.h = h
            for name, v in state_dict.items():
                for pre in ("model.decoder.", "decoder."):
                    if name.startswith(pre):
                        name = name[len(pre):]
                if name == "proj_out.weight" or not (name.startswith("layers.") or name.startswith("embed") or
                                                     name.startswith("layer_norm")):
                    continue
                a = np.ascontiguousarray(v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v),
                                         dtype=np.float32)
                _lib.check(self.lib.cbw_decoder_set_param(self.h, name.encode(), a.ctypes.data, a.size),
                           f"cbw_decoder_set_param({name})")
            _lib.check(self.lib.cbw_decoder_finalize(self.h), "cbw_decoder_finalize")
        self.vpad = self.lib.cbw_decoder_vocab_padded(self.h)
        self._state = None
        self._shape = None
        self._tok = self._logits = None

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.cbw_decoder_destroy(h)
            except Exception:
                pass

    # ------------------------------------------------------------------ window setup
    def start(self, enc_out: torch.Tensor, rows: int):
        """enc_out f32 [Benc, 1500, D] (post-LN encoder output); rows = Benc * beams."""
        enc_out = enc_out.to(self.device, torch.float32).contiguous()
        Benc = enc_out.shape[0]
        nb = self.lib.cbw_decoder_state_bytes(self.h, rows, Benc)
        if nb < 0:
            raise ValueError("rows must be a positive multiple of the encoder batch")
        if self._state is None or self._state.numel() < nb:
            self._state = torch.empty(nb, dtype=torch.uint8, device=self.device)
        self._shape = (rows, Benc)
        if self._tok is None or self._tok.numel() != rows:
            self._tok = torch.empty((rows,), dtype=torch.int32, device=self.device)
            self._logits = torch.empty((rows, self.vpad), dtype=torch.float32, device=self.device)
        self._rows = torch.empty((rows,), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_cross_kv(self.h, enc_out.data_ptr(), Benc, self._state.data_ptr(),
                                                     self._state.numel(), rows, _lib.stream_handle()),
                       "cbw_decoder_cross_kv")

    # ------------------------------------------------------------------ several windows in one step
    def start_windows(self, windows: int, beams: int):
        """State for ``windows`` windows of ``beams`` rows each decoded in lock step (cbw_decoder_step_rows):
        window w's rows are [w beams, (w + 1) beams) and attend to encoder slot w; every row at its own position
        (self._posr, device int32 [rows])."""
        rows = windows * beams
        nb = self.lib.cbw_decoder_state_bytes(self.h, rows, windows)
        if nb < 0 or rows > 16:
            raise ValueError("windows x beams must be <= 16 rows")
        if self._state is None or self._state.numel() < nb:
            self._state = torch.empty(nb, dtype=torch.uint8, device=self.device)
        self._shape = (rows, windows)
        self._tok = torch.zeros((rows,), dtype=torch.int32, device=self.device)
        self._logits = torch.zeros((rows, self.vpad), dtype=torch.float32, device=self.device)
        self._posr = torch.zeros((rows,), dtype=torch.int32, device=self.device)
        self._rows = torch.arange(rows, dtype=torch.int32, device=self.device)

    def set_window(self, slot: int, enc_out: torch.Tensor):
        """Encoder slot ``slot``'s cross-attention K/V from enc_out f32 [1500, D] (or [1, 1500, D])."""
        rows, windows = self._shape
        enc_out = enc_out.to(self.device, torch.float32).reshape(1500, self.d_model).contiguous()
        _lib.check(self.lib.cbw_decoder_cross_kv_slot(self.h, enc_out.data_ptr(), slot, windows, self._state.data_ptr(),
                                                      self._state.numel(), rows, _lib.stream_handle()),
                   "cbw_decoder_cross_kv_slot")

    def prefill_window(self, slot: int, beams: int, prefix: Sequence[int]):
        """cbw_decoder_prefill into window ``slot``'s rows: their K/V at positions 0..len-1, the last token's logits
        in each of its rows, its rows' positions set to len(prefix)."""
        rows, windows = self._shape
        r0 = slot * beams
        toks = torch.as_tensor(list(prefix), dtype=torch.int32).to(self.device)
        _lib.check(self.lib.cbw_decoder_prefill_rows(self.h, toks.data_ptr(), len(prefix), slot, r0, beams, rows,
                                                     windows, self._state.data_ptr(), self._state.numel(),
                                                     self._logits[r0].data_ptr(), _lib.stream_handle()),
                   "cbw_decoder_prefill_rows")
        self._logits[r0 + 1:r0 + beams].copy_(self._logits[r0:r0 + 1].expand(beams - 1, -1))
        self._posr[r0:r0 + beams].fill_(len(prefix))

    def step_rows(self, tokens: torch.Tensor):
        """One step of every row, row r at position self._posr[r] (tokens: device int32 [rows])."""
        rows, windows = self._shape
        _lib.check(self.lib.cbw_decoder_step_rows(self.h, tokens.data_ptr(), self._posr.data_ptr(), rows, windows,
                                                  self._state.data_ptr(), self._state.numel(), self._logits.data_ptr(),
                                                  _lib.stream_handle()), "cbw_decoder_step_rows")
        return self._logits[:, : self.vocab]

    def step(self, tokens: Sequence[int], pos: int) -> torch.Tensor:
        rows, Benc = self._shape
        self._tok.copy_(torch.as_tensor(list(tokens), dtype=torch.int32))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_step(self.h, self._tok.data_ptr(), pos, rows, Benc, self._state.data_ptr(),
                                                 self._state.numel(), self._logits.data_ptr(), _lib.stream_handle()),
                       "cbw_decoder_step")
        return self._logits[:, : self.vocab]

    def prefill(self, prefix: Sequence[int]) -> torch.Tensor:
        """The forced prefix in one pass (cbw_decoder_prefill): K/V of positions 0..len-1 in every beam row,
        the last token's logits copied to every row of the step logits; the next step() is at pos = len."""
        rows, Benc = self._shape
        toks = torch.as_tensor(list(prefix), dtype=torch.int32).to(self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_prefill(self.h, toks.data_ptr(), len(prefix), rows, Benc,
                                                    self._state.data_ptr(), self._state.numel(),
                                                    self._logits.data_ptr(), _lib.stream_handle()),
                       "cbw_decoder_prefill")
        self._logits[1:].copy_(self._logits[:1].expand(rows - 1, -1))
        return self._logits[:, : self.vocab]

    def cross_attn_probs(self, tokens: Sequence[int], heads: np.ndarray) -> torch.Tensor:
        """Cross-attention probabilities of the (layer, head) pairs ``heads`` (host int32 [2 n],
        cbw.token_timestamps.alignment_pairs) along ``tokens`` teacher-forced against the encoder output of the last
        start() (cbw_decoder_cross_attn_probs; cache row 0 is overwritten) -> f32 [n, len(tokens), 1500]."""
        rows, Benc = self._shape
        T = len(tokens)
        n = heads.size // 2
        toks = torch.as_tensor(list(tokens), dtype=torch.int32).to(self.device)
        probs = torch.empty((n, T, 1500), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_cross_attn_probs(self.h, toks.data_ptr(), T, heads.ctypes.data, n, rows, Benc,
                                                             self._state.data_ptr(), self._state.numel(),
                                                             probs.data_ptr(), _lib.stream_handle()),
                       "cbw_decoder_cross_attn_probs")
        return probs

    def reorder(self, src_rows: Sequence[int], length: int):
        rows, Benc = self._shape
        self._rows.copy_(torch.as_tensor(list(src_rows), dtype=torch.int32))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_decoder_reorder(self.h, self._rows.data_ptr(), rows, Benc, length,
                                                    self._state.data_ptr(), self._state.numel(),
                                                    _lib.stream_handle()), "cbw_decoder_reorder")

    def topk(self, k: int, bias: Optional[torch.Tensor] = None, bias_ld: int = 0) -> Tuple[np.ndarray, np.ndarray]:
        """HF beam-search scores log_softmax(logits) + bias (bias [V] shared, or [rows, bias_ld])."""
        rows = self._shape[0]
        lp = torch.empty((rows, k), dtype=torch.float32, device=self.device)
        idx = torch.empty((rows, k), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_logprob_topk(self._logits.data_ptr(), rows, self.vocab, self.vpad,
                                                 _lib.ptr(bias), bias_ld, k, lp.data_ptr(), idx.data_ptr(),
                                                 _lib.stream_handle()), "cbw_logprob_topk")
        return lp.cpu().numpy(), idx.cpu().numpy()

    def timestamp_bias(self, rules, sampled_rows, bias: Optional[torch.Tensor], states=None) -> torch.Tensor:
        """Per-row masks of WhisperTimeStampLogitsProcessor on top of the shared bias
        (cbw_timestamp_rules): -> f32 [rows, V].  ``states`` overrides the rows' rule states (TimestampRules.state)."""
        rows = self._shape[0]
        if states is None:
            states = [rules.state(s) for s in sampled_rows]
        st = torch.tensor(states, dtype=torch.int32).to(self.device)
        out = torch.empty((rows, self.vocab), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_timestamp_rules(self._logits.data_ptr(), rows, self.vocab, self.vpad,
                                                    _lib.ptr(bias), st.data_ptr(), rules.timestamp_begin,
                                                    rules.no_timestamps, rules.eos, rules.max_initial,
                                                    out.data_ptr(), _lib.stream_handle()), "cbw_timestamp_rules")
        return out

    def beam_search_dev(self, prefix: Sequence[int], num_beams: int, eos: int, max_length: int, k: int,
                        bias_at: callable, rules=None, begin_index: int = 0, decoder_prompt_len: int = 1,
                        length_penalty: float = 1.0, check_every: int = 8, return_score: bool = False):
        """cbw.generate.beam_search with the bookkeeping on the GPU: per token the
        scores (timestamp rules from a device-side state, cbw_timestamp_rules; log-softmax + top-k), the
        next-beam choice (cbw_beam_select), the KV reorder by the device parent rows and the decode step are
        enqueued without a host round trip; every ``check_every`` tokens the logged candidates are copied back
        once and replayed through the same BeamProcess the host search runs, which finds the end (EOS
        hypotheses, early stop, max_length) and the result.  Steps enqueued past the end are discarded.
        Returns None when the engine cannot run it (Benc != 1, k or rows > 16): use beam_search."""
        from .generate import BeamProcess
        rows, Benc = self._shape
        if Benc != 1 or rows != num_beams or rows > 16 or k > 16 or k != 2 * num_beams or len(prefix) < 2:
            return None
        dev = self.device
        bp = BeamProcess(prefix, num_beams, eos, max_length, length_penalty, decoder_prompt_len)
        n_max = max(1, max_length - len(prefix))
        lp = torch.empty((rows, k), dtype=torch.float32, device=dev)
        idx = torch.empty((rows, k), dtype=torch.int32, device=dev)
        scores = torch.tensor([0.0] + [-1e9] * (rows - 1), dtype=torch.float64, device=dev)
        # one log row per step, every field a column range of one byte buffer, so a replay is ONE device -> host
        # copy (six separate .cpu() calls cost ~33 copy launches per replay)
        f_cs, f_cr, f_ct = 0, 8 * k, 12 * k
        f_nt, f_nr, f_ok = 16 * k, 16 * k + 4 * rows, 16 * k + 8 * rows
        row_bytes = (f_ok + 4 + 7) // 8 * 8
        log_buf = torch.zeros((n_max, row_bytes), dtype=torch.uint8, device=dev)

        def fields(buf):
            return (buf[:, f_cs:f_cr].view(torch.float64), buf[:, f_cr:f_ct].view(torch.int32),
                    buf[:, f_ct:f_nt].view(torch.int32), buf[:, f_nt:f_nr].view(torch.int32),
                    buf[:, f_nr:f_ok].view(torch.int32), buf[:, f_ok:f_ok + 4].view(torch.int32)[:, 0])
        c_score, c_row, c_tok, nxt_tok, nxt_row, ok = fields(log_buf)
        tb = rules.timestamp_begin if rules is not None else 1 << 30
        sampled = list(prefix[begin_index:]) if begin_index < len(prefix) else []
        tsl = [t for t in sampled if t >= tb]
        ts0 = [len(sampled), sampled[-1] if sampled else -1, sampled[-2] if len(sampled) > 1 else -1,
               tsl[-1] if tsl else -1]
        ts_state = torch.tensor([ts0] * rows, dtype=torch.int32, device=dev)
        st = torch.tensor([list(rules.state(sampled)) if rules is not None else [0, 1, 0, 1]] * rows,
                          dtype=torch.int32, device=dev)
        tsb = torch.empty((rows, self.vocab), dtype=torch.float32, device=dev) if rules is not None else None
        stream = _lib.stream_handle()
        self.prefill(prefix)
        pos = len(prefix)
        s = 0
        replayed = 0

        def replay(upto):
            nonlocal replayed
            if upto <= replayed:
                return
            cs, cr, ct, nt, nr, okh = (t.numpy() for t in fields(log_buf[replayed:upto].cpu()))
            for i in range(upto - replayed):
                toks, par = bp.process([(float(cs[i, j]), int(cr[i, j]), int(ct[i, j])) for j in range(k)])
                if not bp.finished and (not okh[i] or toks != nt[i].tolist() or par != nr[i].tolist()):
                    raise RuntimeError("GPU beam bookkeeping diverged from the host replay")
                if bp.finished:
                    break
            replayed = upto

        with torch.cuda.device(dev):
            while True:
                b = bias_at(pos)
                if rules is not None and pos >= begin_index:
                    _lib.check(self.lib.cbw_timestamp_rules(self._logits.data_ptr(), rows, self.vocab, self.vpad,
                                                            _lib.ptr(b), st.data_ptr(), rules.timestamp_begin,
                                                            rules.no_timestamps, rules.eos, rules.max_initial,
                                                            tsb.data_ptr(), stream), "cbw_timestamp_rules")
                    bias, bias_ld = tsb, self.vocab
                else:
                    bias, bias_ld = b, 0
                _lib.check(self.lib.cbw_logprob_topk(self._logits.data_ptr(), rows, self.vocab, self.vpad,
                                                     _lib.ptr(bias), bias_ld, k, lp.data_ptr(), idx.data_ptr(),
                                                     stream), "cbw_logprob_topk")
                # the next tokens / parent rows go straight into this step's log rows, which the reorder and
                # the decode step then read (no per-token copies)
                tok_s, row_s = nxt_tok[s].data_ptr(), nxt_row[s].data_ptr()
                _lib.check(self.lib.cbw_beam_select(lp.data_ptr(), idx.data_ptr(), rows, k, eos, scores.data_ptr(),
                                                    c_score[s].data_ptr(), c_row[s].data_ptr(), c_tok[s].data_ptr(),
                                                    tok_s, row_s, ok[s].data_ptr(),
                                                    ts_state.data_ptr(), st.data_ptr(), tb,
                                                    int(rules is not None and pos >= begin_index), stream),
                           "cbw_beam_select")
                s += 1
                if pos + 1 >= max_length:
                    break
                _lib.check(self.lib.cbw_decoder_reorder(self.h, row_s, rows, Benc, pos,
                                                        self._state.data_ptr(), self._state.numel(), stream),
                           "cbw_decoder_reorder")
                _lib.check(self.lib.cbw_decoder_step(self.h, tok_s, pos, rows, Benc,
                                                     self._state.data_ptr(), self._state.numel(),
                                                     self._logits.data_ptr(), stream), "cbw_decoder_step")
                pos += 1
                if s - replayed >= check_every:
                    replay(s)
                    if bp.finished:
                        break
            if not bp.finished:
                replay(s)
        if not bp.finished:
            raise RuntimeError("GPU beam search ended before the host replay finished")
        seq = bp.result()
        return (seq, bp.score) if return_score else seq

    def beam_search_windows(self, windows: Sequence[Tuple[torch.Tensor, Sequence[int]]], num_beams: int, eos: int,
                            max_length: int, bias_at: callable, rules=None, begin_index: int = 0,
                            decoder_prompt_len: int = 1, length_penalty: float = 1.0, check_every: int = 8,
                            return_score: bool = False) -> List:
        """beam_search_dev for several windows at once (the windows of one iteration of the batched long-form loop,
        pba_whisper.py:425-442: HF 4.37.2 runs their beam searches as one batch, each batch element's scorer
        independent of the others): windows = [(enc_out f32 [1500, D] post-LN, decoder prefix)], decoded in lock step
        on one decoder state of ``16 // num_beams`` slots -- every row at its own position, each window on its own
        encoder slot (cbw_decoder_step_rows), windows admitted into slots as earlier ones finish.  Each window's
        bookkeeping is beam_search_dev's (cbw_beam_select, replayed on the host every ``check_every`` steps) and each
        row's logits equal a step over its window alone, so every window gets the tokens beam_search_dev gives it.
        Returns the sequences (with ``return_score``: (sequence, score) pairs) in window order."""
        if max_length > self.max_len:
            raise ValueError(f"max_length {max_length} exceeds the decoder's {self.max_len} positions")
        k = min(16, 2 * num_beams)
        slots = max(1, min(len(windows), 16 // num_beams))
        if num_beams > 16 or any(len(p) < 2 for _, p in windows):
            raise ValueError("beam_search_windows needs num_beams <= 16 and prefixes of >= 2 tokens")
        stream = _lib.stream_handle()
        results: List = [None] * len(windows)
        with torch.cuda.device(self.device):
            self.start_windows(slots, num_beams)
            rows = slots * num_beams
            inc = torch.zeros((rows,), dtype=torch.int32, device=self.device)
            tok = torch.zeros((rows,), dtype=torch.int32, device=self.device)
            ident = torch.arange(rows, dtype=torch.int32, device=self.device)
            src_rows = ident.clone()
            active: List[Optional[_WindowSearch]] = [None] * slots
            pending = list(range(len(windows)))

            def retire(w):
                inc[w.r0:w.r0 + num_beams].fill_(0)
                src_rows[w.r0:w.r0 + num_beams].copy_(ident[w.r0:w.r0 + num_beams])
                active[w.slot] = None
                if not w.bp.finished:
                    raise RuntimeError("GPU beam search ended before the host replay finished")
                seq = w.bp.result()
                results[w.index] = (seq, w.bp.score) if return_score else seq

            it = 0
            while pending or any(a is not None for a in active):
                for slot in range(slots):
                    if active[slot] is None and pending:
                        i = pending.pop(0)
                        enc_out, prefix = windows[i]
                        self.set_window(slot, enc_out)
                        self.prefill_window(slot, num_beams, prefix)
                        active[slot] = _WindowSearch(i, slot, prefix, num_beams, k, eos, max_length, rules, begin_index,
                                                     decoder_prompt_len, length_penalty, self.device, self.vocab)
                        inc[slot * num_beams:(slot + 1) * num_beams].fill_(1)
                live = [w for w in active if w is not None]
                for w in live:
                    w.score(self, bias_at, stream)
                    if not w.stopped:   # the step's tokens and (global) parent rows for this window's rows
                        tok[w.r0:w.r0 + num_beams].copy_(w.views[3][w.s - 1])
                        torch.add(w.views[4][w.s - 1], w.r0, out=src_rows[w.r0:w.r0 + num_beams])
                for w in live:   # windows at max_length: replayed now, no further steps
                    if w.stopped:
                        w.replay()
                        retire(w)
                live = [w for w in active if w is not None]
                if not live:
                    continue
                length = max(w.pos for w in live)
                _lib.check(self.lib.cbw_decoder_reorder(self.h, src_rows.data_ptr(), rows, slots, length,
                                                        self._state.data_ptr(), self._state.numel(), stream),
                           "cbw_decoder_reorder")
                self.step_rows(tok)
                self._posr.add_(inc)
                for w in live:
                    w.pos += 1
                it += 1
                if it % check_every == 0:   # one device -> host copy per window, then the finished ones leave
                    for w in live:
                        w.replay()
                        if w.bp.finished:
                            retire(w)
        return results

    def sample_search(self, prefix: Sequence[int], eos: int, max_length: int, bias_at: callable, rules=None,
                      begin_index: int = 0, temperature: float = 0.0, top_k: int = 50,
                      generator: Optional[torch.Generator] = None, forced: Optional[dict] = None,
                      free_pos: Optional[int] = None) -> Tuple[list, list]:
        """One row, token by token, with the per-step log-probs transformers' fallback checks read
        (cbw.fallback.avg_logprob): the processed scores (logits + suppression bias + timestamp rules, the
        processors of HF's greedy / sample loops) -> temperature 0: argmax (ties -> lower id, as
        cbw_logprob_topk), log-prob = log_softmax(scores)[token]; temperature T > 0: HF's sampling warpers
        (scores / T, all but the top_k set to -inf; GenerationConfig's default top_k 50), a token drawn from
        their softmax with ``generator`` (a seeded device RNG), log-prob = log_softmax(warped * T)[token].  The
        decoder step, timestamp rules and masks run in libcbw; the draw is a torch op on the device.
        ``forced`` (position -> token) / ``free_pos``: the free language position of short-form ``language=None``
        and the forced positions after it (``free_position_state``).
        Returns (full sequence incl. the prefix, per-generated-step log-probs)."""
        forced = forced or {}
        rows, Benc = self._shape
        if rows != 1 or Benc != 1:
            raise ValueError("sample_search decodes one row")
        seq = list(prefix)
        lps = []
        if len(prefix) > 1:
            self.prefill(prefix)
        else:
            self.step(list(prefix), 0)
        pos = len(prefix)
        V = self.vocab
        while len(seq) < max_length:
            if pos in forced:   # ForceTokensLogitsProcessor: the forced token at log-prob 0
                tok = int(forced[pos])
                lps.append(0.0)
                seq.append(tok)
                self.step([tok], pos)
                pos += 1
                continue
            b = bias_at(pos)
            logits = self._logits[:, :V]
            if rules is not None and pos == free_pos:
                scores = logits + self.timestamp_bias(rules, None, b, [free_position_state(rules)])
            elif rules is not None and pos >= begin_index:
                scores = logits + self.timestamp_bias(rules, [seq[begin_index:]], b)
            else:
                scores = logits + b if b is not None else logits.clone()
            if temperature and temperature > 0:
                kth = torch.topk(scores, min(top_k, V), dim=-1).values[:, -1:]
                w = torch.where(scores >= kth, scores / temperature, torch.full_like(scores, float("-inf")))
                tok = int(torch.multinomial(torch.softmax(w, -1), 1, generator=generator)[0, 0])
                lp = torch.log_softmax(w * temperature, -1)[0, tok]
            else:
                tok = int(torch.argmax(scores[0]))
                lp = torch.log_softmax(scores, -1)[0, tok]
            lps.append(float(lp))
            seq.append(tok)
            if tok == eos or len(seq) >= max_length:
                break
            self.step([tok], pos)
            pos += 1
        return seq, lps

    def logits_row(self, row: int) -> torch.Tensor:
        """The last step's fp32 logits of one row over the vocabulary (a device view)."""
        return self._logits[row, :self.vocab]

    def no_speech_prob(self, prefix: Sequence[int], sot_index: int, no_speech_token: int) -> float:
        """WhisperNoSpeechDetection: softmax(logits at the <|startoftranscript|> position)[no_speech_token] for the
        window whose decoder input is ``prefix`` (one row; the caller restarts the window before decoding)."""
        if sot_index > 0:
            self.prefill(list(prefix[:sot_index + 1]))
        else:
            self.step([prefix[0]], 0)
        return float(torch.softmax(self._logits[0, :self.vocab].double(), -1)[no_speech_token])

    def scores_fn(self, bias_at: callable, rules=None, begin_index: int = 0):
        """A cbw.generate.beam_sample scores function: reorder the KV cache, run one step, return every row's
        processed log-probs for the next position as a device tensor [rows, V]: log_softmax(logits) + the
        suppression bias (bias_at(pos)) and, with ``rules``, the per-row timestamp rules over each row's tokens since
        ``begin_index`` (the masks step_fn's top-k sees)."""
        seqs = []

        def scores(pos):
            b = bias_at(pos)
            lp = torch.log_softmax(self._logits[:, :self.vocab].float(), dim=-1)
            if rules is not None and pos >= begin_index:
                return lp + self.timestamp_bias(rules, [s[begin_index:] for s in seqs], b)
            return lp + b if b is not None else lp

        def fn(tokens, pos, reorder_rows):
            nonlocal seqs
            if pos == 0:
                seqs = [[] for _ in tokens]
            if reorder_rows is not None:
                self.reorder(reorder_rows, pos)
                seqs = [list(seqs[r]) for r in reorder_rows]
            for r, t in enumerate(tokens):
                seqs[r].append(int(t))
            self.step(tokens, pos)
            return scores(pos + 1)

        def prefill(prefix):
            nonlocal seqs
            if self._shape[1] != 1:
                return None
            seqs = [list(prefix) for _ in range(self._shape[0])]
            self.prefill(prefix)
            return scores(len(prefix))
        fn.prefill = prefill
        return fn

    def processed_step_fn(self, k: int, bias_at: callable, repetition_penalty: Optional[float] = None,
                          no_repeat_ngram_size: int = 0, greedy: bool = False):
        """A cbw.generate StepFn with a caller's repetition_penalty / no_repeat_ngram_size (4.37.2's processor order:
        RepetitionPenaltyLogitsProcessor, NoRepeatNGramLogitsProcessor, then the suppression processors) on the
        step's scores -- log_softmax(logits) for beam search, the raw logits for greedy, as HF applies its processors
        to each.  Each row's token history is the row's sequence so far (decoder prompt included).  The penalty is
        multiplicative, so the scores are formed with torch ops on the device logits and the top-k by a stable sort
        (ties -> lower id, as cbw_logprob_topk); no timestamp rules (the caller raises for that combination)."""
        seqs = []
        V = self.vocab

        def scores(pos):
            x = self._logits[:, :V].float()
            x = x.clone() if greedy else torch.log_softmax(x, dim=-1)
            for r, sq in enumerate(seqs):
                if repetition_penalty is not None and repetition_penalty != 1.0 and sq:
                    ids = torch.tensor(sorted(set(sq)), dtype=torch.long, device=x.device)
                    g = x[r, ids]
                    x[r, ids] = torch.where(g < 0, g * repetition_penalty, g / repetition_penalty)
                ban = banned_ngram_tokens(sq, no_repeat_ngram_size)
                if ban:
                    x[r, torch.tensor(ban, dtype=torch.long, device=x.device)] = float("-inf")
            b = bias_at(pos)
            if b is not None:
                x = x + b
            v, i = torch.sort(x, dim=-1, descending=True, stable=True)
            return v[:, :k].cpu().numpy(), i[:, :k].to(torch.int32).cpu().numpy()

        def fn(tokens, pos, reorder_rows):
            nonlocal seqs
            if pos == 0:
                seqs = [[] for _ in tokens]
            if reorder_rows is not None:
                self.reorder(reorder_rows, pos)
                seqs = [list(seqs[r]) for r in reorder_rows]
            for r, t in enumerate(tokens):
                seqs[r].append(int(t))
            self.step(tokens, pos)
            return scores(pos + 1)

        def prefill(prefix):
            nonlocal seqs
            if self._shape[1] != 1:
                return None
            seqs = [list(prefix) for _ in range(self._shape[0])]
            self.prefill(prefix)
            return scores(len(prefix))
        fn.prefill = prefill
        return fn

    def step_fn(self, k: int, bias_at: callable, rules=None, begin_index: int = 0, free_pos: Optional[int] = None):
        """A cbw.generate StepFn: reorder the KV cache, run one step, return the top-k of
        log_softmax(logits) + the processors' masks for the next position: the suppression bias
        (bias_at(pos) -> tensor or None) and, with ``rules`` (cbw.timestamps.TimestampRules), the
        per-row timestamp rules over each row's tokens since ``begin_index``; at ``free_pos`` (the free language
        position of short-form ``language=None``, before ``begin_index``) the rules in ``free_position_state``."""
        seqs = []

        def fn(tokens, pos, reorder_rows):
            nonlocal seqs
            if pos == 0:
                seqs = [[] for _ in tokens]
            if reorder_rows is not None:
                self.reorder(reorder_rows, pos)
                seqs = [list(seqs[r]) for r in reorder_rows]
            for r, t in enumerate(tokens):
                seqs[r].append(int(t))
            self.step(tokens, pos)
            return scores(pos + 1)

        def scores(pos):
            b = bias_at(pos)
            if rules is not None and pos == free_pos:
                return self.topk(k, self.timestamp_bias(rules, None, b, [free_position_state(rules)] * len(seqs)),
                                 self.vocab)
            if rules is None or pos < begin_index:
                return self.topk(k, b)
            return self.topk(k, self.timestamp_bias(rules, [s[begin_index:] for s in seqs], b), self.vocab)

        def prefill(prefix):
            """the forced prefix in one pass (Benc = 1): scores for position len(prefix)"""
            nonlocal seqs
            if self._shape[1] != 1:
                return None
            seqs = [list(prefix) for _ in range(self._shape[0])]
            self.prefill(prefix)
            return scores(len(prefix))
        fn.prefill = prefill
        return fn


def banned_ngram_tokens(seq: Sequence[int], n: int) -> List[int]:
    """NoRepeatNGramLogitsProcessor (transformers 4.37.2 _get_ngrams / _calc_banned_ngram_tokens) for one row: the
    tokens that would complete an n-gram already in ``seq`` (the row's tokens so far, decoder prompt included)."""
    if n <= 0 or len(seq) + 1 < n:
        return []
    prev = tuple(seq[len(seq) - n + 1:]) if n > 1 else ()
    out = []
    for i in range(len(seq) - n + 1):
        if tuple(seq[i:i + n - 1]) == prev:
            out.append(int(seq[i + n - 1]))
    return out


def free_position_state(rules) -> Tuple[int, int, int, int]:
    """WhisperTimeStampLogitsProcessor (4.37.2) at a position before its begin_index -- the free language position
    of short-form ``language=None``: input_ids[k, begin_index:] is empty (no pair rule, no floor) and
    input_ids.shape[1] != begin_index (no initial-timestamp rule); <|notimestamps|> is still suppressed and the
    timestamp-mass rule still applies.  As a cbw_timestamp_rules state (TimestampRules.state's fields)."""
    return (0, 1, int(rules.timestamp_begin), 0)


class _WindowSearch:
    """One window's beam search inside DecoderEngine.beam_search_windows: its HF 4.37.2 BeamProcess, the device log
    rows cbw_beam_select writes (one row per step: candidate scores / rows / tokens, next tokens, next parent rows,
    ok flag) and the timestamp-rule state of its rows -- beam_search_dev's per-window state."""

    def __init__(self, index, slot, prefix, beams, k, eos, max_length, rules, begin_index, decoder_prompt_len,
                 length_penalty, dev, vocab):
        from .generate import BeamProcess
        self.index, self.slot, self.r0, self.beams, self.k = index, slot, slot * beams, beams, k
        self.eos, self.max_length, self.rules, self.begin = eos, max_length, rules, begin_index
        self.bp = BeamProcess(prefix, beams, eos, max_length, length_penalty, decoder_prompt_len)
        n_max = max(1, max_length - len(prefix))
        self.lp = torch.empty((beams, k), dtype=torch.float32, device=dev)
        self.idx = torch.empty((beams, k), dtype=torch.int32, device=dev)
        self.scores = torch.tensor([0.0] + [-1e9] * (beams - 1), dtype=torch.float64, device=dev)
        self.f = (0, 8 * k, 12 * k, 16 * k, 16 * k + 4 * beams, 16 * k + 8 * beams)
        row_bytes = (self.f[5] + 4 + 7) // 8 * 8
        self.log = torch.zeros((n_max, row_bytes), dtype=torch.uint8, device=dev)
        self.views = self.fields(self.log)   # (scores, rows, tokens, next tokens, next rows, ok) column views
        self.tb = rules.timestamp_begin if rules is not None else 1 << 30
        sampled = list(prefix[begin_index:]) if begin_index < len(prefix) else []
        tsl = [t for t in sampled if t >= self.tb]
        ts0 = [len(sampled), sampled[-1] if sampled else -1, sampled[-2] if len(sampled) > 1 else -1,
               tsl[-1] if tsl else -1]
        self.ts_state = torch.tensor([ts0] * beams, dtype=torch.int32, device=dev)
        self.st = torch.tensor([list(rules.state(sampled)) if rules is not None else [0, 1, 0, 1]] * beams,
                               dtype=torch.int32, device=dev)
        self.tsb = torch.empty((beams, vocab), dtype=torch.float32, device=dev) if rules is not None else None
        self.pos = len(prefix)
        self.s = 0
        self.replayed = 0
        self.stopped = False   # reached max_length: no further steps

    def fields(self, buf):
        f = self.f
        return (buf[:, f[0]:f[1]].view(torch.float64), buf[:, f[1]:f[2]].view(torch.int32),
                buf[:, f[2]:f[3]].view(torch.int32), buf[:, f[3]:f[4]].view(torch.int32),
                buf[:, f[4]:f[5]].view(torch.int32), buf[:, f[5]:f[5] + 4].view(torch.int32)[:, 0])

    def score(self, eng: "DecoderEngine", bias_at, stream):
        """this window's scores -> next beams (its log row self.s), as beam_search_dev's loop body"""
        lib, nb, k = eng.lib, self.beams, self.k
        b = bias_at(self.pos)
        lg = eng._logits[self.r0]
        ts_on = self.rules is not None and self.pos >= self.begin
        if ts_on:
            r = self.rules
            _lib.check(lib.cbw_timestamp_rules(lg.data_ptr(), nb, eng.vocab, eng.vpad, _lib.ptr(b), self.st.data_ptr(),
                                               r.timestamp_begin, r.no_timestamps, r.eos, r.max_initial,
                                               self.tsb.data_ptr(), stream), "cbw_timestamp_rules")
            bias, bias_ld = self.tsb, eng.vocab
        else:
            bias, bias_ld = b, 0
        _lib.check(lib.cbw_logprob_topk(lg.data_ptr(), nb, eng.vocab, eng.vpad, _lib.ptr(bias), bias_ld, k,
                                        self.lp.data_ptr(), self.idx.data_ptr(), stream), "cbw_logprob_topk")
        c_score, c_row, c_tok, nxt_tok, nxt_row, ok = self.views
        s = self.s
        _lib.check(lib.cbw_beam_select(self.lp.data_ptr(), self.idx.data_ptr(), nb, k, self.eos, self.scores.data_ptr(),
                                       c_score[s].data_ptr(), c_row[s].data_ptr(), c_tok[s].data_ptr(),
                                       nxt_tok[s].data_ptr(), nxt_row[s].data_ptr(), ok[s].data_ptr(),
                                       self.ts_state.data_ptr(), self.st.data_ptr(), self.tb, int(ts_on), stream),
                   "cbw_beam_select")
        self.s += 1
        if self.pos + 1 >= self.max_length:
            self.stopped = True

    def replay(self):
        if self.s <= self.replayed:
            return
        cs, cr, ct, nt, nr, okh = (t.numpy() for t in self.fields(self.log[self.replayed:self.s].cpu()))
        for i in range(self.s - self.replayed):
            toks, par = self.bp.process([(float(cs[i, j]), int(cr[i, j]), int(ct[i, j])) for j in range(self.k)])
            if not self.bp.finished and (not okh[i] or toks != nt[i].tolist() or par != nr[i].tolist()):
                raise RuntimeError("GPU beam bookkeeping diverged from the host replay")
            if self.bp.finished:
                break
        self.replayed = self.s
