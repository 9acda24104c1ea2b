"""Several long-form windows decoded in lock step on one decoder state (rows = windows x beams <= 16).

The reference decodes one audio per ``generate`` call (src/model/pba_whisper.py:343-475): per 30 s window one HF
4.37.2 beam search, each step one pass over the decoder weights for ``num_beams`` rows.  On the GPU that step is a
chain of latency-bound launches that streams ~1.9 GB of weights (large-v3) for 5 rows; the rows of further windows
ride along almost free.  ``WindowBatcher`` runs the beam searches of several audios' current windows as one
search over their concatenated rows: per iteration each window's scoring (timestamp rules, log-softmax + top-k,
cbw_beam_select on its rows), one KV reorder over all rows, one cbw_decoder_step_rows with every row at its own
position.  Each window's bookkeeping is the same as DecoderEngine.beam_search_dev's (the logged candidates replayed
through the host BeamProcess every ``check_every`` steps), and each row's logits equal those of a step over its
window alone, so every window decodes to the tokens its own beam search gives.

Callers are the long-form lanes (one thread per audio in flight): ``beam_search`` blocks the calling thread until
its window is done, while one batcher thread owns the GPU decode state and admits windows into free slots.
"""
from __future__ import annotations

import atexit
import queue
import threading
import weakref
from typing import List, Optional, Sequence

import torch

from . import _lib
from .decoder import DecoderEngine
from .generate import BeamProcess


class _Window:
    """One window's beam search in a slot: its BeamProcess, device log rows and timestamp state."""

    def __init__(self, req, slot, beams, k, dev, vocab):
        self.req, self.slot, self.r0 = req, slot, slot * beams
        prefix, eos, max_length = req["prefix"], req["eos"], req["max_length"]
        rules, begin = req["rules"], req["begin_index"]
        self.bp = BeamProcess(prefix, beams, eos, max_length, req["length_penalty"], req["decoder_prompt_len"])
        n_max = max(1, max_length - len(prefix))
        self.lp = torch.empty((beams, k), dtype=torch.float32, device=dev)
        self.idx = torch.empty((beams, k), dtype=torch.int32, device=dev)
        self.scores = torch.tensor([0.0] + [-1e9] * (beams - 1), dtype=torch.float64, device=dev)
        self.f = (0, 8 * k, 12 * k, 16 * k, 16 * k + 4 * beams, 16 * k + 8 * beams)
        row_bytes = (self.f[5] + 4 + 7) // 8 * 8
        self.log = torch.zeros((n_max, row_bytes), dtype=torch.uint8, device=dev)
        self.views = self.fields(self.log)   # (scores, rows, tokens, next tokens, next rows, ok) column views, made once
        self.tb = rules.timestamp_begin if rules is not None else 1 << 30
        sampled = list(prefix[begin:]) if begin < len(prefix) else []
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

    def replay(self, upto=None):
        upto = self.s if upto is None else upto
        if upto <= self.replayed:
            return
        cs, cr, ct, nt, nr, okh = (t.numpy() for t in self.fields(self.log[self.replayed:upto].cpu()))
        k = cs.shape[1]
        for i in range(upto - self.replayed):
            toks, par = self.bp.process([(float(cs[i, j]), int(cr[i, j]), int(ct[i, j])) for j in range(k)])
            if not self.bp.finished and (not okh[i] or toks != nt[i].tolist() or par != nr[i].tolist()):
                raise RuntimeError("GPU beam bookkeeping diverged from the host replay")
            if self.bp.finished:
                break
        self.replayed = upto


_STOP = object()   # queue sentinel: the batcher thread ends once no window is in flight


def _close_at_exit(ref):
    b = ref()
    if b is not None:
        b.close()


class WindowBatcher:
    """A decoder state of ``slots`` windows x ``beams`` rows shared by the threads that call ``beam_search``.
    ``close()`` (also run at interpreter exit) ends the batcher thread: no thread of it is left inside the runtime
    while the process tears the HIP runtime down."""

    def __init__(self, config, state_dict, slots: int, beams: int, device=None, max_len: int = 448,
                 check_every: int = 8, priority: int = -1):
        if slots * beams > 16:
            raise ValueError("slots x beams must be <= 16 rows")
        self.eng = DecoderEngine(config, state_dict, device, max_len=max_len)
        self.dev = self.eng.device
        self.slots, self.beams, self.k = slots, beams, min(16, 2 * beams)
        self.check_every = check_every
        self.stream = torch.cuda.Stream(device=self.dev, priority=priority)
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            self.eng.start_windows(slots, beams)
            self._inc = torch.zeros((slots * beams,), dtype=torch.int32, device=self.dev)
            self._tok = torch.zeros((slots * beams,), dtype=torch.int32, device=self.dev)
            self._ident = torch.arange(slots * beams, dtype=torch.int32, device=self.dev)
            self._rows = self._ident.clone()
        self.q: "queue.Queue" = queue.Queue()
        self.active: List[Optional[_Window]] = [None] * slots
        self.stats = {"iterations": 0, "row_steps": 0, "live_row_steps": 0}
        self._thread = None
        self._lock = threading.Lock()
        self._error = None
        self._closed = False
        atexit.register(_close_at_exit, weakref.ref(self))

    def close(self):
        """End the batcher thread (after every caller's window has returned); later beam_search calls raise."""
        with self._lock:
            th, self._thread, self._closed = self._thread, None, True
        if th is not None and th.is_alive():
            self.q.put(_STOP)
            th.join()

    # ---------------------------------------------------------------- caller side
    def beam_search(self, enc_out: torch.Tensor, prefix: Sequence[int], eos: int, max_length: int, bias_at,
                    rules=None, begin_index: int = 0, decoder_prompt_len: int = 1, length_penalty: float = 1.0,
                    return_score: bool = False):
        """DecoderEngine.beam_search_dev's contract for one window (num_beams = self.beams), decoded beside the
        other threads' windows.  enc_out: the window's post-LN encoder output, produced on the caller's stream."""
        if len(prefix) < 2:
            raise ValueError("the batched search needs a prefix of >= 2 tokens")
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        req = {"enc": enc_out, "event": ev, "prefix": list(prefix), "eos": eos, "max_length": max_length,
               "bias_at": bias_at, "rules": rules, "begin_index": begin_index,
               "decoder_prompt_len": decoder_prompt_len, "length_penalty": length_penalty,
               "done": threading.Event(), "result": None, "error": None}
        with self._lock:
            if self._error is not None:
                raise RuntimeError("window batcher failed") from self._error
            if self._closed:
                raise RuntimeError("window batcher closed")
            if self._thread is None:
                self._thread = threading.Thread(target=self._loop, daemon=True)
                self._thread.start()
        self.q.put(req)
        req["done"].wait()
        if req["error"] is not None:
            raise req["error"]
        seq, score = req["result"]
        return (seq, score) if return_score else seq

    # ---------------------------------------------------------------- batcher thread
    def _admit(self, req, slot):
        eng, nb = self.eng, self.beams
        torch.cuda.current_stream(self.dev).wait_event(req["event"])
        req["enc"].record_stream(torch.cuda.current_stream(self.dev))
        eng.set_window(slot, req["enc"])
        eng.prefill_window(slot, nb, req["prefix"])
        w = _Window(req, slot, nb, self.k, self.dev, eng.vocab)
        self._inc[w.r0:w.r0 + nb].fill_(1)
        self.active[slot] = w

    def _retire(self, w: _Window, error=None):
        self._inc[w.r0:w.r0 + self.beams].fill_(0)
        self._rows[w.r0:w.r0 + self.beams].copy_(self._ident[w.r0:w.r0 + self.beams])
        self.active[w.slot] = None
        req = w.req
        if error is None and not w.bp.finished:
            error = RuntimeError("GPU beam search ended before the host replay finished")
        if error is None:
            req["result"] = (w.bp.result(), w.bp.score)
        req["error"] = error
        req["done"].set()

    def _score(self, w: _Window, stream):
        """window w's scores -> next beams (its log row w.s), as beam_search_dev's loop body."""
        eng, lib, nb, k = self.eng, self.eng.lib, self.beams, self.k
        req = w.req
        b = req["bias_at"](w.pos)
        lg = eng._logits[w.r0]
        rules = req["rules"]
        if rules is not None and w.pos >= req["begin_index"]:
            _lib.check(lib.cbw_timestamp_rules(lg.data_ptr(), nb, eng.vocab, eng.vpad, _lib.ptr(b), w.st.data_ptr(),
                                               rules.timestamp_begin, rules.no_timestamps, rules.eos,
                                               rules.max_initial, w.tsb.data_ptr(), stream), "cbw_timestamp_rules")
            bias, bias_ld = w.tsb, eng.vocab
        else:
            bias, bias_ld = b, 0
        _lib.check(lib.cbw_logprob_topk(lg.data_ptr(), nb, eng.vocab, eng.vpad, _lib.ptr(bias), bias_ld, k,
                                        w.lp.data_ptr(), w.idx.data_ptr(), stream), "cbw_logprob_topk")
        c_score, c_row, c_tok, nxt_tok, nxt_row, ok = w.views
        s = w.s
        _lib.check(lib.cbw_beam_select(w.lp.data_ptr(), w.idx.data_ptr(), nb, k, req["eos"], w.scores.data_ptr(),
                                       c_score[s].data_ptr(), c_row[s].data_ptr(), c_tok[s].data_ptr(),
                                       nxt_tok[s].data_ptr(), nxt_row[s].data_ptr(), ok[s].data_ptr(),
                                       w.ts_state.data_ptr(), w.st.data_ptr(), w.tb,
                                       int(rules is not None and w.pos >= req["begin_index"]), stream),
                   "cbw_beam_select")
        w.s += 1
        if w.pos + 1 >= req["max_length"]:
            w.stopped = True
            return
        # the step's tokens and (global) parent rows for this window's rows
        self._tok[w.r0:w.r0 + nb].copy_(nxt_tok[s])
        torch.add(nxt_row[s], w.r0, out=self._rows[w.r0:w.r0 + nb])

    def _loop(self):
        try:
            with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
                self._run()
        except BaseException as e:   # every waiting caller sees the failure
            with self._lock:
                self._error = e
            for w in self.active:
                if w is not None:
                    w.req["error"] = e
                    w.req["done"].set()
            while True:
                try:
                    req = self.q.get_nowait()
                except queue.Empty:
                    break
                if req is _STOP:
                    continue
                req["error"] = e
                req["done"].set()

    def _run(self):
        eng, lib = self.eng, self.eng.lib
        stream = _lib.stream_handle()
        it = 0
        while True:
            # admit waiting windows into free slots (block when nothing is in flight)
            for slot in range(self.slots):
                if self.active[slot] is None:
                    try:
                        req = self.q.get(block=all(a is None for a in self.active), timeout=None)
                    except queue.Empty:
                        break
                    if req is _STOP:
                        if all(a is None for a in self.active):
                            return
                        self.q.put(req)   # windows still in flight: finish them first
                        break
                    self._admit(req, slot)
            live = [w for w in self.active if w is not None]
            for w in live:
                self._score(w, stream)
            for w in live:   # windows at max_length: replayed now, no further steps
                if w.stopped:
                    w.replay()
                    self._retire(w)
            live = [w for w in self.active if w is not None]
            if not live:
                continue
            rows, windows = eng._shape
            length = max(w.pos for w in live)
            _lib.check(lib.cbw_decoder_reorder(eng.h, self._rows.data_ptr(), rows, windows, length,
                                               eng._state.data_ptr(), eng._state.numel(), stream),
                       "cbw_decoder_reorder")
            eng.step_rows(self._tok)
            eng._posr.add_(self._inc)
            for w in live:
                w.pos += 1
            self.stats["iterations"] += 1
            self.stats["row_steps"] += rows
            self.stats["live_row_steps"] += len(live) * self.beams
            it += 1
            if it % self.check_every == 0:   # one device -> host copy per window, then the finished ones leave
                for w in live:
                    w.replay()
                    if w.bp.finished:
                        self._retire(w)
