"""Beam-search generation for PBAWhisper, restated from the HF transformers==4.37.2
semantics the reference runs (pinned in requirements.txt:21; `PBAWhisper.generate`
short-form path src/model/pba_whisper.py:283-338 calls
``GenerationMixin.generate(num_beams=5, do_sample=False)``):

* the decoder prefix (``<|startofprev|>`` + keyword prompt, then
  ``<|startoftranscript|> <|lang|> <|task|> <|notimestamps|>``) is forced token by
  token (ForceTokensLogitsProcessor: score 0, beams stay [0, -1e9, ...]);
* per free step: ``log_softmax(logits)`` -> SuppressTokens / SuppressTokensAtBegin
  (additive -inf) -> ``+ beam_scores`` -> top ``2*num_beams`` over
  ``num_beams*V``;
* BeamSearchScorer.process: EOS candidates ranked < num_beams become hypotheses
  scored ``sum_logprobs / generated_len ** length_penalty`` with
  ``generated_len = cur_len - decoder_prompt_len`` (4.37: decoder_prompt_len = 1,
  the start token; the forced prefix counts as generated); the other candidates fill
  the next beams in order; BeamHypotheses.is_done with early_stopping=False;
* finalize at max_length: open beams are added as hypotheses; the best hypothesis
  (stable sort, last of equal scores) is returned;
* ``forced`` (position -> token): forced positions AFTER a free one -- 4.37.2's
  ``forced_decoder_ids`` with ``(1, None)`` when ``language`` is None (_set_forced_decoder_ids:
  the language position is left to the search, the task / notimestamps tokens after it are
  still forced).  ForceTokensLogitsProcessor makes every row's step log-probs -inf except the
  forced token's 0, so the candidates are each beam with the forced token at its running score
  (the beams re-sorted by score, HF's top-k over ``num_beams*V``).

The per-step math (decoder forward, log-softmax, top-k) runs in libcbw; only the
O(num_beams) bookkeeping of the scorer runs on the host, as in the reference.
`step_fn` abstracts the decoder so tests can drive the same search with the oracle.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np


@dataclass
class BeamHyps:
    num_beams: int
    length_penalty: float = 1.0
    beams: List[Tuple[float, List[int]]] = field(default_factory=list)
    worst_score: float = 1e9

    def add(self, hyp: List[int], sum_logprobs: float, generated_len: int):
        score = sum_logprobs / (generated_len ** self.length_penalty)
        if len(self.beams) < self.num_beams or score > self.worst_score:
            self.beams.append((score, list(hyp)))
            if len(self.beams) > self.num_beams:
                sorted_scores = sorted([(s, idx) for idx, (s, _) in enumerate(self.beams)])
                del self.beams[sorted_scores[0][1]]
                self.worst_score = sorted_scores[1][0]
            else:
                self.worst_score = min(score, self.worst_score)

    def is_done(self, best_sum_logprobs: float, cur_len: int, decoder_prompt_len: int) -> bool:
        if len(self.beams) < self.num_beams:
            return False
        highest = best_sum_logprobs / ((cur_len - decoder_prompt_len) ** self.length_penalty)
        return self.worst_score >= highest

    def best(self) -> Tuple[float, List[int]]:
        return sorted(self.beams, key=lambda x: x[0])[-1]


StepFn = Callable[[Sequence[int], int, Optional[Sequence[int]]], Tuple[np.ndarray, np.ndarray]]
"""step_fn(tokens_per_row, pos, reorder_rows_or_None) -> (logprobs [rows, k], token ids [rows, k])
after log_softmax and the additive suppression bias for that position; the decoder
applies `reorder_rows` to its KV cache before consuming `tokens_per_row` at `pos`."""


class BeamProcess:
    """The per-step bookkeeping of HF 4.37.2 beam search (BeamSearchScorer.process + finalize) over the
    sorted top ``2*num_beams`` candidates of a step.  Shared by ``beam_search`` (candidates from the host
    top-k) and the GPU-resident loop (``DecoderEngine.beam_search_dev``: candidates logged by
    cbw_beam_select, replayed here), so both follow the same semantics token for token."""

    def __init__(self, prefix: Sequence[int], num_beams: int, eos: int, max_length: int,
                 length_penalty: float = 1.0, decoder_prompt_len: int = 1):
        self.num_beams, self.eos, self.max_length = num_beams, eos, max_length
        self.decoder_prompt_len = decoder_prompt_len
        self.k = 2 * num_beams
        self.hyps = BeamHyps(num_beams, length_penalty)
        self.seqs = [list(prefix) for _ in range(num_beams)]
        self.beam_scores = np.array([0.0] + [-1e9] * (num_beams - 1))
        self.cur_len = len(prefix)
        self.done = False
        self.finished = False

    def candidates(self, lp: np.ndarray, idx: np.ndarray) -> List[Tuple[float, int, int]]:
        """top-k per row -> the top 2*num_beams over rows (HF topk over num_beams*V)."""
        cand = []
        for r in range(self.num_beams):
            for j in range(self.k):
                cand.append((self.beam_scores[r] + float(lp[r, j]), r, int(idx[r, j])))
        cand.sort(key=lambda c: (-c[0], c[1] * 10**9 + c[2]))
        return cand[:self.k]

    def forced_candidates(self, tok: int) -> List[Tuple[float, int, int]]:
        """A forced position (ForceTokensLogitsProcessor): every row's only finite continuation is ``tok`` at log-prob
        0, so the top candidates are the rows with ``tok`` in score order (ties: lower row first, as ``candidates``)."""
        cand = [(float(self.beam_scores[r]), r, int(tok)) for r in range(self.num_beams)]
        cand.sort(key=lambda c: (-c[0], c[1]))
        return cand

    def process(self, cand: Sequence[Tuple[float, int, int]]) -> Tuple[List[int], List[int]]:
        """One step: EOS candidates ranked < num_beams become hypotheses, the others fill the next beams.
        Returns (next tokens, parent rows); sets ``finished`` when the search ends after this step."""
        next_scores, next_tokens, next_rows = [], [], []
        for rank, (score, r, tok) in enumerate(cand):
            if tok == self.eos:
                if rank >= self.num_beams:
                    continue
                self.hyps.add(self.seqs[r], score, self.cur_len - self.decoder_prompt_len)
            else:
                next_scores.append(score)
                next_tokens.append(tok)
                next_rows.append(r)
            if len(next_scores) == self.num_beams:
                break
        self.done = self.done or self.hyps.is_done(max(c[0] for c in cand), self.cur_len, self.decoder_prompt_len)
        self.seqs = [self.seqs[r] + [t] for r, t in zip(next_rows, next_tokens)]
        self.beam_scores = np.array(next_scores)
        self.cur_len += 1
        self.finished = self.done or self.cur_len >= self.max_length
        return next_tokens, next_rows

    def result(self, num_return_sequences: int = 1):
        """BeamSearchScorer.finalize: open beams join the hypotheses, the best ``num_return_sequences`` come out best
        first, each followed by EOS when shorter than ``max_length`` (a hypothesis is stored without the EOS that
        ended it; finalize writes it back, decoded[i, sent_lengths[i]] = eos, and pads with the pad token = EOS for
        Whisper up to min(longest + 1, max_length)).  One sequence: the list; several: a list of equal-length lists.
        ``score`` / ``scores``: HF's sequences_scores of the returned hypotheses."""
        if not self.done:
            for r in range(self.num_beams):
                self.hyps.add(self.seqs[r], float(self.beam_scores[r]), len(self.seqs[r]) - self.decoder_prompt_len)
            self.done = True
        ranked = sorted(self.hyps.beams, key=lambda x: x[0])   # stable: the last of equal scores is the best
        top = [ranked.pop() for _ in range(min(num_return_sequences, len(ranked)))]
        self.scores = [sc for sc, _ in top]
        self.score = self.scores[0]
        width = min(max(len(h) for _, h in top) + 1, self.max_length)
        rows = [list(h) + [self.eos] * (width - len(h)) for _, h in top]
        return rows[0] if num_return_sequences == 1 else rows


def beam_search(step_fn: StepFn, prefix: Sequence[int], num_beams: int, eos: int, max_length: int,
                length_penalty: float = 1.0, decoder_prompt_len: int = 1, pad: Optional[int] = None,
                return_score: bool = False, forced: Optional[Dict[int, int]] = None, num_return_sequences: int = 1):
    """Returns the full best sequence (prefix included), HF 4.37.2 beam_search semantics; with ``return_score``
    (sequence, its score sum_logprobs / generated_len ** length_penalty = HF's sequences_scores).  ``forced``:
    sequence position -> token for positions after the prefix that ForceTokensLogitsProcessor fixes.
    ``num_return_sequences`` > 1: the best that many (BeamProcess.result), a list of equal-length sequences."""
    forced = forced or {}
    bp = BeamProcess(prefix, num_beams, eos, max_length, length_penalty, decoder_prompt_len)
    # forced prefix: every row consumes prefix[t] at position t; all rows stay identical -- in one
    # prefill pass when the step function offers one (its logits at the intermediate positions are unused)
    pos = 0
    lp = idx = None
    pre = getattr(step_fn, "prefill", None)
    out = pre(list(prefix)) if pre is not None and len(prefix) > 1 else None
    if out is not None:
        lp, idx = out
        pos = len(prefix)
    else:
        for t in range(len(prefix)):
            lp, idx = step_fn([prefix[t]] * num_beams, pos, None)
            pos += 1
    while True:
        cand = bp.forced_candidates(forced[bp.cur_len]) if bp.cur_len in forced else bp.candidates(lp, idx)
        next_tokens, next_rows = bp.process(cand)
        if bp.finished:
            break
        lp, idx = step_fn(next_tokens, pos, next_rows)
        pos += 1
    seq = bp.result(num_return_sequences)
    if return_score:
        return (seq, bp.score if num_return_sequences == 1 else bp.scores)
    return seq


def greedy(step_fn: StepFn, prefix: Sequence[int], eos: int, max_length: int,
           forced: Optional[Dict[int, int]] = None) -> List[int]:
    """Greedy search from ``prefix``; ``forced`` as in ``beam_search``."""
    forced = forced or {}
    seq = list(prefix)
    pos = 0
    lp = idx = None
    pre = getattr(step_fn, "prefill", None)
    out = pre(list(prefix)) if pre is not None and len(prefix) > 1 else None
    if out is not None:
        lp, idx = out
        pos = len(prefix)
    else:
        for t in range(len(prefix)):
            lp, idx = step_fn([prefix[t]], pos, None)
            pos += 1
    while len(seq) < max_length:
        tok = forced.get(len(seq), int(idx[0, 0]))
        seq.append(tok)
        if tok == eos:
            break
        lp, idx = step_fn([tok], pos, None)
        pos += 1
    return seq


def beam_sample(scores_fn, prefix: Sequence[int], num_beams: int, eos: int, max_length: int, temperature: float,
                generator=None, top_k: int = 50, length_penalty: float = 1.0, decoder_prompt_len: int = 1,
                return_score: bool = False, trace: Optional[list] = None, warp_order: str = "4.37"):
    """Beam-sample decoding (``do_sample=True`` with ``num_beams > 1``), HF 4.37.2 ``GenerationMixin._beam_sample``
    as the reference's short-form call reaches it (src/model/pba_whisper.py:318-329 passes do_sample / num_beams /
    temperature through to ``GenerationMixin.generate``; transformers pinned at 4.37.2, requirements.txt:21):

    * per step, per beam row: the processed log-probs ``log_softmax(logits)`` + the processors' masks
      (``scores_fn``: a torch tensor [num_beams, V] on the decoder's device), then -- 4.37.2 order, the default --
      ``+ beam_scores`` FIRST and the warpers on the sum ("logits warpers are intentionally applied after adding
      running beam scores"): TemperatureLogitsWarper (``/ temperature``) and TopKLogitsWarper (all but the row's
      ``top_k`` largest -> -inf; GenerationConfig's default 50).  The warped sums are the candidates' scores, so the
      next beam scores carry the division by the temperature of every step.  ``warp_order="5.x"`` is the later
      transformers order (warpers on the log-probs, then ``+ beam_scores``: transformers 5.15, installed here, which
      generated tests/golden/beam_sample_micro.npz);
    * softmax over all ``num_beams * V`` continuations, ``2 * num_beams`` of them drawn without replacement
      (torch.multinomial's exponential race with ``generator``; a device generator draws on the device), their scores sorted
      descending -> BeamSearchScorer.process (``BeamProcess``: EOS candidates ranked < num_beams by score become
      hypotheses, the others fill the next beams) and finalize, as in beam search.

    ``scores_fn(tokens, pos, reorder_rows)`` consumes one token per row at ``pos`` (after reordering the rows' KV by
    ``reorder_rows``) and returns the next position's processed log-probs; ``scores_fn.prefill(prefix)`` (optional)
    consumes the forced prefix in one pass.  Returns the best sequence (prefix included), with ``return_score`` also
    its score sum_logprobs / generated_len ** length_penalty.  ``trace`` (a list) collects per step the rows'
    sequences and beam scores, the warped scores + beam scores (``acc``, [num_beams, V]), log q of the race and the
    draws in draw order as (score, row, token) tuples."""
    import torch
    if not temperature or temperature <= 0:
        raise ValueError("beam_sample needs a temperature > 0 (temperature 0 is beam search)")
    if warp_order not in ("4.37", "5.x"):
        raise ValueError(f"warp_order {warp_order!r}: '4.37' or '5.x'")
    bp = BeamProcess(prefix, num_beams, eos, max_length, length_penalty, decoder_prompt_len)
    pos = 0
    scores = None
    pre = getattr(scores_fn, "prefill", None)
    if pre is not None and len(prefix) > 1:
        scores = pre(list(prefix))
        pos = len(prefix)
    if scores is None:
        pos = 0
        for t in range(len(prefix)):
            scores = scores_fn([prefix[t]] * num_beams, pos, None)
            pos += 1
    while True:
        V = scores.shape[-1]
        bs = torch.as_tensor(bp.beam_scores, dtype=torch.float32, device=scores.device)[:, None]
        w = (scores.float() + bs if warp_order == "4.37" else scores.float()) / temperature
        if top_k and top_k < V:
            kth = torch.topk(w, top_k, dim=-1).values[:, -1:]
            w = w.masked_fill(w < kth, float("-inf"))
        acc = (w if warp_order == "4.37" else w + bs).reshape(1, -1)
        probs = torch.softmax(acc, dim=-1)
        # torch.multinomial(probs, n, replacement=False) as an explicit exponential race (its CPU algorithm, the draws
        # bit for bit: keys p / q with q ~ Exp(1), the n largest keys), drawn on the generator's device
        gdev = generator.device if generator is not None else probs.device
        q = torch.empty(probs.shape, dtype=probs.dtype, device=gdev).exponential_(1.0, generator=generator)
        draws = torch.topk(probs.to(gdev) / q, 2 * num_beams, dim=-1).indices.to(acc.device)
        sc = acc.gather(1, draws)
        if trace is not None:
            trace.append({"seqs": [list(x) for x in bp.seqs], "beam_scores": bp.beam_scores.copy(),
                          "acc": acc.reshape(num_beams, V).cpu(), "log_q": torch.log(q).reshape(num_beams, V).cpu(),
                          "draws": [(float(a), int(b) // V, int(b) % V) for a, b in zip(sc[0].tolist(), draws[0].tolist())]})
        sc, order = torch.sort(sc, dim=1, descending=True)
        draws = draws.gather(1, order)
        cand = [(float(a), int(d) // V, int(d) % V) for a, d in zip(sc[0].tolist(), draws[0].tolist())]
        next_tokens, next_rows = bp.process(cand)
        if bp.finished:
            break
        scores = scores_fn(next_tokens, pos, next_rows)
        pos += 1
    seq = bp.result()
    return (seq, bp.score) if return_score else seq
