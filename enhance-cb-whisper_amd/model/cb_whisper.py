"""model.cb_whisper.CBWhisper — MI355X counterpart of src/model/cb_whisper.py:20-187.

Two spotters, both on the GPU:
  * the reference's own (``cnn=model.model.KWSModel``, ``keyword_hs`` = the DatabaseLite
    hidden states, 12 layers ``[10:22]`` per keyword): per 30 s window the encoder's
    hidden_states[10:22] (cb_whisper.py:100-106) against every keyword — similarity matrices,
    bilinear resize to ``kws_features_size`` (:189-210) and the 12-channel ResNet-50
    (model/model.py:78-93) in one libcbw call (KwsEngine.score_resized);
  * the efficient_kws LEF classifier (``kws`` + the pre-projected database) — SURVEY.md §0.6:
    the adapter that lets cb-whisper.py run the faster classifier.
Keywords with argmax(logits) == 1 (cb_whisper.py:128) become the ``<|startofprev|>`` prompt
``prepend + sep.join(keywords) + append`` (:140-147).

Differences to the reference, by design: keywords are deduplicated in database
order (the reference's ``set`` gives a non-deterministic order, :132); the
``[[]] * num_segments`` aliasing bug (:89, :129) is not reproduced; no HF
tokenizer files exist offline, so text <-> ids goes through caller-supplied
``tokenize``/``detokenize`` callables (HF ``WhisperTokenizer`` methods fit).
"""
from __future__ import annotations

import random
import re
from typing import Callable, Dict, List, Optional, Sequence

import torch

from cbw.kws import KwsEngine, spot
from cbw.metrics import evaluate_with_conf_int
from cbw.whisper import EncoderEngine, default_layer_ids
from scorer import entity_recall


class CBWhisper:
    def __init__(self, whisper, kws: Optional[KwsEngine], kws_encoder: EncoderEngine, keywords: Sequence[str],
                 keyword_feats: Optional[torch.Tensor], keyword_mask: Optional[torch.Tensor],
                 tokenize: Callable[[str], List[int]],
                 detokenize: Optional[Callable[[List[int]], str]] = None, language: str = "english",
                 prompt: bool = True, oracle: str = "kws", keyword_prompt_prepend: str = "(",
                 keyword_prompt_append: str = ")", keyword_separator: str = " ", keywords_per_group: int = 100,
                 layer_ids: Optional[Sequence[int]] = None, num_beams: int = 5, cnn=None,
                 keyword_hs: Optional[Sequence[torch.Tensor]] = None, kws_features_size=(150, 750)):
        """LEF spotter: ``kws`` + keyword_feats/keyword_mask, the projected keyword database
        (KwsEngine.project of the keyword hs) — bf16 [K, L, Tk', E], f32 [K, L, Tk'].
        Reference spotter: ``cnn`` (model.model.KWSModel) + ``keyword_hs`` (list of [12, Tk_k, D],
        L2-normalised: DatabaseLite.group(..)['hidden_states'], cb_whisper.py:108)."""
        assert oracle in ("gold", "kws", "random"), f"the provided oracle type is not supported, got {oracle}"
        if (cnn is None) == (kws is None):
            raise ValueError("give exactly one spotter: kws (LEF) or cnn (model.model.KWSModel)")
        self.cnn, self.keyword_hs, self.kws_features_size = cnn, keyword_hs, tuple(kws_features_size)
        self.whisper, self.kws, self.kws_encoder = whisper, kws, kws_encoder
        self.keywords = list(keywords)
        self.keyword_feats, self.keyword_mask = keyword_feats, keyword_mask
        self.tokenize, self.detokenize = tokenize, detokenize
        self.language, self.prompt, self.oracle = language, prompt, oracle
        self.prepend, self.append, self.sep = keyword_prompt_prepend, keyword_prompt_append, keyword_separator
        self.keywords_per_group = keywords_per_group
        n_sel = 12 if cnn is not None else kws.n_layers
        self.layer_ids = list(layer_ids) if layer_ids is not None else default_layer_ids(kws_encoder.n_layers, n_sel)
        self.num_beams = num_beams
        self.oracle_buffer: List[str] = []
        self.last_spotted: List[List[str]] = []

    def get_prompt_ids(self, text: str) -> List[int]:
        """WhisperProcessor.get_prompt_ids: [<|startofprev|>] + tokens(" " + text.strip())."""
        return [self.whisper.tokens.startofprev] + list(self.tokenize(" " + text.strip()))

    def spot_keywords(self, input_features: torch.Tensor) -> List[List[str]]:
        """cb_whisper.py:93-132 on the LEF classifier: [S, n_mel, 3000] -> keywords per segment."""
        S = input_features.size(0)
        dev = self.kws_encoder.device
        pk = torch.zeros((S, 3000, self.kws_encoder.cpad), dtype=torch.bfloat16, device=dev)
        pk[:, :, : input_features.shape[1]] = input_features.to(dev).transpose(1, 2).to(torch.bfloat16)
        hs = self.kws_encoder.hidden_states(pk, self.layer_ids, normalize=True)     # [S, L, 1500, D]
        if self.cnn is not None:   # cb_whisper.py:108-128 with the reference's 12-channel CNN
            return [[self.keywords[i] for i in self.cnn.spot_keywords(hs[s], self.keyword_hs, self.kws_features_size)]
                    for s in range(S)]
        out = []
        for s in range(S):
            u, um = self.kws.project(hs[s:s + 1], torch.ones((1, hs.shape[1], hs.shape[2]), device=self.kws.device))
            logits = self.kws.score(u[0], um[0], self.keyword_feats, self.keyword_mask)
            _, idx = spot(logits, None, 0.5, mode="argmax")
            out.append([self.keywords[i] for i in sorted(set(idx.tolist()))])
        return out

    def keyword_spotting(self, input_features: torch.Tensor, start_of_prev: bool = False) -> List[List[int]]:
        """cb_whisper.py:82-149 — the PBAWhisper.generate callback."""
        S = input_features.size(0)
        if not self.prompt:
            return [[] for _ in range(S)]
        if self.oracle == "kws":
            keywords = self.spot_keywords(input_features) if len(self.keywords) else [[] for _ in range(S)]
        else:
            keywords = [list(self.oracle_buffer) for _ in range(S)]
        self.last_spotted = keywords
        ids = []
        for kwds in keywords:
            if not kwds:
                ids.append([])
                continue
            p = self.get_prompt_ids(self.prepend + self.sep.join(kwds) + self.append)
            ids.append(p if start_of_prev else p[1:])
        return ids

    def forward(self, input_features: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                oracle: Sequence[str] = ()):
        """cb_whisper.py:151-187 (always short-form there: is_shortform tests dim 0)."""
        self.oracle_buffer = list(oracle)
        pred = self.whisper.generate(input_features=input_features, attention_mask=attention_mask, task="transcribe",
                                     language=self.language, return_timestamps=False,
                                     condition_on_prev_tokens=False, return_segments=False,
                                     num_beams=self.num_beams, do_sample=False, temperature=0,
                                     keyword_spotting=self.keyword_spotting)
        toks = pred[0].tolist()
        if self.detokenize is None:
            return toks
        special = set(range(self.whisper.tokens.eot, self.whisper.decoder.vocab))
        return self.detokenize([t for t in toks if t not in special]).strip()

    __call__ = forward

    # ------------------------------------------------------------------ evaluation (cb_whisper.py:212-289)
    def on_test_epoch_start(self):
        self.test_step_outputs = []

    def test_step(self, batch: dict, batch_idx: int = 0, rng: Optional[random.Random] = None):
        """cb_whisper.py:218-242: the oracle keyword list (gold = the labelled keywords, random =
        as many non-labelled ones, kws = none: the spotter runs), then forward."""
        labels = batch.get("hotword_labels")
        pos = [] if labels is None else torch.argwhere(torch.cat(list(labels), 0)).view(-1).tolist()
        if self.oracle == "gold":
            oracle = [self.keywords[i] for i in pos]
        elif self.oracle == "random":
            pool = sorted(set(range(len(self.keywords))) - set(pos))
            oracle = [self.keywords[i] for i in (rng or random).sample(pool, len(pos))]
        else:
            oracle = []
        preds = self.forward(input_features=batch["utterance"]["features"],
                             attention_mask=batch["utterance"].get("attention_mask"), oracle=oracle)
        out = {"preds": preds, "target": batch["transcript"], "speaker": batch.get("speaker")}
        if batch.get("keywords") is not None:
            out["keywords"] = batch["keywords"]
        if not hasattr(self, "test_step_outputs"):
            self.test_step_outputs = []
        self.test_step_outputs.append(out)
        return out

    def on_test_epoch_end(self, num_bootstraps: int = 1000, alpha: float = 5) -> Dict[str, float]:
        """cb_whisper.py:244-289: entity recall (scorer.entity_recall, ner_tags='ALL',
        char_split=True) with a speaker-conditioned bootstrap CI.  Mentions come from the batch's
        'keywords' records, else from every database keyword's regex matches in the reference
        transcript (:256-261)."""
        outs = self.test_step_outputs
        preds = [o["preds"] for o in outs]
        refs = [o["target"] for o in outs]
        if outs and outs[0].get("keywords") is not None:
            mentions = [[{**kw, "ner_tag": "UNK"} for kw in o["keywords"]] for o in outs]
        else:
            mentions = [[{"mention": kw, "total_offset": m.start(), "end_offset": m.end(), "ner_tag": "UNK"}
                         for kw in self.keywords for m in re.finditer(kw, ref)] for ref in refs]

        def f_entity_recall(lab, smp, smp2=None):
            refs_, kws_ = zip(*lab) if len(lab) else ((), ())
            return entity_recall(preds=list(smp), refs=list(refs_), mentions=list(kws_), ner_tags="ALL",
                                 char_split=True)["ALL"]

        speakers = [o["speaker"] for o in outs]
        conditions = None
        if speakers and speakers[0] is not None:
            sid = {s: i for i, s in enumerate(dict.fromkeys(speakers))}
            conditions = [sid[s] for s in speakers]
        c, (lo, hi) = evaluate_with_conf_int(preds, f_entity_recall, list(zip(refs, mentions)), conditions,
                                             num_bootstraps=num_bootstraps, alpha=alpha)
        self.test_step_outputs = []
        return {"Entity Recall": c, "Entity Recall LB": lo, "Entity Recall UB": hi}
