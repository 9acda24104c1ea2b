"""model.cb_whisper.CBWhisper — MI355X counterpart of src/model/cb_whisper.py:20-187.

The reference's spotter is the original 12-channel CNN on bilinearly resized
similarity maps (cb_whisper.py:189-210, model/model.py:78-93); SURVEY.md §0.6
notes that running the efficient_kws LEF classifier inside cb-whisper.py needs an
adapter — this class is that adapter: per 30 s window the KWS encoder's
hidden_states (cb_whisper.py:100-106) are projected (LEF), scored against the
pre-projected keyword database by the ResNet classifier, and keywords with
argmax(logits) == 1 (cb_whisper.py:128) become the ``<|startofprev|>`` prompt
``prepend + sep.join(keywords) + append`` (:140-147).

Differences to the reference, by design: keywords are deduplicated in database
order (the reference's ``set`` gives a non-deterministic order, :132); the
``[[]] * num_segments`` aliasing bug (:89, :129) is not reproduced; no HF
tokenizer files exist offline, so text <-> ids goes through caller-supplied
``tokenize``/``detokenize`` callables (HF ``WhisperTokenizer`` methods fit).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch

from cbw.kws import KwsEngine, spot
from cbw.whisper import EncoderEngine, default_layer_ids


class CBWhisper:
    def __init__(self, whisper, kws: KwsEngine, kws_encoder: EncoderEngine, keywords: Sequence[str],
                 keyword_feats: torch.Tensor, keyword_mask: torch.Tensor, tokenize: Callable[[str], List[int]],
                 detokenize: Optional[Callable[[List[int]], str]] = None, language: str = "english",
                 prompt: bool = True, oracle: str = "kws", keyword_prompt_prepend: str = "(",
                 keyword_prompt_append: str = ")", keyword_separator: str = " ", keywords_per_group: int = 100,
                 layer_ids: Optional[Sequence[int]] = None, num_beams: int = 5):
        """keyword_feats/keyword_mask: the projected keyword database (KwsEngine.project of the
        keyword hs, cb_whisper.py:63-69 DatabaseLite) — bf16 [K, L, Tk', E], f32 [K, L, Tk']."""
        assert oracle in ("gold", "kws", "random"), f"the provided oracle type is not supported, got {oracle}"
        self.whisper, self.kws, self.kws_encoder = whisper, kws, kws_encoder
        self.keywords = list(keywords)
        self.keyword_feats, self.keyword_mask = keyword_feats, keyword_mask
        self.tokenize, self.detokenize = tokenize, detokenize
        self.language, self.prompt, self.oracle = language, prompt, oracle
        self.prepend, self.append, self.sep = keyword_prompt_prepend, keyword_prompt_append, keyword_separator
        self.keywords_per_group = keywords_per_group
        self.layer_ids = list(layer_ids) if layer_ids is not None else default_layer_ids(kws_encoder.n_layers,
                                                                                         kws.n_layers)
        self.num_beams = num_beams
        self.oracle_buffer: List[str] = []
        self.last_spotted: List[List[str]] = []

    def get_prompt_ids(self, text: str) -> List[int]:
        """WhisperProcessor.get_prompt_ids: [<|startofprev|>] + tokens(" " + text.strip())."""
        return [self.whisper.tokens.startofprev] + list(self.tokenize(" " + text.strip()))

    def spot_keywords(self, input_features: torch.Tensor) -> List[List[str]]:
        """cb_whisper.py:93-132 on the LEF classifier: [S, n_mel, 3000] -> keywords per segment."""
        S = input_features.size(0)
        pk = torch.zeros((S, 3000, self.kws_encoder.cpad), dtype=torch.bfloat16, device=self.kws.device)
        pk[:, :, : input_features.shape[1]] = input_features.to(self.kws.device).transpose(1, 2).to(torch.bfloat16)
        hs = self.kws_encoder.hidden_states(pk, self.layer_ids, normalize=True)     # [S, L, 1500, D]
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
