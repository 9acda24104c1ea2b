"""model.cb_whisper.CBWhisper — MI355X counterpart of src/model/cb_whisper.py:20-367.

``CBWhisper(dataset, split, root, kw_type, encoder_ckpt, whisper_ckpt, kws_ckpt, language, prompt, oracle,
kws_features_size, keyword_prompt_prepend, keyword_prompt_append, keyword_separator, keywords_per_group)``
is the reference constructor (cb_whisper.py:21-80), so ``cb-whisper.py test --config
configs/cb-whisper-*.yaml`` builds it from the same ``init_args``:

* ``whisper_ckpt`` -> ``PBAWhisper.from_pretrained`` (:57) and its tokenizer (the ``WhisperProcessor`` of
  :46-49: ``get_prompt_ids`` / ``batch_decode``, cbw.tokenizer), from a local HF-format directory;
* ``kws_ckpt`` -> ``model.model.KWSModel.load_from_checkpoint`` (:60, the 12-channel CNN) -- or, when the
  checkpoint's hyper-parameters are an efficient_kws LEF/LE model, ``efficient_kws.model.KWSModel``
  (the adapter of SURVEY.md §0.6);
* ``DatabaseLite(dataset, split, root, kw_type, keywords_per_group)`` (:63-69, :298-367) over the keyword
  hs ``.bin`` files;
* ``encoder_ckpt`` -> the WhisperModel encoder (:72) whose ``hidden_states[10:22]`` feed the spotter.

GPU engines are created on first use, so construction needs no GPU.  ``keyword_spotting`` (:82-149) runs per
30 s window: the encoder's hidden states (L2-normalised), the similarity + resize + 12-channel ResNet-50 of
every keyword (one libcbw call, KwsEngine.score_resized) or the LEF scores, argmax(logits) == 1 (:128), and
the ``<|startofprev|>`` prompt ``prepend + sep.join(keywords) + append`` (:140-147).

Differences to the reference, by design: keywords are deduplicated in database order (the reference's
``set`` gives a non-deterministic order, :132); the ``[[]] * num_segments`` aliasing (:89, :129) is not
reproduced; the keyword hs stay resident on the GPU instead of a host->device copy per window (:111, :365);
an encoder whose mel bins differ from the features raises ValueError (the reference crashes later, SURVEY.md
Appendix A.5).
"""
from __future__ import annotations

import os
import random
import re
from types import SimpleNamespace
from typing import Callable, Dict, List, Optional, Sequence, Union

import torch

from cbw.keyword_db import KeywordDatabase
from cbw.kws import KwsEngine, pack_keywords, spot
from cbw.metrics import evaluate_with_conf_int
from cbw.whisper import EncoderEngine, default_layer_ids
from scorer import entity_recall


class DatabaseLite:
    """cb_whisper.py:298-367 over the dataset layouts of data/dataset.py: ACL 6060 (root/2/acl_6060/{dev,eval},
    text/keywords.txt, :371-407) and Aishell (root/{dev,test}, hotword.txt, :236-251); keyword hs in
    keywords-hs/<kw_type>/<idx>.bin; missing files are zero 'ghost' keywords."""

    def __init__(self, dataset: str, split: str, root: str, kw_type: str, keywords_per_group: int = 100):
        assert dataset in ["aishell", "acl"], f"DatabaseLite: the dataset is not supported, got {dataset}"
        assert split in ["dev", "test"], f"DatabaseLite: the split is not supported, got {split} for {dataset}"
        assert kw_type in ["tts", "natural"], f"DatabaseLite: the keyword type is not supported, got {kw_type} for {dataset}"
        if dataset == "acl":
            folder = os.path.join(root, "2", "acl_6060", split if split == "dev" else "eval")
            kfile = os.path.join("text", "keywords.txt")
        else:
            folder = os.path.join(root, split)
            kfile = "hotword.txt"
        self.db = KeywordDatabase.from_split_folder(folder, kw_type, keywords_per_group, keywords_file=kfile)
        self.keywords_per_group = self.db.keywords_per_group
        self.num_keywords = len(self.db)

    def __len__(self) -> int:
        return self.num_keywords

    def __getitem__(self, idx: int) -> dict:
        return self.db[idx]

    def num_groups(self) -> int:
        return self.db.num_groups()

    def group(self, idx: int, device: str = "cpu", load_hs: bool = True) -> dict:
        return self.db.group(idx, device, load_hs)


def _is_efficient_kws(hp: dict) -> bool:
    return bool(hp.get("learn_features")) and bool(hp.get("proj_mlp"))


def _check_segment_keywords(mode: str) -> str:
    if mode not in ("union", "per_segment"):
        raise ValueError(f"segment_keywords must be 'union' (the reference's) or 'per_segment', got {mode!r}")
    return mode


class CBWhisper:
    def __init__(self, dataset: str, split: str, root: str, kw_type: str, encoder_ckpt: str, whisper_ckpt: str,
                 kws_ckpt: str, language: str, prompt: bool = True, oracle: Union[bool, str] = "kws",
                 kws_features_size=(150, 750), keyword_prompt_prepend: str = "(", keyword_prompt_append: str = ")",
                 keyword_separator: str = " ", keywords_per_group: int = 100, num_beams: int = 5):
        """cb_whisper.py:21-80 (see the module docstring); every *_ckpt is a local directory / file."""
        from cbw.checkpoint import encoder_state, load_state_dict, read_json, whisper_configs
        from model.pba_whisper import PBAWhisper
        if isinstance(oracle, bool):
            oracle = "gold" if oracle else "kws"
        assert oracle in ("gold", "kws", "random"), f"the provided oracle type is not supported, got {oracle}"
        self.hparams = SimpleNamespace(dataset=dataset, split=split, root=root, kw_type=kw_type,
                                       encoder_ckpt=encoder_ckpt, whisper_ckpt=whisper_ckpt, kws_ckpt=kws_ckpt,
                                       language=language, prompt=prompt, oracle=oracle,
                                       kws_features_size=kws_features_size, keyword_prompt_prepend=keyword_prompt_prepend,
                                       keyword_prompt_append=keyword_prompt_append, keyword_separator=keyword_separator,
                                       keywords_per_group=keywords_per_group)
        whisper = PBAWhisper.from_pretrained(whisper_ckpt)
        if whisper.tokenizer is None:
            raise FileNotFoundError(f"no tokenizer files in {whisper_ckpt} (WhisperProcessor.from_pretrained, :46-49)")
        ckpt = torch.load(kws_ckpt, map_location="cpu", weights_only=True)
        hp = dict(ckpt.get("hyper_parameters", {}))
        database = DatabaseLite(dataset, split, root, kw_type, keywords_per_group)
        enc_sd = encoder_state(load_state_dict(encoder_ckpt))
        enc_cfg, _, _ = whisper_configs(read_json(encoder_ckpt, "config.json"))
        self._setup(whisper, None, None, database.db.keywords, tokenize=None, detokenize=None, language=language,
                    prompt=prompt, oracle=oracle, keyword_prompt_prepend=keyword_prompt_prepend,
                    keyword_prompt_append=keyword_prompt_append, keyword_separator=keyword_separator,
                    keywords_per_group=keywords_per_group, num_beams=num_beams, kws_features_size=kws_features_size)
        self.kw_database = database
        self._encoder_parts = (enc_cfg, enc_sd)
        if _is_efficient_kws(hp):
            from efficient_kws.model import KWSModel as EffKWSModel
            self.kws_model = EffKWSModel.load_from_checkpoint(kws_ckpt)
        else:
            from model.model import KWSModel as CNNKWSModel
            self.cnn = CNNKWSModel.load_from_checkpoint(kws_ckpt)

    # ------------------------------------------------------------------ component constructor
    @classmethod
    def from_components(cls, whisper, kws: Optional[KwsEngine], kws_encoder: EncoderEngine, keywords: Sequence[str],
                        keyword_feats: Optional[torch.Tensor], keyword_mask: Optional[torch.Tensor],
                        tokenize: Optional[Callable[[str], List[int]]] = None,
                        detokenize: Optional[Callable[[List[int]], str]] = None, language: str = "english",
                        prompt: bool = True, oracle: str = "kws", keyword_prompt_prepend: str = "(",
                        keyword_prompt_append: str = ")", keyword_separator: str = " ", keywords_per_group: int = 100,
                        layer_ids: Optional[Sequence[int]] = None, num_beams: int = 5, cnn=None,
                        keyword_hs: Optional[Sequence[torch.Tensor]] = None, kws_features_size=(150, 750),
                        keyword_feats32: Optional[torch.Tensor] = None,
                        exact_band: Union[float, str] = "auto", fp8_band: Optional[float] = None,
                        segment_keywords: str = "union") -> "CBWhisper":
        """Already-built engines: the LEF spotter (``kws`` + the projected database keyword_feats /
        keyword_mask, bf16 [K, L, Tk', E] / f32 [K, L, Tk']) or the reference spotter (``cnn`` =
        model.model.KWSModel + ``keyword_hs``, a list of [12, Tk_k, D] L2-normalised keyword hs).
        ``tokenize`` maps text to ids (default: the whisper tokenizer's).  ``keyword_feats32`` (the fp32
        projections, KwsEngine.project_f32) turns on the exact-decision tiers for the LEF spotter: pairs
        within ``exact_band`` of the argmax boundary (p = 0.5) are re-scored (KwsEngine.score_exact); "auto"
        measures the band on the engine's weights at the first spotted window (efficient_kws.model.calibrate_band).
        ``fp8_band`` (the engine's fp8 tier calibrated first, KwsEngine.calibrate_fp8): every pair is scored by the
        e4m3 network and only the pairs within fp8_band of the boundary go on to bf16 and the exact tiers."""
        if (cnn is None) == (kws is None):
            raise ValueError("give exactly one spotter: kws (LEF) or cnn (model.model.KWSModel)")
        self = cls.__new__(cls)
        self.hparams = SimpleNamespace(language=language, prompt=prompt, oracle=oracle,
                                       kws_features_size=kws_features_size, keyword_prompt_prepend=keyword_prompt_prepend,
                                       keyword_prompt_append=keyword_prompt_append, keyword_separator=keyword_separator,
                                       keywords_per_group=keywords_per_group)
        self._setup(whisper, kws, kws_encoder, keywords, tokenize, detokenize, language, prompt, oracle,
                    keyword_prompt_prepend, keyword_prompt_append, keyword_separator, keywords_per_group, num_beams,
                    kws_features_size, layer_ids=layer_ids)
        self.cnn, self.keyword_hs = cnn, keyword_hs
        self.keyword_feats, self.keyword_mask = keyword_feats, keyword_mask
        self.keyword_feats32 = keyword_feats32
        self._set_band(exact_band)
        self.fp8_band = fp8_band
        self.segment_keywords = _check_segment_keywords(segment_keywords)
        return self

    def _set_band(self, exact_band: Union[float, str]):
        """A number is used as given; "auto" starts at EXACT_BAND and is replaced by the band measured on these
        weights at the first spotted window (the 0.03 default was measured on the synthetic weights
        only, so a real checkpoint's bf16 error could exceed it and decisions would silently differ from fp32)."""
        from efficient_kws.model import EXACT_BAND
        if isinstance(exact_band, str) and exact_band != "auto":
            raise ValueError(f"exact_band must be a number or 'auto', got {exact_band!r}")
        self._band_auto = isinstance(exact_band, str)
        self.exact_band = EXACT_BAND if self._band_auto else float(exact_band)
        self.band_calibration: Optional[dict] = None

    def _setup(self, whisper, kws, kws_encoder, keywords, tokenize, detokenize, language, prompt, oracle,
               keyword_prompt_prepend, keyword_prompt_append, keyword_separator, keywords_per_group, num_beams,
               kws_features_size, layer_ids=None):
        assert oracle in ("gold", "kws", "random"), f"the provided oracle type is not supported, got {oracle}"
        self.whisper, self._kws, self._kws_encoder = whisper, kws, kws_encoder
        self.keywords = list(keywords)
        self.tokenize, self.detokenize = tokenize, detokenize
        self.language, self.prompt, self.oracle = language, prompt, oracle
        self.prepend, self.append, self.sep = keyword_prompt_prepend, keyword_prompt_append, keyword_separator
        self.keywords_per_group = keywords_per_group
        self.num_beams = num_beams
        self.kws_features_size = None if kws_features_size is None else tuple(kws_features_size)
        self._layer_ids = list(layer_ids) if layer_ids is not None else None
        self.cnn = self.kws_model = None
        self.keyword_hs = self.keyword_feats = self.keyword_mask = self.keyword_feats32 = None
        self._set_band("auto")
        self.fp8_band = None
        self.kw_database = None
        self._encoder_parts = None
        self._packed = None
        self.oracle_buffer: List[str] = []
        self.last_spotted: List[List[str]] = []
        self.segment_keywords = "union"

    # ------------------------------------------------------------------ lazily built GPU pieces
    @property
    def kws_encoder(self) -> EncoderEngine:
        if self._kws_encoder is None:
            cfg, sd = self._encoder_parts
            self._kws_encoder = EncoderEngine(cfg, sd)
        return self._kws_encoder

    @property
    def kws(self) -> Optional[KwsEngine]:
        if self._kws is None and self.kws_model is not None:
            self._kws = self.kws_model.engine()
        return self._kws

    @property
    def layer_ids(self) -> List[int]:
        if self._layer_ids is None:
            n_sel = 12 if self.cnn is not None else self.kws.n_layers
            self._layer_ids = default_layer_ids(self.kws_encoder.n_layers, n_sel)
        return self._layer_ids

    def _database_on_device(self):
        """Keyword side, once: the CNN's keyword hs (device, 12 layers) or the LEF-projected database."""
        dev = self.kws_encoder.device
        if self.cnn is not None and self.keyword_hs is None:
            self.keyword_hs = [h.to(dev, torch.float32) for h in self.kw_database.db.hidden_states]
        if self.cnn is None and self.keyword_feats is None:
            frames = tuple(getattr(self.kws_model.hparams, "features_size", (150, 1500)))[0]
            pk, pm, _ = self.kw_database.db.projected(self.kws, frames)
            self.keyword_feats, self.keyword_mask = pk, pm
            if self.exact_band > 0 and self.kws.has_fp32:   # no fp32 network for n_layers > 4: bf16 decisions
                self.keyword_feats32 = self.kw_database.db.projected_f32(self.kws, frames)

    # ------------------------------------------------------------------ tokenizer
    def get_prompt_ids(self, text: str) -> List[int]:
        """WhisperProcessor.get_prompt_ids: [<|startofprev|>] + tokens(" " + text.strip())."""
        tok = getattr(self.whisper, "tokenizer", None)
        if self.tokenize is None and tok is not None:
            return tok.get_prompt_ids(text)
        if self.tokenize is None:
            raise ValueError("no tokenizer: give whisper_ckpt tokenizer files or a tokenize callable")
        return [self.whisper.tokens.startofprev] + list(self.tokenize(" " + text.strip()))

    # ------------------------------------------------------------------ spotting (cb_whisper.py:82-149)
    def _groups(self):
        K = len(self.keywords)
        g = self.keywords_per_group if self.keywords_per_group and self.keywords_per_group > 0 else K
        return [(lo, min(lo + g, K)) for lo in range(0, K, g)]

    def spot_keywords(self, input_features: torch.Tensor) -> List[List[str]]:
        """cb_whisper.py:93-132: [S, n_mel, 3000] -> keywords per segment (database order, deduplicated)."""
        S = input_features.size(0)
        enc = self.kws_encoder
        dev = enc.device
        if input_features.shape[1] != enc.n_mel:
            raise ValueError(f"the spotting encoder takes {enc.n_mel} mel bins, the features have "
                             f"{input_features.shape[1]} (SURVEY.md Appendix A.5)")
        self._database_on_device()
        pk = torch.zeros((S, 3000, enc.cpad), dtype=torch.bfloat16, device=dev)
        pk[:, :, : input_features.shape[1]] = input_features.to(dev).transpose(1, 2).to(torch.bfloat16)
        hs = enc.hidden_states(pk, self.layer_ids, normalize=True)     # [S, L, 1500, D]
        out = []
        for s in range(S):
            if self.cnn is not None:
                if self.kws_features_size is not None:
                    if self._packed is None:   # keyword rows packed once, resident on the GPU
                        self._packed = pack_keywords(self.keyword_hs, dev)
                    idx = self.cnn.spot_keywords(hs[s], self._packed, self.kws_features_size)
                else:   # cb_whisper.py:202-204: resize to (longest keyword of the group, utterance frames)
                    idx = []
                    for lo, hi in self._groups():
                        size = (max(int(h.shape[1]) for h in self.keyword_hs[lo:hi]), int(hs.shape[2]))
                        idx += [lo + i for i in self.cnn.spot_keywords(hs[s], self.keyword_hs[lo:hi], size)]
            else:
                ones = torch.ones((1, hs.shape[1], hs.shape[2]), device=dev)
                u, um = self.kws.project(hs[s:s + 1], ones)
                if self.keyword_feats32 is not None and self.exact_band > 0:
                    # argmax(logits) == 1 <=> p > 0.5: the pairs near p = 0.5 re-scored
                    u32 = self.kws.project_f32(hs[s:s + 1], ones)[0][0]
                    if self._band_auto and self.band_calibration is None:
                        from efficient_kws.model import calibrate_band
                        self.band_calibration = calibrate_band(self.kws, u[0], um[0], u32, self.keyword_feats,
                                                               self.keyword_mask, self.keyword_feats32)
                        self.exact_band = self.band_calibration["band"]
                    logits, _ = self.kws.score_exact(u[0], um[0], self.keyword_feats, self.keyword_mask, u32,
                                                     self.keyword_feats32, 0.5, self.exact_band, band_x3=1e-4,
                                                     fp8_band=self.fp8_band)
                else:
                    logits = self.kws.score(u[0], um[0], self.keyword_feats, self.keyword_mask)
                _, ix = spot(logits, None, 0.5, mode="argmax")
                idx = ix.tolist()
            out.append([self.keywords[i] for i in sorted(set(idx))])
        return out

    def keyword_spotting(self, input_features: torch.Tensor, start_of_prev: bool = False) -> List[List[int]]:
        """cb_whisper.py:82-149 — the PBAWhisper.generate callback."""
        S = input_features.size(0)
        if not self.prompt:
            return [[] for _ in range(S)]
        if self.oracle == "kws":
            keywords = self.spot_keywords(input_features) if len(self.keywords) else [[] for _ in range(S)]
            if S > 1 and self.segment_keywords == "union":
                # cb_whisper.py:89,129: ``keywords = [[]] * num_segments`` then ``keywords[seg_idx] += ...``
                # extends ONE list shared by every segment, so each segment of a batch gets the keywords spotted in
                # any of them (then set()); the reference's behaviour, kept (segment_keywords="per_segment": each
                # segment its own)
                index = {k: i for i, k in enumerate(self.keywords)}
                union = sorted(set(k for kw in keywords for k in kw), key=lambda k: index[k])
                keywords = [list(union) for _ in range(S)]
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
        tok = getattr(self.whisper, "tokenizer", None)
        if self.detokenize is None and tok is not None:
            return tok.decode(toks, skip_special_tokens=True).strip()
        if self.detokenize is None:
            return toks
        special = set(range(self.whisper.tokens.eot, self.whisper.decoder_config[0]))
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
