"""Whisper text <-> token ids from a local checkpoint directory (no network, no HF dependency).

The reference builds ``WhisperProcessor.from_pretrained(whisper_ckpt)`` (src/model/cb_whisper.py:46-49)
and uses two of its methods on the hot path's host side:

* ``get_prompt_ids(text)`` (cb_whisper.py:140-147) -> ``[<|startofprev|>] + ids(" " + text.strip())``,
  raising ValueError when the prompt text encodes to a special token (transformers 4.37.2
  ``WhisperTokenizer.get_prompt_ids``);
* ``tokenizer.batch_decode(pred, skip_special_tokens=True)`` (cb_whisper.py:180-186).

This module restates the GPT-2 byte-level BPE those methods run (``WhisperTokenizer._tokenize`` /
``bpe`` / ``convert_tokens_to_string``) over the checkpoint's own files: ``vocab.json`` + ``merges.txt``
(+ ``added_tokens.json``) or a fast-tokenizer ``tokenizer.json``.  Pinned against transformers'
``WhisperTokenizer`` on the same files by tests/test_tokenizer.py.
"""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import Dict, List, Optional, Sequence

import regex

_TS = regex.compile(r"<\|\d+\.\d+\|>")   # timestamp tokens <|0.00|> .. <|30.00|>
# GPT-2 / Whisper pre-tokenisation pattern (WhisperTokenizer.pat)
_PAT = regex.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


@lru_cache()
def bytes_to_unicode() -> Dict[int, str]:
    """The reversible byte -> printable-unicode map of byte-level BPE."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


class WhisperTokenizerLite:
    def __init__(self, vocab: Dict[str, int], merges: Sequence[tuple], added: Dict[str, int],
                 special: Optional[Sequence[str]] = None, bos: Optional[str] = None):
        """``added``: every added token (added_tokens.json / added_tokens_decoder / tokenizer.json), kept even
        when vocab.json lists the same token at the same id (real Whisper files list <|endoftext|> in both);
        ``special``: the tokens transformers counts in all_special_ids (special_tokens_map.json's bos / eos / unk
        / pad + additional_special_tokens, and added tokens flagged special) -- None: every added token;
        ``bos``: the first of all_special_ids (get_prompt_ids rejects prompt ids at or above it)."""
        self.encoder = dict(vocab)
        self.encoder.update(added)
        self.decoder = {v: k for k, v in self.encoder.items()}
        self.bpe_ranks = {tuple(m): i for i, m in enumerate(merges)}
        self.added = dict(added)
        self.special = set(added) if special is None else {t for t in special if t in self.encoder}
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.cache: Dict[str, str] = {}
        specials = sorted(self.added, key=len, reverse=True)
        self._special_re = regex.compile("(" + "|".join(regex.escape(s) for s in specials) + ")") if specials else None
        self.eot = self.encoder.get("<|endoftext|>")
        # transformers' all_special_ids[0]: the bos token (<|endoftext|> for Whisper), else the lowest special id
        if bos is not None and bos in self.encoder:
            self.first_special = self.encoder[bos]
        else:
            ids = [self.encoder[t] for t in self.special] or list(self.added.values())
            self.first_special = min(ids) if ids else None

    # ------------------------------------------------------------------ loading
    @classmethod
    def from_dir(cls, path: str) -> "WhisperTokenizerLite":
        tj = os.path.join(path, "tokenizer.json")

        def load(name):
            f = os.path.join(path, name)
            if not os.path.exists(f):
                return None
            with open(f, encoding="utf-8") as fh:
                return json.load(fh)

        def tok(v):   # special_tokens_map entries are strings or AddedToken dicts
            return v.get("content") if isinstance(v, dict) else v

        smap = load("special_tokens_map.json")
        tcfg = load("tokenizer_config.json") or {}
        special, bos = None, None
        if smap is not None:
            special = [tok(smap[k]) for k in ("bos_token", "eos_token", "unk_token", "pad_token") if smap.get(k)]
            special += [tok(v) for v in smap.get("additional_special_tokens") or []]
            bos = tok(smap.get("bos_token")) if smap.get("bos_token") else None
        flagged = [v["content"] for v in (tcfg.get("added_tokens_decoder") or {}).values() if v.get("special")]
        if os.path.exists(os.path.join(path, "vocab.json")) and os.path.exists(os.path.join(path, "merges.txt")):
            vocab = load("vocab.json")
            with open(os.path.join(path, "merges.txt"), encoding="utf-8") as f:
                lines = f.read().split("\n")
            merges = [tuple(ln.split()) for ln in lines if ln and not ln.startswith("#version") and len(ln.split()) == 2]
            added: Dict[str, int] = dict(load("added_tokens.json") or {})
            for k, v in (tcfg.get("added_tokens_decoder") or {}).items():
                added.setdefault(v["content"], int(k))
            if special is not None or flagged:
                special = list(special or []) + flagged
            return cls(vocab, merges, added, special, bos)
        if os.path.exists(tj):
            d = load("tokenizer.json")
            m = d["model"]
            merges = [tuple(x.split()) if isinstance(x, str) else tuple(x) for x in m["merges"]]
            added = {t["content"]: int(t["id"]) for t in d.get("added_tokens", [])}
            flagged += [t["content"] for t in d.get("added_tokens", []) if t.get("special")]
            if special is not None or flagged:
                special = list(special or []) + flagged
            return cls(m["vocab"], merges, added, special, bos)
        raise FileNotFoundError(f"no tokenizer files (vocab.json + merges.txt or tokenizer.json) in {path}")

    # ------------------------------------------------------------------ BPE
    def bpe(self, token: str) -> str:
        if token in self.cache:
            return self.cache[token]
        word = tuple(token)
        if len(word) < 2:
            return token
        while True:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            a, b = best
            out, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(word[i])
                    i += 1
            word = tuple(out)
            if len(word) == 1:
                break
        res = " ".join(word)
        self.cache[token] = res
        return res

    def _encode_plain(self, text: str) -> List[int]:
        ids = []
        for piece in _PAT.findall(text):
            u = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            for t in self.bpe(u).split(" "):
                if t not in self.encoder:
                    raise KeyError(f"BPE piece {t!r} missing from the vocabulary")
                ids.append(self.encoder[t])
        return ids

    def encode(self, text: str) -> List[int]:
        """add_special_tokens=False: added tokens in the text map to their ids, the rest is BPE."""
        if self._special_re is None:
            return self._encode_plain(text)
        ids = []
        for part in self._special_re.split(text):
            if not part:
                continue
            ids.extend([self.added[part]] if part in self.added else self._encode_plain(part))
        return ids

    def convert_tokens_to_ids(self, token: str) -> Optional[int]:
        return self.encoder.get(token)

    # ------------------------------------------------------------------ reference methods
    def get_prompt_ids(self, text: str) -> List[int]:
        """WhisperTokenizer.get_prompt_ids (transformers 4.37.2) as a list."""
        sop = self.encoder["<|startofprev|>"]
        ids = self.encode(" " + text.strip())
        bad = next((x for x in ids if self.first_special is not None and x >= self.first_special), None)
        if bad is not None:
            raise ValueError(f"Encountered text in the prompt corresponding to disallowed special token: "
                             f"{self.decoder.get(bad)}.")
        return [sop] + ids

    def decode(self, ids: Sequence[int], skip_special_tokens: bool = False, decode_with_timestamps: bool = False) -> str:
        """WhisperTokenizer.decode: timestamp tokens are filtered unless decode_with_timestamps
        (_filter_timestamp_ids); skip_special_tokens drops the <|startofprev|> prompt up to
        <|startoftranscript|> (_strip_prompt) and every special token (all_special_ids)."""
        ids = [int(i) for i in ids]
        if not decode_with_timestamps:
            ids = [i for i in ids if not _TS.fullmatch(self.decoder.get(i, ""))]
        if skip_special_tokens:
            sop, sot = self.encoder.get("<|startofprev|>"), self.encoder.get("<|startoftranscript|>")
            if sop is not None and sop in ids:
                a = ids.index(sop)
                b = ids.index(sot, a) if sot in ids[a:] else len(ids)
                ids = ids[:a] + ids[b:]
            ids = [i for i in ids if i not in self.decoder or self.decoder[i] not in self.special]
        out, buf = [], []

        def flush():
            if buf:
                out.append(bytearray(self.byte_decoder[c] for c in "".join(buf) if c in self.byte_decoder)
                           .decode("utf-8", errors="replace"))
                buf.clear()

        for i in ids:
            t = self.decoder.get(i, "")
            if t in self.added:      # added tokens decode to their literal text
                flush()
                out.append(t)
            else:
                buf.append(t)
        flush()
        return "".join(out)

    def batch_decode(self, seqs, skip_special_tokens: bool = False) -> List[str]:
        return [self.decode(s, skip_special_tokens) for s in seqs]
