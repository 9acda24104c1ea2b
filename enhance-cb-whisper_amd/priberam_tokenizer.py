"""priberam_tokenizer — the word/sentence tokenizer entity recall runs on (reference
src/priberam_tokenizer.py:5-153; imported by src/scorer.py:3).

Same surface: ``Token(index, start, end, text, type)`` and
``PriberamTokenizer().tokenize(text) -> List[List[Token]]`` (sentences of tokens),
``just_split_sentences(text)``.  Token classes, tried in this order at every position
(priberam_tokenizer.py:21-26):
  text         a run of word characters (``\\w+``)
  paragraph    a run of CR/LF
  space        a run of other whitespace / NBSP
  full_stop    ". " or the non-latin stops U+3002, U+1362
  punctuation  one BMP character of Unicode category P*
anything in between is an ``UNK`` token.  A sentence closes after a paragraph token, after a
non-latin stop, and after ". " when the sentence already holds > 2 tokens and the token
before the stop is longer than 2 characters (the abbreviation guard, :125-132).  Token
``index`` counts from 1 inside a sentence; a trailing UNK continues the running count even
when it opens a new sentence (:136-151).

Pinned: tests/test_scorer.py checks token lists against tests/golden/scorer.json, produced by
the reference module itself (tests/golden/make_golden_scorer.py).
"""
from __future__ import annotations

import re
import unicodedata
from collections import namedtuple
from typing import Iterator, List, Tuple

Token = namedtuple("Token", ["index", "start", "end", "text", "type"])

_NONLATIN_STOPS = ("。", "።")


def _punctuation_class() -> str:
    chars = (chr(c) for c in range(0x10000) if unicodedata.category(chr(c))[0] == "P")
    return "".join(re.escape(ch) for ch in chars)


_PATTERN = None


def _pattern() -> "re.Pattern":
    global _PATTERN
    if _PATTERN is None:
        _PATTERN = re.compile(
            r"(?P<text>\w+)"
            r"|(?P<paragraph>[\r\n]+)"
            r"|(?P<space>[\s\u00a0]+)"
            r"|(?P<full_stop>\. |" + "|".join(_NONLATIN_STOPS) + ")"
            r"|(?P<punctuation>[" + _punctuation_class() + "])",
            re.UNICODE | re.MULTILINE)
    return _PATTERN


class PriberamTokenizer:
    def __init__(self):
        self.regex = _pattern()

    @staticmethod
    def is_nonlatin_fullstop(char: str) -> bool:
        return char in _NONLATIN_STOPS

    def _spans(self, text: str) -> Iterator[Tuple[str, int, int]]:
        """(type, start, end) over the whole string; UNK for unmatched gaps, TAIL for the last one."""
        cursor = 0
        for m in self.regex.finditer(text):
            if m.start() > cursor:
                yield "UNK", cursor, m.start()
            yield m.lastgroup, m.start(), m.end()
            cursor = m.end()
        if cursor < len(text):
            yield "TAIL", cursor, len(text)

    def tokenize(self, text: str) -> List[List[Token]]:
        sentences: List[List[Token]] = []
        open_sentence = False      # False: the next token starts a new sentence
        count = -1
        for kind, s, e in self._spans(text):
            if kind == "TAIL":     # trailing UNK: no index reset (priberam_tokenizer.py:137-151)
                if not open_sentence:
                    sentences.append([])
                count += 1
                sentences[-1].append(Token(count, s, e, text[s:e], "UNK"))
                break
            if not open_sentence:
                sentences.append([])
                open_sentence = True
                count = 0
            count += 1
            sentences[-1].append(Token(count, s, e, text[s:e], kind))
            if kind == "paragraph":
                open_sentence = False
            elif kind == "full_stop":
                cur = sentences[-1]
                if self.is_nonlatin_fullstop(text[s:e]) or (len(cur) > 2 and len(cur[-2].text) > 2):
                    open_sentence = False
        return sentences

    def just_split_sentences(self, text: str) -> List[List[Token]]:
        out = []
        for sent in self.tokenize(text):
            s, e = sent[0].start, sent[-1].end
            out.append([Token(0, s, e, text[s:e], "UNK")])
        return out
