"""Global (Needleman-Wunsch) alignment of token sequences — the aligner entity recall uses
(reference src/scorer.py:2,22,67: ``string2string.alignment.NeedlemanWunsch(gap_char='[SKIP]')``).

string2string==0.0.150 (requirements.txt:14) is a third-party dependency absent from the
reference tree and from this image; this module restates its published algorithm:
  * scores: match +1, mismatch -1, gap -1 (the library defaults);
  * first row / column: cumulative gap scores; cell = max(diagonal + match/mismatch,
    up + gap, left + gap);
  * traceback from (n, m) preferring diagonal, then "up" (gap in the second sequence), then
    "left" (gap in the first), each aligned pair right-padded with spaces to equal width;
  * output: the two aligned sequences as strings joined by " | " (scorer.py:70-99 parses
    exactly that form, including the two empty fields a literal "|" token produces).
The DP row update is vectorised: with t[j] = max(diagonal, up), the left-gap recurrence
s[j] = max(t[j], s[j-1] - 1) is a prefix maximum of t[j] + j, minus j.  Scores are small
integers, so the float comparisons of the traceback are exact.
Parity: "unpinned" against string2string itself (absent); tests/test_scorer.py pins the
reference scorer's use of it through golden outputs generated with this restatement
substituted for the library (tests/golden/make_golden_scorer.py).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


class NeedlemanWunsch:
    def __init__(self, match_weight: float = 1.0, mismatch_weight: float = -1.0, gap_weight: float = -1.0,
                 gap_char: str = "-"):
        self.match_weight = match_weight
        self.mismatch_weight = mismatch_weight
        self.gap_weight = gap_weight
        self.gap_char = gap_char

    @staticmethod
    def _pad(a: str, b: str) -> Tuple[str, str]:
        w = max(len(a), len(b))
        return a.ljust(w), b.ljust(w)

    def score_matrix(self, s1: Sequence[str], s2: Sequence[str]) -> np.ndarray:
        n, m = len(s1), len(s2)
        g = self.gap_weight
        S = np.zeros((n + 1, m + 1), dtype=np.float64)
        S[0, :] = g * np.arange(m + 1)
        S[:, 0] = g * np.arange(n + 1)
        if n == 0 or m == 0:
            return S
        # match matrix via integer codes of the tokens
        vocab = {}
        c1 = np.array([vocab.setdefault(t, len(vocab)) for t in s1], dtype=np.int64)
        c2 = np.array([vocab.setdefault(t, len(vocab)) for t in s2], dtype=np.int64)
        jj = np.arange(1, m + 1, dtype=np.float64)
        for i in range(1, n + 1):
            sub = np.where(c2 == c1[i - 1], self.match_weight, self.mismatch_weight)
            t = np.maximum(S[i - 1, :-1] + sub, S[i - 1, 1:] + g)
            t = np.concatenate(([S[i, 0]], t))
            if g == -1.0:
                jv = np.concatenate(([0.0], jj))
                S[i, :] = np.maximum.accumulate(t + jv) - jv
            else:   # general gap weight: sequential left-gap pass
                row = t.copy()
                for j in range(1, m + 1):
                    row[j] = max(row[j], row[j - 1] + g)
                S[i, :] = row
        return S

    def get_alignment(self, str1: Sequence[str], str2: Sequence[str], return_score_matrix: bool = False):
        S = self.score_matrix(str1, str2)
        i, j = len(str1), len(str2)
        a1: List[str] = []
        a2: List[str] = []
        g = self.gap_weight
        while i > 0 or j > 0:
            if i > 0 and j > 0 and S[i, j] == S[i - 1, j - 1] + (
                    self.match_weight if str1[i - 1] == str2[j - 1] else self.mismatch_weight):
                x, y = self._pad(str1[i - 1], str2[j - 1])
                i, j = i - 1, j - 1
            elif i > 0 and S[i, j] == S[i - 1, j] + g:
                x, y = self._pad(str1[i - 1], self.gap_char)
                i -= 1
            else:
                x, y = self._pad(self.gap_char, str2[j - 1])
                j -= 1
            a1.append(x)
            a2.append(y)
        out1 = " | ".join(reversed(a1))
        out2 = " | ".join(reversed(a2))
        if return_score_matrix:
            return out1, out2, S
        return out1, out2
