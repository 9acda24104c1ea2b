"""scorer.entity_recall — CB-Whisper's evaluation metric (reference src/scorer.py:6-149, called by
CBWhisper.on_test_epoch_end, src/model/cb_whisper.py:263-285 with ner_tags='ALL', char_split=True).

A mention counts as recalled when every reference token it covers is aligned to an identical
prediction token.  Steps, per (prediction, reference, mentions) triple:
  1. empty prediction: every mention of a counted tag is a miss (scorer.py:33-44);
  2. tokens of the FIRST sentence of each text (PriberamTokenizer; the reference keeps only
     ``tokenize(..)[0]``), optionally split into one token per character (:48-64);
  3. global alignment (Needleman-Wunsch, gap token '[SKIP]'), the aligned strings re-split on
     '|' exactly as the reference does, so a literal '|' token reads back as '|' (:66-99);
  4. reference-token -> mention map by the sign test (end - tok.start)·(start - tok.end) < 0
     (the last overlapping mention wins, :108-112), stretched over the gap positions of the
     aligned reference (a gap inherits the mention of its neighbours when they agree, :113-117);
  5. each maximal run of one mention index is one mention occurrence: TP if all its aligned
     positions agree, else FN (:118-144).
Recall per tag = TP / N (0 when N = 0).
Restated as code of this package; the aligner is cbw.alignment (string2string is absent).
Pinned by tests/golden/scorer.json (the reference scorer run with that aligner substituted).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Union

from cbw.alignment import NeedlemanWunsch
from priberam_tokenizer import PriberamTokenizer, Token

GAP = "[SKIP]"


def _split_aligned(seq: str) -> List[str]:
    """Aligned string -> per-position tokens (scorer.py:70-83): a field equal to ' ' marks a
    literal '|' token, which also consumed the following field."""
    fields = seq.split("|")
    out: List[str] = []
    k = 0
    while k < len(fields):
        if fields[k] == " ":
            out.append("|")
            k += 2
        else:
            out.append(fields[k].strip())
            k += 1
    return out


def _chars(tokens: Sequence[Token]) -> List[Token]:
    return [Token(-1, t.start + c, t.start + c + 1, ch, "text") for t in tokens for c, ch in enumerate(t.text)]


def _mention_runs(ref_tokens: Sequence[Token], ref_aligned: Sequence[str], mentions: Sequence[dict]) -> List[list]:
    owner = [-1] * len(ref_tokens)
    for k, tok in enumerate(ref_tokens):
        for mi, m in enumerate(mentions):
            if (m["end_offset"] - tok.start) * (m["total_offset"] - tok.end) < 0:
                owner[k] = mi
    # gap positions of the aligned reference, ascending, inserted one by one
    gaps = [p for p, t in enumerate(ref_aligned) if t.strip() == GAP]
    for p in gaps:
        if 0 < p < len(owner) and owner[p - 1] == owner[p]:
            owner.insert(p, owner[p - 1])
        else:
            owner.insert(p, -1)
    runs: List[list] = []
    p = 0
    while p < len(owner):
        mi = owner[p]
        if mi == -1:
            p += 1
            continue
        run = []
        while p < len(owner) and owner[p] == mi:
            run.append(p)
            p += 1
        runs.append([mi, run])
    return runs


def entity_recall(preds: List[str], refs: List[str], mentions: List[List[dict]],
                  ner_tags: Union[str, List[str]], char_split: bool = False) -> Dict[str, float]:
    assert not isinstance(ner_tags, str) or ner_tags == "ALL", "invalid NER tags"
    tags = ["ALL"] if ner_tags == "ALL" else list(ner_tags)
    open_tags = tags == ["ALL"]
    counts = {t: {"TP": 0, "FN": 0, "N": 0} for t in set(tags + ["ALL"])}
    tok = PriberamTokenizer()
    nw = NeedlemanWunsch(gap_char=GAP)

    def tally(tag: str, hit: bool):
        if open_tags and tag not in counts:
            counts[tag] = {"TP": 0, "FN": 0, "N": 0}
        if tag in counts:
            key = "TP" if hit else "FN"
            counts[tag]["N"] += 1
            counts["ALL"]["N"] += 1
            counts[tag][key] += 1
            counts["ALL"][key] += 1

    for pred, ref, ms in zip(preds, refs, mentions):
        if pred.strip() == "":
            for m in ms:
                tally(m["ner_tag"], False)
            continue
        p_tok = [t for t in tok.tokenize(pred)[0] if t.type != "newline"]
        r_tok = [t for t in tok.tokenize(ref)[0] if t.type != "newline"]
        if char_split:
            p_tok, r_tok = _chars(p_tok), _chars(r_tok)
        s1, s2 = nw.get_alignment([t.text for t in p_tok], [t.text for t in r_tok])
        a1, a2 = _split_aligned(s1), _split_aligned(s2)
        for mi, run in _mention_runs(r_tok, a2, ms):
            tally(ms[mi]["ner_tag"], all(a1[q] == a2[q] for q in run))

    return {k: (c["TP"] / c["N"] if c["N"] != 0 else 0) for k, c in counts.items()}
