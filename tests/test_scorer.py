"""Evaluation — CPU.

* tokenizer + entity recall vs tests/golden/scorer.json, produced by the reference's own
  src/priberam_tokenizer.py and src/scorer.py (make_golden.py scorer; string2string, absent,
  replaced by cbw.alignment in that run: the aligner itself is "parity unpinned");
* the Needleman-Wunsch restatement on hand-checked alignments;
* the PR-curve restatement (torchmetrics 1.2.0, absent) vs scikit-learn's precision_recall_curve,
  the operating-point rule and the bootstrap CI plumbing of KWSModel.on_test_epoch_end.
"""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "tests"))


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLDEN, "scorer.json"), encoding="utf-8") as f:
        return json.load(f)


def test_tokenizer_matches_reference(gold):
    from priberam_tokenizer import PriberamTokenizer
    from scorer_cases import TOKENIZER_TEXTS
    tk = PriberamTokenizer()
    for text, want in zip(TOKENIZER_TEXTS, gold["tokenize"]):
        got = [[list(t) for t in sent] for sent in tk.tokenize(text)]
        assert got == want, text
    texts = [s for s in TOKENIZER_TEXTS if s.strip()]
    for text, want in zip(texts, gold["just_split_sentences"]):
        assert [[list(t) for t in sent] for sent in tk.just_split_sentences(text)] == want, text


def test_entity_recall_matches_reference(gold):
    from scorer import entity_recall
    from scorer_cases import RECALL_CASES
    preds = [c[0] for c in RECALL_CASES]
    refs = [c[1] for c in RECALL_CASES]
    ments = [c[2] for c in RECALL_CASES]
    for rec in gold["recall"]:
        tags, cs = rec["ner_tags"], rec["char_split"]
        assert entity_recall(preds, refs, ments, tags, char_split=cs) == rec["all"], (tags, cs)
        for (p, r, m), want in zip(RECALL_CASES, rec["per_case"]):
            assert entity_recall([p], [r], [m], tags, char_split=cs) == want, (tags, cs, p)


def test_needleman_wunsch_alignment():
    from cbw.alignment import NeedlemanWunsch
    nw = NeedlemanWunsch()
    a, b = nw.get_alignment(list("abcbd"), list("abcde"))
    # the library's documented example (string2string README, NeedlemanWunsch defaults)
    assert (a, b) == ("a | b | c | b | d | -", "a | b | c | - | d | e")
    # the score of the optimum equals the classic edit-distance form: matches - mismatches - gaps
    S = nw.score_matrix(list("kitten"), list("sitting"))
    assert S[-1, -1] == 1.0          # 4 matches, 2 substitutions, 1 gap
    a, b = nw.get_alignment(["ab", "c"], ["ab", "xyz", "c"])
    assert a.split(" | ") == ["ab", "-  ", "c"] and b.split(" | ") == ["ab", "xyz", "c"]
    assert nw.get_alignment([], ["x"]) == ("-", "x") and nw.get_alignment([], []) == ("", "")
    # vectorised row update == the plain triple loop
    rng = np.random.default_rng(0)
    for _ in range(20):
        s1 = list(rng.choice(list("abcd"), rng.integers(0, 12)))
        s2 = list(rng.choice(list("abcd"), rng.integers(0, 12)))
        S = nw.score_matrix(s1, s2)
        R = np.zeros((len(s1) + 1, len(s2) + 1))
        R[:, 0] = -np.arange(len(s1) + 1)
        R[0, :] = -np.arange(len(s2) + 1)
        for i in range(1, len(s1) + 1):
            for j in range(1, len(s2) + 1):
                R[i, j] = max(R[i - 1, j - 1] + (1 if s1[i - 1] == s2[j - 1] else -1), R[i - 1, j] - 1, R[i, j - 1] - 1)
        np.testing.assert_array_equal(S, R)


def test_pr_curve_matches_sklearn():
    from sklearn.metrics import precision_recall_curve
    from cbw.metrics import binary_precision_recall_curve
    rng = np.random.default_rng(1)
    for n in (1, 7, 200):
        p = np.round(rng.random(n), 2)          # ties included
        t = (rng.random(n) < 0.4).astype(int)
        t[0] = 1
        P, R, T = binary_precision_recall_curve(p, t)
        sp, sr, st = precision_recall_curve(t, p)
        np.testing.assert_allclose(P, sp)
        np.testing.assert_allclose(R, sr)
        np.testing.assert_allclose(T, st)


def test_operating_point_and_ci():
    from cbw.metrics import binary_precision_recall_curve, evaluate_with_conf_int, operating_point
    probs = np.array([0.9, 0.8, 0.6, 0.4, 0.3, 0.1])
    labels = np.array([1, 0, 1, 1, 0, 0])
    P, R, T = binary_precision_recall_curve(probs, labels)
    # threshold 0.5: predicted positive = {0.9, 0.8, 0.6} -> precision 2/3, recall 2/3
    pr, rc, f1 = operating_point(P, R, T, 0.5)
    assert pr == pytest.approx(2 / 3) and rc == pytest.approx(2 / 3) and f1 == pytest.approx(2 / 3)
    assert operating_point(P, R, T, 0.95)[:2] == (1.0, 0.0)

    def f(lab, smp, smp2=None):
        return operating_point(*binary_precision_recall_curve(smp, lab), 0.5)[1]

    c, (lo, hi) = evaluate_with_conf_int(probs, f, labels, [0, 0, 1, 1, 2, 2], num_bootstraps=50)
    assert c == pytest.approx(2 / 3) and 0.0 <= lo <= hi <= 1.0
    c2, ci2 = evaluate_with_conf_int(probs, f, labels, [0, 0, 1, 1, 2, 2], num_bootstraps=50)
    assert (c2, ci2) == (c, (lo, hi))   # seeded resamples: reproducible


def test_kwsmodel_test_epoch_metrics():
    import torch
    from efficient_kws.model import KWSModel
    m = KWSModel(threshold=0.5)
    m.on_test_epoch_start()
    m.test_step_outputs.append({"preds": torch.tensor([0.9, 0.8, 0.6]), "targets": torch.tensor([1, 0, 1]),
                                "speaker": "a"})
    m.test_step_outputs.append({"preds": torch.tensor([0.4, 0.3, 0.1]), "targets": torch.tensor([1, 0, 0]),
                                "speaker": "b"})
    out = m.on_test_epoch_end(num_bootstraps=20)
    assert out["Precision"] == pytest.approx(2 / 3) and out["Recall"] == pytest.approx(2 / 3)
    assert out["Recall_LB"] <= out["Recall_UB"] and m.test_step_outputs == []
    assert out["pr_data"]["thresholds"] == sorted(out["pr_data"]["thresholds"])


def test_cbwhisper_entity_recall_epoch():
    """CBWhisper.on_test_epoch_end (cb_whisper.py:244-289) over recorded step outputs: mentions from
    the database keywords' regex matches, speaker-conditioned CI."""
    from types import SimpleNamespace
    from model.cb_whisper import CBWhisper
    from scorer import entity_recall
    cb = CBWhisper.from_components(whisper=None, kws=SimpleNamespace(n_layers=3),
                                   kws_encoder=SimpleNamespace(n_layers=32),
                                   keywords=["BERT", "Transformer", "Dublin"], keyword_feats=None, keyword_mask=None,
                                   tokenize=lambda s: [])
    cb.on_test_epoch_start()
    refs = ["we use the Transformer model with BERT", "the ACL conference in Dublin", "no entities here"]
    preds = ["we use the transformer model with BERT", "the ACL conference in Dublin", "no entities"]
    for p, r, s in zip(preds, refs, ["a", "b", "a"]):
        cb.test_step_outputs.append({"preds": p, "target": r, "speaker": s})
    out = cb.on_test_epoch_end(num_bootstraps=10)
    ments = [[{"mention": k, "total_offset": r.index(k), "end_offset": r.index(k) + len(k), "ner_tag": "UNK"}
              for k in ["BERT", "Transformer", "Dublin"] if k in r] for r in refs]
    want = entity_recall(preds, refs, ments, "ALL", char_split=True)["ALL"]
    assert out["Entity Recall"] == pytest.approx(want) == pytest.approx(2 / 3)
    assert out["Entity Recall LB"] <= out["Entity Recall UB"]
