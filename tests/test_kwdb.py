"""Keyword database (cbw.keyword_db) — CPU tests.

Golden: tests/golden/kwdb_acl.npz, produced by the reference's own ACL6060KeywordDataset
(efficient_kws/dataset.py:1677-1796) on a synthetic split folder (make_golden.py kwdb).
Checked here: the numpy oracle against it, the product's host-side loader against it
(exact: padding and masks are copies), the .bin round trip through the reference layout,
and the hs frame count (utils.py:187) against HF WhisperFeatureExtractor's unpadded length.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def golden():
    return np.load(os.path.join(GOLDEN, "kwdb_acl.npz"))


def inputs():
    from make_golden import KWDB_LENGTHS, kwdb_inputs  # seeded inputs (no reference import)
    return [f"kw{i}" for i in range(len(KWDB_LENGTHS))], kwdb_inputs()


def check_groups(groups, g):
    assert len(groups) == int(g["n_groups"])
    for gi, grp in enumerate(groups):
        assert list(grp["keywords"]) == list(g[f"g{gi}_keywords"])
        np.testing.assert_array_equal(np.asarray(grp["mask"]), g[f"g{gi}_mask"])
        np.testing.assert_array_equal(np.asarray(grp["kwd"]), g[f"g{gi}_kwd"])
        np.testing.assert_array_equal(np.asarray(grp["kwd_mask"]), g[f"g{gi}_kwd_mask"])


def test_oracle_matches_reference_dataset():
    import oracle.kwdb as okw
    kws, hs = inputs()
    groups = okw.build_groups(kws, hs, 4, 150)
    g = golden()
    check_groups(groups, g)
    for gi, grp in enumerate(groups):
        assert grp["max_length"] == int(g[f"g{gi}_max_length"])
        np.testing.assert_array_equal(grp["hs_lengths"], g[f"g{gi}_hs_lengths"])


def test_keyword_database_matches_reference(tmp_path):
    from cbw.keyword_db import KeywordDatabase, write_bin
    kws, hs = inputs()
    # through the reference's on-disk layout (.bin files, missing file = ghost)
    sf = tmp_path / "dev"
    (sf / "text").mkdir(parents=True)
    (sf / "keywords-hs" / "tts").mkdir(parents=True)
    (sf / "text" / "keywords.txt").write_text("\n".join(kws) + "\n")
    for i, x in enumerate(hs):
        if x is not None:
            write_bin(str(sf / "keywords-hs" / "tts" / f"{i}.bin"), torch.from_numpy(x))
    db = KeywordDatabase.from_split_folder(str(sf), "tts", keywords_per_group=4)
    feats, masks, ghost = db.padded(150)
    groups = []
    for gi in range(db.num_groups()):
        grp = db.group(gi)
        lo, hi = gi * 4, gi * 4 + len(grp["keywords"])
        groups.append({"keywords": grp["keywords"], "mask": grp["mask"].numpy().astype(np.int64),
                       "kwd": feats[lo:hi].numpy(), "kwd_mask": masks[lo:hi].numpy()})
    check_groups(groups, golden())
    assert ghost.tolist() == [0.0 if x is None else 1.0 for x in hs]
    assert len(db) == len(kws) and db[2]["keyword"] == "kw2"
    # last-n-layers selection (efficient_kws/dataset.py:570-573)
    f3, m3, _ = db.padded(150, n_layers=3)
    np.testing.assert_array_equal(f3.numpy(), feats[:, -3:].numpy())
    np.testing.assert_array_equal(m3.numpy(), masks[:, -3:].numpy())


def test_all_ghost_database_is_rejected():
    from cbw.keyword_db import KeywordDatabase
    with pytest.raises(ValueError):
        KeywordDatabase(["a", "b"], [None, None])


def test_bin_names_follow_reference():
    from cbw.keyword_db import bin_name
    assert bin_name("sent_12") == "sent_12.bin"
    assert bin_name("audio-00042") == "00042.bin"      # utils.py:197 strips the prefix


@pytest.mark.parametrize("n", [1600, 16000 + 80, 123457, 480000, 600000])
def test_hs_frames_match_hf_feature_extractor(n):
    """t_len (utils.py:187) = ceil(frames of the unpadded HF features / 2)."""
    from transformers import WhisperFeatureExtractor
    import oracle.kwdb as okw
    from cbw.keyword_db import hs_frames
    x = np.random.default_rng(n).standard_normal(n).astype(np.float32) * 0.1
    fe = WhisperFeatureExtractor(feature_size=80)
    frames = fe(x, sampling_rate=16000, return_tensors="np", padding=True).input_features.shape[-1]
    expect = int(np.ceil(frames / 2))
    assert okw.hs_frames(n) == expect
    assert hs_frames(n) == expect
