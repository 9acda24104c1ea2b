"""CB-Whisper's own spotter (model/cb_whisper.py:110-128, :189-210; model/model.py:18-93) — CPU.

The numpy oracle (oracle/cnn12.py) is checked against tests/golden/cnn12.npz (the reference's
model.model.KWSModel forward; make_golden.py cnn12) and its bilinear resize against torch's
F.interpolate(bilinear, align_corners=False, antialias=False) — the kernel torchvision's tensor
resize runs (torchvision itself is not installed: resize parity pinned to that kernel).
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


@pytest.mark.parametrize("tk", [1, 9, 150, 171])
def test_resize_matches_torch_bilinear(tk):
    import oracle.cnn12 as oc
    x = np.random.default_rng(tk).standard_normal((12, tk, 1500)).astype(np.float32)
    ref = torch.nn.functional.interpolate(torch.from_numpy(x)[None], size=(150, 750), mode="bilinear",
                                          align_corners=False, antialias=False)[0].numpy()
    # fp32 rounding of the source coordinate (FMA contraction in the CPU kernel) moves a lambda by
    # ~1 ulp on a few rows: 5e-5 absolute on N(0, 1) inputs
    np.testing.assert_allclose(oc.resize_bilinear(x, (150, 750)), ref, atol=5e-5)


def test_oracle_matches_reference_cnn():
    import oracle.cnn12 as oc
    from cbw import synth
    from make_golden import cnn12_inputs
    g = np.load(os.path.join(GOLDEN, "cnn12.npz"))
    sd = synth.synth_kws_state_dict(seed=3, n_layers=12, embedding_dim=128, learn_features=False, proj_mlp=False)
    utt, kwd = cnn12_inputs()
    sims = oc.sim_matrices([kwd[1]], utt)
    m1 = oc.resize_bilinear(sims[0], (150, 750))
    np.testing.assert_allclose(m1[:, ::7, ::11], g["maps_k1_sub"], atol=1e-5)
    for k in (1, 4):   # two of the five keywords keep the CPU suite short
        lo = oc.keyword_spotting_logits(sd, [kwd[k]], utt)
        np.testing.assert_allclose(lo[0], g["logits"][k], atol=2e-4 * max(1.0, np.abs(g["logits"]).max()))


def test_model_api_state_dict_and_checkpoint(tmp_path):
    from cbw import synth
    from model.model import KWSModel
    sd = synth.synth_kws_state_dict(seed=3, n_layers=12, embedding_dim=128, learn_features=False, proj_mlp=False)
    m = KWSModel()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=True)
    assert m.hparams.num_domains == 72 and not m.hparams.adversarial_training
    with pytest.raises(RuntimeError):
        KWSModel().load_state_dict({"model.classifier.1.bias": torch.zeros(2)}, strict=True)
    p = str(tmp_path / "cb.ckpt")
    torch.save({"state_dict": m.state_dict(), "hyper_parameters": {"learning_rate": 3e-4}}, p)
    m2 = KWSModel.load_from_checkpoint(p)
    assert m2.hparams.learning_rate == 3e-4 and set(m2.state_dict()) == set(m.state_dict())
