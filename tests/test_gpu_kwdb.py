"""Keyword database on the GPU: hs extraction (utils.py:182-201) vs the numpy oracle
(mel + encoder), .bin round trip through the reference layout, and the projected cache
equal to KwsEngine.project of the padded keywords (bit-exact)."""
import numpy as np
import pytest
import torch

from cbw import synth

pytestmark = pytest.mark.gpu


def test_extract_hidden_states_vs_oracle(tmp_path):
    import oracle.encoder as oenc
    import oracle.mel as omel
    from cbw.keyword_db import KeywordDatabase, build_split_folder, extract_hidden_states, hs_frames
    from cbw.whisper import EncoderEngine
    cfg = synth.WHISPER_CONFIGS["micro"]
    sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    eng = EncoderEngine(cfg, sd)
    pcm = synth.synth_clip(3, seconds=2.37)
    ids = [1, 2, 3]
    hs = extract_hidden_states(pcm, eng, ids).cpu().numpy()
    T = hs_frames(pcm.size)
    assert hs.shape == (3, T, cfg[1]) and T == 119
    ref = np.stack(oenc.encoder_hidden_states(sd, omel.log_mel(pcm, cfg[0]), cfg[3]))[ids][:, :T]
    ref = ref / np.linalg.norm(ref, axis=-1, keepdims=True)
    np.testing.assert_allclose(hs, ref, atol=2e-2)
    # .bin files in the reference layout, one ghost
    build_split_folder(str(tmp_path), ["a", "b", "c"], {0: pcm, 2: synth.synth_clip(4, seconds=1.1)}, eng, "tts", ids)
    db = KeywordDatabase.from_split_folder(str(tmp_path), "tts", keywords_per_group=2)
    assert db.ghost_mask.tolist() == [1.0, 0.0, 1.0]
    np.testing.assert_array_equal(db.hidden_states[0].numpy(), hs)
    assert db.hidden_states[1].shape == db.hidden_states[2].shape      # ghost = zeros like the shortest
    assert float(db.hidden_states[1].abs().sum()) == 0.0


def test_projected_cache_equals_project(tmp_path):
    from cbw.keyword_db import KeywordDatabase
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
    g = np.random.default_rng(1)
    hs = []
    for T in (12, None, 150, 170, 40):
        if T is None:
            hs.append(None)
            continue
        x = g.standard_normal((12, T, 128)).astype(np.float32)
        hs.append(torch.from_numpy(x / np.linalg.norm(x, axis=-1, keepdims=True)))
    db = KeywordDatabase([f"k{i}" for i in range(5)], hs, keywords_per_group=2)
    pk, pm, ghost = db.projected(eng, chunk=2)
    f, m, _ = db.padded(150, 3)
    ek, em = eng.project(f.to(eng.device), m.to(eng.device))
    torch.testing.assert_close(pk, ek, rtol=0, atol=0)
    torch.testing.assert_close(pm, em, rtol=0, atol=0)
    assert ghost.tolist() == [1.0, 0.0, 1.0, 1.0, 1.0]
    p = str(tmp_path / "db.safetensors")
    db.save_projected(p, eng)
    lk, lm, lg = KeywordDatabase.load_projected(p, eng.device)
    torch.testing.assert_close(lk, pk, rtol=0, atol=0)
    torch.testing.assert_close(lm, pm, rtol=0, atol=0)
