"""CB-Whisper built by its reference constructor (src/model/cb_whisper.py:21-80) from local checkpoints, and
its ``keyword_spotting`` (:82-149) against the oracle restatement (oracle/cbwhisper.py): encoder
hidden_states[10:22] -> per-keyword similarity + bilinear resize + 12-channel ResNet-50 -> argmax -> dedup ->
``get_prompt_ids`` prompt (VERDICT r01 a11 / ADVICE: spotting pinned, not self-compared).

Three keywords are planted (their hs are slices of the utterance's own hidden states) and the CNN's class-1
bias is shifted so that exactly those win: the oracle's argmax margins are >= 0.5 logits away from a tie
(asserted), far outside the bf16 logit tolerance (2e-2 of max|logit|), so the spotted keyword lists and the
prompt token ids must be identical.
"""
import os

import numpy as np
import pytest
import torch

from cbw import synth

pytestmark = pytest.mark.gpu

PROMPT = dict(keyword_prompt_prepend="The topic of today's speech is, ah, ",
              keyword_prompt_append=". Okay, then I'll continue.", keyword_separator=", ")


@pytest.fixture(scope="module")
def planted(tmp_path_factory):
    import oracle.cbwhisper as ocb
    import oracle.mel as omel
    enc_sd = synth.synth_whisper_encoder_state_dict("micro-deep", 0)
    mel = omel.log_mel(synth.synth_clip(0), 80)
    u = ocb.utterance_hs(enc_sd, mel, synth.WHISPER_CONFIGS["micro-deep"][3])
    khs = {0: u[:, 100:140], 2: u[:, 700:725], 4: u[:, 1200:1260]}
    paths = synth.write_cbwhisper_fixture(str(tmp_path_factory.mktemp("cbwgpu")), keyword_hs=khs,
                                          cnn_class1_shift=-2.5)
    return paths, enc_sd, mel


def build(paths, **kw):
    from model.cb_whisper import CBWhisper
    args = dict(dataset="acl", split="test", root=paths["acl"], kw_type="tts", encoder_ckpt=paths["encoder"],
                whisper_ckpt=paths["whisper"], kws_ckpt=paths["kws_ckpt"], language="English", prompt=True,
                oracle="kws", kws_features_size=(150, 750), keywords_per_group=100, **PROMPT)
    args.update(kw)
    return CBWhisper(**args)


def test_keyword_spotting_matches_oracle(planted):
    import oracle.cbwhisper as ocb
    paths, enc_sd, mel = planted
    cb = build(paths)
    feats = torch.from_numpy(mel[None]).cuda()
    ids = cb.keyword_spotting(feats, start_of_prev=True)
    got = cb.last_spotted
    ck = torch.load(paths["kws_ckpt"], map_location="cpu", weights_only=True)["state_dict"]
    ksd = {k: v.numpy() for k, v in ck.items()}
    khs = [h.numpy() for h in cb.kw_database.db.hidden_states]
    want, want_ids, lgs = ocb.keyword_spotting(enc_sd, synth.WHISPER_CONFIGS["micro-deep"][3], mel[None], ksd, khs,
                                               cb.keywords, cb.get_prompt_ids, 100, (150, 750), cb.prepend, cb.append,
                                               cb.sep, start_of_prev=True)
    margin = lgs[0][:, 1] - lgs[0][:, 0]
    print("oracle argmax margins", np.round(margin, 3), "spotted", want[0])
    assert np.abs(margin).min() >= 0.5, "test setup: a keyword sits near the argmax tie"
    assert want[0] == ["alpha", "charlie", "echo"]          # the planted keywords; the ghost is not spotted
    assert got == want
    assert ids == want_ids
    assert ids[0][0] == cb.whisper.tokenizer.convert_tokens_to_ids("<|startofprev|>")
    assert cb.keyword_spotting(feats, start_of_prev=False) == [want_ids[0][1:]]
    # GPU logits of the same spotter against the oracle's
    from cbw.kws import pack_keywords
    eng = cb.cnn.engine(128)
    pk = torch.zeros((1, 3000, cb.kws_encoder.cpad), dtype=torch.bfloat16, device=feats.device)
    pk[0, :, :80] = feats[0].t().to(torch.bfloat16)
    hs = cb.kws_encoder.hidden_states(pk, cb.layer_ids, normalize=True)[0]
    lg = eng.score_resized(hs, pack_keywords(cb.keyword_hs, feats.device)).cpu().numpy()
    np.testing.assert_allclose(lg, lgs[0], atol=2e-2 * np.abs(lgs[0]).max())


def test_prompt_off_and_oracle_modes(planted):
    paths, _, mel = planted
    feats = torch.from_numpy(mel[None]).cuda()
    assert build(paths, prompt=False).keyword_spotting(feats) == [[]]
    cb = build(paths, oracle="gold")
    cb.oracle_buffer = ["bravo", "delta"]
    ids = cb.keyword_spotting(feats, start_of_prev=True)
    assert ids == [cb.get_prompt_ids(cb.prepend + "bravo, delta" + cb.append)]


def test_forward_transcribes_and_runner_synthetic(planted, capsys):
    import importlib.util
    import json
    paths, _, mel = planted
    cb = build(paths)
    gen = cb.whisper.generate
    cb.whisper.generate = lambda *a, **k: gen(*a, max_new_tokens=8, **k)
    text = cb.forward(torch.from_numpy(mel[None]).cuda(), None)
    assert isinstance(text, str)
    assert cb.last_spotted == [["alpha", "charlie", "echo"]]
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "enhance-cb-whisper_amd")
    spec = importlib.util.spec_from_file_location("cb_whisper_cli", os.path.join(here, "cb-whisper.py"))
    runner = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(runner)
    import yaml
    cfg = {"model": {"class_path": "model.cb_whisper.CBWhisper",
                     "init_args": dict(dataset="acl", split="test", root=paths["acl"], kw_type="tts",
                                       encoder_ckpt=paths["encoder"], whisper_ckpt=paths["whisper"],
                                       kws_ckpt=paths["kws_ckpt"], language="English", prompt=True, oracle="kws",
                                       kws_features_size=[150, 750], keywords_per_group=100, **PROMPT)}}
    p = os.path.join(os.path.dirname(paths["acl"]), "cfg.yaml")
    with open(p, "w") as f:
        yaml.safe_dump(cfg, f)
    assert runner.main(["test", "--config", p, "--synthetic", "1", "--max-new-tokens", "6"]) == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert len(out["results"]) == 1 and isinstance(out["results"][0]["pred"], str)
