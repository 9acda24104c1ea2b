"""CPU-only tests: the C-ABI library loads and exports every symbol include/cbw.h
declares, host-side API logic (hparams, variants, state-dict naming, checkpoint
remap), synthetic-data determinism.  No compute calls (no GPU here)."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO


def header_functions():
    src = open(os.path.join(REPO, "include", "cbw.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(cbw_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    from cbw import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"libcbw.so does not export {n}"
    # the ctypes table covers exactly the header
    assert sorted(_lib.SIGNATURES) == names
    assert lib.cbw_version() == 1


def _check_library_matches_sources():
    import hashlib
    from cbw import _lib
    csrc = os.path.join(REPO, "enhance-cb-whisper_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    srcs = re.search(r"^SRCS = (.*)$", mk, flags=re.M).group(1).split()
    hdrs = re.search(r"^HDRS = (.*)$", mk, flags=re.M).group(1).split()
    h = hashlib.sha256()
    for f in srcs + hdrs:
        h.update(open(os.path.join(csrc, f), "rb").read())
    assert _lib.load().cbw_source_id().decode() == h.hexdigest()[:16]


def test_library_matches_sources():
    """The libcbw.so in the tree was built from the sources in the tree (csrc/Makefile's SRC_ID: sha256 over SRCS then
    HDRS): a stale prebuilt library would fail here."""
    _check_library_matches_sources()


@pytest.mark.gpu
def test_library_matches_sources_on_gpu_box():
    """The same check in the GPU suite: the driver's `pytest -m gpu` runs on the box with the
    prebuilt libcbw.so that travelled there, so a stale library fails the GPU suite too."""
    _check_library_matches_sources()


def test_runtime_host_sanitizers():
    """The runtime's host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; tools/sanitize_host.sh:
    runtime.cpp rebuilt with -Xarch_host -fsanitize=address,undefined, linked with tests/sanitize/host_driver.cpp):
    cbw_dtw over 209 shapes (path properties and minimal cost vs an f64 dynamic programme) and every constructor's
    argument checks, including the zero-head configurations whose d_model / n_heads check divided by zero before
    this test existed.  Any sanitizer report or failed check exits non-zero."""
    import shutil
    import subprocess
    script = os.path.join(REPO, "tools", "sanitize_host.sh")
    built = os.path.join(REPO, "enhance-cb-whisper_amd", "csrc", "build", "runtime.cpp.o")
    if not (os.path.exists(script) and os.path.exists(built) and shutil.which("/opt/rocm/bin/hipcc")):
        pytest.skip("needs hipcc, the in-tree build objects and tools/sanitize_host.sh (not on the GPU box)")
    out = os.path.join("/tmp", f"cbw_sanitize_{os.getpid()}")
    r = subprocess.run(["bash", script], env={**os.environ, "OUT": out}, capture_output=True, text=True, timeout=600)
    shutil.rmtree(out, ignore_errors=True)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "all checks passed" in r.stdout


def test_null_handle_errors_are_reported():
    from cbw import _lib
    lib = _lib.load()
    rc = lib.cbw_kws_finalize(None)
    assert rc == -1
    assert b"null" in lib.cbw_last_error()
    with pytest.raises(ValueError):
        _lib.check(rc, "cbw_kws_finalize")


def test_kws_create_validates_config():
    import ctypes
    from cbw import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    bad = _lib.KwsConfig(12, 1280, 2, 64, 50)          # n_layers > 4
    assert lib.cbw_kws_create(ctypes.byref(bad), ctypes.byref(h)) == -1
    bad = _lib.KwsConfig(3, 1280, 2, 64, 101)          # resnet depth
    # create succeeds (depth is checked at finalize); finalize must fail without params
    if lib.cbw_kws_create(ctypes.byref(bad), ctypes.byref(h)) == 0:
        assert lib.cbw_kws_finalize(h) != 0
        lib.cbw_kws_destroy(h)


def test_variant_mapping():
    from cbw.kws import variant_of, VARIANT_L, VARIANT_LE, VARIANT_LEF, lef_frames
    assert variant_of(dict(learn_features=False)) == VARIANT_L
    assert variant_of(dict(learn_features=True, proj_mlp=False)) == VARIANT_L      # train-L.yaml (reference crashes)
    assert variant_of(dict(learn_features=True, proj_mlp=True)) == VARIANT_LE
    assert variant_of(dict(learn_features=True, proj_mlp=True, frames_conv=True)) == VARIANT_LEF
    assert lef_frames(150) == 75 and lef_frames(1500) == 750 and lef_frames(1) == 1 and lef_frames(8) == 4


def test_state_dict_names_match_reference_layout():
    from cbw.synth import kws_param_shapes
    names = kws_param_shapes(3, 1280, True, True, True, 64, "resnet-50")
    assert len(names) == 353                       # 353 LEF keys
    d = {n: s for n, s, _ in names}
    assert d["model.feature_extractor.embedder.embedder.convolution.weight"] == (64, 3, 7, 7)
    assert d["model.classifier.1.weight"] == (2, 2048)
    assert d["projector.0.0.weight"] == (640, 1280)
    assert d["time_projector.2.0.weight"] == (64, 64, 3)


def test_synth_is_deterministic():
    from cbw import synth
    a = synth.synth_kws_state_dict(seed=3, n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True,
                                   frames_conv=True)
    b = synth.synth_kws_state_dict(seed=3, n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True,
                                   frames_conv=True)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    x = synth.synth_kws_batch(seed=1, K=3, n_layers=3, D=64, ghost=(2,))
    y = synth.synth_kws_batch(seed=1, K=3, n_layers=3, D=64, ghost=(2,))
    np.testing.assert_array_equal(x["kwd"], y["kwd"])
    assert x["ghost_mask"].tolist() == [1, 1, 0]
    n = np.linalg.norm(x["kwd"][0, 0, :150], axis=-1)
    np.testing.assert_allclose(n, 1.0, rtol=1e-5)


def test_kwsmodel_load_state_dict_strict_and_remap(tmp_path):
    from cbw import synth
    from efficient_kws.model import KWSModel
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True,
              features_size=(150, 1500))
    m = KWSModel(**hp)
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    m.load_state_dict(sd)
    assert len(m.state_dict()) == 353
    bad = dict(sd)
    bad.pop("model.classifier.1.bias")
    with pytest.raises(RuntimeError):
        KWSModel(**hp).load_state_dict(bad)
    # Lightning checkpoint round trip (weights_only load) with the legacy `model.resnet.` layout
    legacy = {}
    for k, v in sd.items():
        if k.startswith("model.feature_extractor."):
            legacy["model.resnet." + k[len("model.feature_extractor."):]] = torch.from_numpy(np.asarray(v))
        elif k.startswith("model.classifier"):
            legacy["model.resnet.classifier" + k[len("model.classifier"):]] = torch.from_numpy(np.asarray(v))
        else:
            legacy[k] = torch.from_numpy(np.asarray(v))
    ckpt = {"state_dict": legacy, "hyper_parameters": hp}
    path = tmp_path / "kws.ckpt"
    torch.save(ckpt, path)
    m2 = KWSModel.load_from_checkpoint(str(path))
    assert m2.hparams.frames_conv is True
    for k, v in sd.items():
        np.testing.assert_array_equal(m2.state_dict()[k].numpy(), v)


def test_default_layer_ids():
    from cbw.whisper import default_layer_ids
    assert default_layer_ids(32) == [19, 20, 21]      # large-v3: hs[10:22][-3:]
    assert default_layer_ids(12) == [10, 11, 12]      # small: 12 = post-LN
    assert default_layer_ids(4) == [2, 3, 4]          # tiny: [10:22] empty -> hs[-3:]


@pytest.mark.parametrize("cfg", ["eval-LEF-comp-acl.yaml", "eval-LE-comp-acl.yaml", "eval-L-comp-acl.yaml",
                                 "train-LEF.yaml", "train-L.yaml"])
def test_reference_yaml_builds_model(cfg):
    """The reference's own YAML configs (read as text, this container only) build the
    drop-in KWSModel through the same class_path/init_args as LightningCLI would."""
    path = os.path.join("/root/reference/src/efficient_kws/configs", cfg)
    if not os.path.exists(path):
        pytest.skip("reference configs not present (GPU box)")
    import yaml
    from run_efficient_kws import build_model
    from cbw.kws import variant_of
    m = build_model(yaml.safe_load(open(path)))
    assert type(m).__name__ == "KWSModel"
    assert m.hparams.n_layers == 3
    assert tuple(m.hparams.features_size) == (150, 1500)
    expect = {"LEF": 2, "LE": 1, "L": 0}[cfg.split("-")[1].split(".")[0]]
    assert variant_of(vars(m.hparams)) == expect


def test_entry_point_builds_from_yaml(tmp_path, capsys):
    import yaml
    from run_efficient_kws import main
    cfg = {"model": {"class_path": "efficient_kws.model.KWSModel",
                     "init_args": {"n_layers": 3, "embedding_dim": 1280, "learn_features": True, "proj_mlp": True,
                                   "frames_conv": True, "features_size": [150, 1500], "threshold": ["THRESHOLD"]}},
           "ckpt_path": ["CKPT"]}
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(cfg))
    assert main(["test", "--config", str(p)]) == 0
    assert "KWSModel" in capsys.readouterr().out
    with pytest.raises(SystemExit):
        main(["fit", "--config", str(p)])


def test_shortform_prefix_cuts_long_keyword_prompts():
    """transformers 4.37.2 _set_forced_decoder_ids (requirements.txt:21): <|startofprev|> + the last
    -max_target_positions // 2 - 1 text prompt tokens + the init tokens; short prompts pass unchanged."""
    from model.pba_whisper import shortform_prefix
    sop, init = 50361, [50258, 50259, 50360, 50363]
    assert shortform_prefix([], init) == init
    short = [sop, 11, 12, 13]
    assert shortform_prefix(short, init) == short + init
    long = [sop] + list(range(1000, 1600))
    p = shortform_prefix(long, init)
    assert p[0] == sop and p[1:-4] == long[-225:] and p[-4:] == init and len(p) == 1 + 225 + 4
    assert len(shortform_prefix(long, init, 449)) == 1 + 226 + 4   # Python's floor division: -449 // 2 - 1 = -226
    edge = [sop] + list(range(225))
    assert shortform_prefix(edge, init) == edge + init


def checksum_host(buf: bytes) -> int:
    """cbw_checksum restated on the host (kws_kernels.hip, content checksum): splitmix64 of every 8-byte half of each
    16-byte word plus C (2i + 1) / C (2i + 2), wrapping sum; the < 16 tail bytes as one last word pair (bytes 0-7 and
    8-15, each with its own position constant)."""
    M = (1 << 64) - 1
    C = 0x9e3779b97f4a7c15

    def mix(z):
        z &= M
        z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M
        z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M
        return z ^ (z >> 31)
    n16 = len(buf) // 16
    w = np.frombuffer(buf[:n16 * 16], dtype="<u8")
    s = 0
    for i in range(n16):
        s += mix(int(w[2 * i]) + C * (2 * i + 1)) + mix(int(w[2 * i + 1]) + C * (2 * i + 2))
    tail = buf[n16 * 16:]
    if tail:
        t = [0, 0]
        for b, v in enumerate(tail):
            t[b >> 3] |= v << (8 * (b & 7))
        s += mix(t[0] + C * (2 * n16 + 1) + len(tail)) + mix(t[1] + C * (2 * n16 + 2) + len(tail))
    return s & M


def test_checksum_host_restatement_properties():
    """The host restatement the GPU test pins cbw_checksum to: position-dependent (swapping two words changes it),
    every byte matters, the tail counts."""
    rng = np.random.default_rng(0)
    b = bytearray(rng.integers(0, 256, 4 * 16 + 5, dtype=np.uint8).tobytes())
    a = checksum_host(bytes(b))
    sw = bytes(b[16:32] + b[:16] + b[32:])
    assert checksum_host(sw) != a
    for pos in (0, 17, 63, 64, 68):
        c = bytearray(b)
        c[pos] ^= 1
        assert checksum_host(bytes(c)) != a
    assert checksum_host(bytes(b) + b"\x00") != a
    # a tail element flipping in the second half of the tail (bytes 8-15) must not fold onto bytes 0-7
    t = bytearray(16 + 12)
    t[16 + 2] = 0x80
    u = bytearray(t)
    u[16 + 10] = 0x80          # same bit position as byte 2, eight bytes later
    assert checksum_host(bytes(u)) != checksum_host(bytes(t))


def test_generate_rejects_what_it_does_not_restate():
    """PBAWhisper.generate keeps the reference's parameters (pba_whisper.py:17-43) and raises for those it does not
    restate instead of dropping them silently (VERDICT r04 missing 2): a caller's logits_processor /
    stopping_criteria / prefix_allowed_tokens_fn / generation_config, a non-default num_segment_frames or
    time_precision -> NotImplementedError; an unknown keyword -> TypeError; 4.37.2's _set_language_and_task ValueError
    for a language on an English-only call; the short-form ModelOutput slice (return_dict_in_generate=True, or
    return_token_timestamps=True which forces it, pba_whisper.py:338) -> TypeError; return_token_timestamps without the
    checkpoint's alignment_heads -> 4.37.2 _set_num_frames' ValueError.  All raise before any GPU work."""
    import torch
    from cbw import synth
    from model.pba_whisper import PBAWhisper
    sd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict("micro", seed=0).items()}
    sd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict("micro", seed=0).items()})
    w = PBAWhisper(synth.WHISPER_CONFIGS["micro"], synth.WHISPER_DECODERS["micro"], sd)
    feats = torch.zeros((1, synth.WHISPER_CONFIGS["micro"][0], 3000))
    for kw in ({"logits_processor": [lambda ids, s: s]}, {"stopping_criteria": [object()]},
               {"prefix_allowed_tokens_fn": lambda b, ids: [1]}, {"generation_config": object()},
               {"num_segment_frames": 1500}, {"time_precision": 0.01}):
        with pytest.raises(NotImplementedError):
            w.generate(feats, language="en", **kw)
    with pytest.raises(ValueError, match="alignment_heads"):
        w.generate(feats, language="en", return_token_timestamps=True)
    wa = PBAWhisper(synth.WHISPER_CONFIGS["micro"], synth.WHISPER_DECODERS["micro"], sd, alignment_heads=[[1, 0]])
    with pytest.raises(TypeError):
        wa.generate(feats, language="en", return_token_timestamps=True)
    with pytest.raises(TypeError):
        w.generate(feats, language="en", top_p=0.9)
    with pytest.raises(ValueError):
        w.generate(feats, language="en", is_multilingual=False)
    with pytest.raises(TypeError):
        w.generate(feats, language="en", return_dict_in_generate=True)
    with pytest.raises(ValueError):
        w.generate(feats, language="en", prompt_ids=torch.tensor([1, 2]))


def test_generate_control_argument_checks():
    """The restated generation controls keep transformers 4.37.2's argument checks and raise
    NotImplementedError for the combinations not restated -- all before any GPU work: num_return_sequences > 1 with
    greedy (ValueError), above num_beams (ValueError), in long-form (NotImplementedError); a non-positive
    repetition_penalty / negative no_repeat_ngram_size (ValueError); either with timestamps, sampling or long-form
    (NotImplementedError); a non-positive max_length (ValueError)."""
    import torch
    from cbw import synth
    from model.pba_whisper import PBAWhisper
    sd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict("micro", seed=0).items()}
    sd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict("micro", seed=0).items()})
    w = PBAWhisper(synth.WHISPER_CONFIGS["micro"], synth.WHISPER_DECODERS["micro"], sd)
    short = torch.zeros((1, synth.WHISPER_CONFIGS["micro"][0], 3000))
    long = torch.zeros((1, synth.WHISPER_CONFIGS["micro"][0], 4000))
    with pytest.raises(ValueError, match="greedy"):
        w.generate(short, language="en", num_return_sequences=2)
    with pytest.raises(ValueError, match="smaller or equal"):
        w.generate(short, language="en", num_beams=2, num_return_sequences=3)
    with pytest.raises(NotImplementedError):
        w.generate(long, language="en", num_beams=3, num_return_sequences=2, return_timestamps=True)
    with pytest.raises(ValueError):
        w.generate(short, language="en", repetition_penalty=0.0)
    with pytest.raises(ValueError):
        w.generate(short, language="en", no_repeat_ngram_size=-1)
    for kw in ({"return_timestamps": True}, {"do_sample": True, "temperature": 0.7}):
        with pytest.raises(NotImplementedError):
            w.generate(short, language="en", repetition_penalty=1.3, **kw)
    with pytest.raises(NotImplementedError):
        w.generate(long, language="en", no_repeat_ngram_size=2, return_timestamps=True)
    with pytest.raises(ValueError):
        w.generate(short, language="en", max_length=0)
    assert w._controls == {}   # reset after a raising call


class _GenOut(dict):
    """generate's ModelOutput as transformers' _extract_token_timestamps reads it (attribute access, `in`)."""
    __getattr__ = dict.__getitem__


def test_dtw_matches_transformers():
    """cbw_dtw (libcbw host code, the token timestamps' warping) against transformers' _dynamic_time_warping: the same
    path on random cost matrices and on integer-valued ones (ties everywhere: the comparison order decides)."""
    from transformers.models.whisper.generation_whisper import _dynamic_time_warping
    from cbw.token_timestamps import dtw
    rng = np.random.default_rng(3)
    for shape in [(1, 1), (1, 9), (7, 1), (5, 40), (23, 300), (60, 750)]:
        for m in (rng.standard_normal(shape), rng.integers(-2, 3, shape).astype(np.float64)):
            ti, tj = dtw(m)
            ri, rj = _dynamic_time_warping(m)
            assert np.array_equal(ti, ri) and np.array_equal(tj, rj), shape


def test_token_timestamps_match_transformers():
    """cbw.token_timestamps.extract_token_timestamps (variant "5.x") against transformers 5.15's
    _extract_token_timestamps on the same alignment-head weights (random probabilities over 1500 frames, 2 layers x 3
    heads, 3 alignment heads): identical timestamps with and without num_frames cropping and decoder input ids; the
    median filter alone matches too.  Variant "4.37" (the pinned version's row handling, restated) keeps
    timestamps[0] = 0 and one jump time per decoder position."""
    import types
    import torch
    from transformers.models.whisper.generation_whisper import WhisperGenerationMixin, _median_filter
    from cbw.token_timestamps import extract_token_timestamps, median_filter
    g = torch.Generator().manual_seed(0)
    heads = [[0, 1], [1, 0], [1, 2]]
    for T, k, nf in [(12, 4, None), (30, 4, 3000), (9, 1, 1200), (5, 4, None)]:
        ca = [torch.softmax(torch.randn((1, 3, T, 1500), generator=g) * 3, -1) for _ in range(2)]
        out = _GenOut(cross_attentions=(tuple(ca),), sequences=torch.zeros((1, T + 1), dtype=torch.long))
        fake = types.SimpleNamespace(config=types.SimpleNamespace(decoder_layers=2, median_filter_width=7))
        ref = WhisperGenerationMixin._extract_token_timestamps(fake, out, heads, num_frames=nf, num_input_ids=k)[0]
        w = torch.stack([ca[l][0, h] for l, h in heads])
        ours = extract_token_timestamps(w, 7, 0.02, nf, "5.x", k)
        assert torch.equal(ours, ref.float()), (T, k, nf)
        t437 = extract_token_timestamps(w, 7, 0.02, nf, "4.37")
        assert t437.shape == (T + 1,) and t437[0] == 0 and bool((t437[1:].diff() >= 0).all())
    x = torch.randn((3, 11, 40), generator=g)
    assert torch.equal(median_filter(x, 7), _median_filter(x, 7))
