"""GPU parity of the efficient_kws hot path through the C ABI (libcbw) against the
golden vectors of the reference modules and the numpy oracle.

Tolerances (bf16 operands, fp32 accumulation over a 53-conv ResNet-50; the
reference is fp32): logits within 2e-2 of max|logit|, probabilities within 3e-2,
similarity maps within 1e-2 absolute (|sim| <= 1); spotted-keyword indices
identical for every pair whose reference probability is farther than 0.03 from
the threshold (pairs inside the band are reported, SURVEY.md §7 hard part 3).
"""
import os

import numpy as np
import pytest
import torch

from cbw import synth
from golden_cases import KWS_CASES, THRESHOLDS

pytestmark = pytest.mark.gpu

LOGIT_RTOL = 2e-2
PROB_ATOL = 3e-2
SIM_ATOL = 1e-2
BAND = 0.03


def dev():
    return torch.device("cuda:0")


def run_engine(hp, sd, b, features=True, chunk=None):
    from cbw.kws import KwsEngine
    eng = KwsEngine(hp, sd)
    d = eng.device
    pk, pkm = eng.project(torch.from_numpy(b["kwd"]).to(d), torch.from_numpy(b["kwd_mask"]).to(d))
    pu, pum = eng.project(torch.from_numpy(b["utt"]).to(d), torch.from_numpy(b["utt_mask"]).to(d))
    out = eng.score(pu[0], pum[0], pk, pkm, features=features, chunk=chunk)
    return eng, out


def assert_decisions(p_gpu, p_ref, thr):
    sure = np.abs(p_ref - thr) > BAND
    got = p_gpu >= thr
    want = p_ref >= thr
    bad = np.nonzero(sure & (got != want))[0]
    assert bad.size == 0, f"decision flips outside the ±{BAND} band at {bad.tolist()}"


@pytest.mark.parametrize("name", list(KWS_CASES))
def test_golden_parity(name, golden_dir):
    from cbw.kws import spot
    hp, bk = KWS_CASES[name]
    g = np.load(os.path.join(golden_dir, f"kws_{name}.npz"))
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
    eng, (logits, feats) = run_engine(hp, sd, b, features=True)
    lg = logits.cpu().numpy()
    np.testing.assert_allclose(lg, g["logits"], atol=LOGIT_RTOL * np.abs(g["logits"]).max())
    f = feats.cpu().numpy()
    assert tuple(f.shape) == tuple(g["feat_shape"])
    np.testing.assert_allclose(f[:, :, ::7, ::11], g["feat_sub"], atol=SIM_ATOL)
    ghost = torch.from_numpy(b["ghost_mask"]).to(eng.device)
    for t in THRESHOLDS:
        p, idx = spot(logits, ghost, t)
        p = p.cpu().numpy()
        np.testing.assert_allclose(p, g["probs"], atol=PROB_ATOL)
        assert_decisions(p, g["probs"], t)
        assert set(idx.cpu().tolist()) == set(np.nonzero(p >= t)[0].tolist())
        assert idx.cpu().tolist() == sorted(idx.cpu().tolist())
    # ghost keywords are never spotted (prob * 0)
    for gi in np.nonzero(b["ghost_mask"] == 0)[0]:
        assert p[gi] == 0.0


def test_kwsmodel_forward_api_matches_golden(golden_dir):
    """The reference-shaped API: efficient_kws.model.KWSModel.forward -> KWSOutput."""
    from efficient_kws.model import KWSModel
    hp, bk = KWS_CASES["LEF"]
    g = np.load(os.path.join(golden_dir, "kws_LEF.npz"))
    m = KWSModel(features_size=(150, 1500), **hp)
    m.load_state_dict(synth.synth_kws_state_dict(seed=0, **hp))
    b = synth.synth_kws_batch(n_layers=3, D=hp["embedding_dim"], **bk)
    out = m.forward(kwd_features=torch.from_numpy(b["kwd"]), utt_features=torch.from_numpy(b["utt"]),
                    labels=torch.zeros(len(b["kwd"]), dtype=torch.long),
                    kwd_mask=torch.from_numpy(b["kwd_mask"]), utt_mask=torch.from_numpy(b["utt_mask"]))
    np.testing.assert_allclose(out.logits.cpu().numpy(), g["logits"], atol=LOGIT_RTOL * np.abs(g["logits"]).max())
    assert tuple(out.features.shape) == tuple(g["feat_shape"])
    assert out.loss is not None and out.loss_alt["loss_resnet"] is out.loss
    # pre-pooled masks (what the fixed reference receives) give the same result
    pool = torch.nn.MaxPool1d(3, 2, 1)
    out2 = m.forward(kwd_features=torch.from_numpy(b["kwd"]), utt_features=torch.from_numpy(b["utt"]),
                     kwd_mask=pool(torch.from_numpy(b["kwd_mask"])), utt_mask=pool(torch.from_numpy(b["utt_mask"])))
    np.testing.assert_array_equal(out.logits.cpu().numpy(), out2.logits.cpu().numpy())


@pytest.mark.parametrize("D,variant", [(1280, "LEF"), (768, "LE"), (384, "L")])
def test_baseline_config_shapes_vs_oracle(D, variant):
    """C3 (large-v3 LEF, D=1280), C2 (small LE, D=768) and C1 (tiny.en L, D=384)
    shapes at full features_size (150, 1500) against the numpy oracle."""
    import oracle.kws as okws
    hp = dict(n_layers=3, embedding_dim=D, learn_features=variant != "L", proj_mlp=variant != "L",
              frames_conv=variant == "LEF", proj_mlp_units=64)
    sd = synth.synth_kws_state_dict(seed=2, **hp)
    b = synth.synth_kws_batch(seed=21, K=3, n_layers=3, D=D, plant=(0,), utt_len=1400)
    _, logits = run_engine(hp, sd, b, features=False)
    ref, _ = okws.kws_forward(sd, hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], return_features=False)
    np.testing.assert_allclose(logits.cpu().numpy(), ref, atol=LOGIT_RTOL * np.abs(ref).max())


@pytest.mark.parametrize("version", ["resnet-34", "resnet-18"])
def test_basic_block_resnets_vs_oracle(version):
    """The basic-block classifiers (`resnet.py:51-58` with `version` 34 / 18: HF ResNetBasicLayer stacks [3, 4, 6, 3]
    / [2, 2, 2, 2]) at LEF widths against the numpy oracle, incl. the spot decisions outside the bf16 band."""
    import oracle.kws as okws
    from cbw.kws import spot
    hp = dict(n_layers=3, embedding_dim=256, learn_features=True, proj_mlp=True, frames_conv=True,
              proj_mlp_units=64, resnet_version=version)
    sd = synth.synth_kws_state_dict(seed=5, **hp)
    b = synth.synth_kws_batch(seed=31, K=6, n_layers=3, D=256, plant=(0, 3), utt_len=1300)
    eng, logits = run_engine(hp, sd, b, features=False)
    ref, _ = okws.kws_forward(sd, hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], return_features=False)
    np.testing.assert_allclose(logits.cpu().numpy(), ref, atol=LOGIT_RTOL * np.abs(ref).max())
    ref_p = np.exp(ref[:, 1]) / np.exp(ref).sum(1) * b["ghost_mask"]
    p, _ = spot(logits, torch.from_numpy(b["ghost_mask"]).to(eng.device), 0.5)
    assert_decisions(p.cpu().numpy(), ref_p, 0.5)


def test_pool_unroll_bit_exact(monkeypatch):
    """The pool + classifier kernel with 1, 4 or 8 pixels' loads in flight per lane (CBW_POOL_UNROLL) sums the
    pixels in the same order: identical logits (LEF, ragged keywords, a partial last unroll group: 66 pixels)."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
    b = synth.synth_kws_batch(seed=9, K=40, n_layers=3, D=128, Tu=1400, plant=(1, 5), utt_len=1100)   # 3 x 22 px
    d = eng.device
    pk, pkm = eng.project(torch.from_numpy(b["kwd"]).to(d), torch.from_numpy(b["kwd_mask"]).to(d))
    pu, pum = eng.project(torch.from_numpy(b["utt"]).to(d), torch.from_numpy(b["utt_mask"]).to(d))
    outs = []
    for u in ("1", "4", "8"):
        monkeypatch.setenv("CBW_POOL_UNROLL", u)
        outs.append(eng.score(pu[0], pum[0], pk, pkm))
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=0)
    torch.testing.assert_close(outs[0], outs[2], rtol=0, atol=0)


def test_chunking_and_order_invariance():
    """Size-independent properties at many keywords: results do not depend on the
    chunk size (bit-identical), on keyword order (permutation equivariance, bit-identical)
    and duplicated keywords score identically."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    eng = KwsEngine(hp, sd)
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(0)
    K = 300
    kwd = torch.randn((K, 3, 75, 64), generator=g, device=d)
    kwd = (kwd / kwd.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    kwd[7] = kwd[3]
    km = torch.ones((K, 3, 75), device=d)
    km[5, :, 40:] = 0
    utt = torch.randn((3, 750, 64), generator=g, device=d)
    utt = (utt / utt.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    um = torch.ones((3, 750), device=d)
    a = eng.score(utt, um, kwd, km, chunk=300)
    b = eng.score(utt, um, kwd, km, chunk=37)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    perm = torch.randperm(K, generator=torch.Generator().manual_seed(1)).to(d)
    c = eng.score(utt, um, kwd[perm].contiguous(), km[perm].contiguous(), chunk=64)
    torch.testing.assert_close(c, a[perm], rtol=0, atol=0)
    torch.testing.assert_close(a[7], a[3], rtol=0, atol=0)
    assert torch.isfinite(a).all()


def test_classify_matches_score_path():
    """Resnet.forward on caller-built NCHW maps == the fused score path on the same maps."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
    b = synth.synth_kws_batch(seed=4, K=5, n_layers=3, D=128, plant=(2,), utt_len=900)
    d = eng.device
    pk, pkm = eng.project(torch.from_numpy(b["kwd"]).to(d), torch.from_numpy(b["kwd_mask"]).to(d))
    pu, pum = eng.project(torch.from_numpy(b["utt"]).to(d), torch.from_numpy(b["utt_mask"]).to(d))
    logits, feats = eng.score(pu[0], pum[0], pk, pkm, features=True)
    logits2 = eng.classify(feats)
    torch.testing.assert_close(logits, logits2, rtol=0, atol=0)
    # the Resnet module on its own (classifier-only handle: no projector parameters at all)
    from efficient_kws.resnet import Resnet
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    net = Resnet(3, 2, "resnet-50")
    net.load_state_dict({k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")})
    torch.testing.assert_close(net(feats), logits2, rtol=0, atol=0)


def test_spot_kernel_exact():
    """Ordered compaction, ghost masking, ties and the argmax rule, vs numpy (exact)."""
    from cbw.kws import spot
    rng = np.random.default_rng(0)
    K = 5000
    lg = rng.standard_normal((K, 2)).astype(np.float32)
    lg[10] = [0.25, 0.25]          # tie: prob 0.5, argmax -> class 0
    ghost = (rng.random(K) > 0.1).astype(np.float32)
    t = torch.from_numpy(lg).to(dev())
    p, idx = spot(t, torch.from_numpy(ghost).to(dev()), 0.5)
    p_np = (1.0 / (1.0 + np.exp(lg[:, 0].astype(np.float64) - lg[:, 1]))) * ghost
    np.testing.assert_allclose(p.cpu().numpy(), p_np, atol=1e-6)
    want = np.nonzero(p.cpu().numpy() >= 0.5)[0]
    assert idx.cpu().numpy().tolist() == want.tolist()
    assert 10 in want.tolist() or ghost[10] == 0
    _, idx2 = spot(t, None, 0.5, mode="argmax")
    assert idx2.cpu().numpy().tolist() == np.nonzero(lg[:, 1] > lg[:, 0])[0].tolist()
    _, idx3 = spot(t[:0], None, 0.5)
    assert idx3.numel() == 0


def test_edge_cases_and_errors():
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp))
    d = eng.device
    utt = torch.zeros((3, 750, 64), dtype=torch.bfloat16, device=d)
    um = torch.ones((3, 750), device=d)
    # K = 0 -> empty logits, no launch
    out = eng.score(utt, um, torch.zeros((0, 3, 75, 64), dtype=torch.bfloat16, device=d),
                    torch.zeros((0, 3, 75), device=d))
    assert out.shape == (0, 2)
    # all-zero features (ghost keyword, silent utterance): finite logits
    out = eng.score(utt, um, torch.zeros((2, 3, 75, 64), dtype=torch.bfloat16, device=d),
                    torch.ones((2, 3, 75), device=d))
    assert torch.isfinite(out).all()
    torch.testing.assert_close(out[0], out[1], rtol=0, atol=0)
    # wrong layer count / dims raise ValueError (the reference raises in HF ResNet, modeling_resnet.py:86-91)
    with pytest.raises(ValueError):
        eng.project(torch.zeros((1, 2, 10, 128), device=d), torch.ones((1, 2, 10), device=d))
    with pytest.raises(ValueError):
        eng.classify(torch.zeros((1, 2, 75, 750), device=d))
    # shortest keyword (8 frames -> 4 pooled) and maximum lengths
    b = synth.synth_kws_batch(seed=9, K=2, n_layers=3, D=128, min_len=8)
    b["kwd_mask"][1, :, 8:] = 0
    b["kwd"][1, :, 8:] = 0
    pk, pkm = eng.project(torch.from_numpy(b["kwd"]).to(d), torch.from_numpy(b["kwd_mask"]).to(d))
    import oracle.kws as okws
    np.testing.assert_array_equal(pkm.cpu().numpy(), okws.pool_mask(b["kwd_mask"]))
    assert pkm[1, 0].sum().item() == 5.0 and pkm[0, 0].sum().item() == 75.0   # frames 0..7 -> pooled 0..4


def test_shortcut_fusion_matches_separate_shortcut(monkeypatch):
    """The expand+shortcut K-concatenated conv equals the separate shortcut conv + residual
    (bf16 rounding of the shortcut tensor is the only difference)."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    b = synth.synth_kws_batch(seed=6, K=6, n_layers=3, D=128, plant=(1,), utt_len=1200)
    _, fused = run_engine(hp, sd, b, features=False)
    monkeypatch.setenv("CBW_NO_SC_FUSION", "1")
    _, sep = run_engine(hp, sd, b, features=False)
    f, s = fused.cpu().numpy(), sep.cpu().numpy()
    np.testing.assert_allclose(f, s, atol=1e-2 * np.abs(s).max())


@pytest.mark.parametrize("Tk,Tu", [(75, 750), (150, 1500), (23, 61)])
def test_stem_pool_fusion_matches_separate_kernels(monkeypatch, Tk, Tu):
    """The fused stem conv + maxpool kernel equals the separate stem conv and maxpool kernels
    on the classifier logits (LEF maps, LE/L maps with two row tiles, odd sizes with partial
    tiles).  Both paths round the stem output to bf16 before the max."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    eng = KwsEngine(hp, sd)
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(11)
    maps = torch.rand((5, 3, Tk, Tu), generator=g, device=d) * 2 - 1
    maps[:, :, :, Tu // 2:] *= 0.1
    fused = eng.classify(maps, chunk=3)
    monkeypatch.setenv("CBW_NO_STEM_FUSION", "1")
    sep = eng.classify(maps, chunk=3)
    f, s = fused.cpu().numpy(), sep.cpu().numpy()
    assert np.isfinite(f).all()
    np.testing.assert_allclose(f, s, atol=1e-3 * max(1.0, np.abs(s).max()))


@pytest.mark.parametrize("Tk,Tu", [(75, 750), (150, 1500), (23, 61), (41, 97)])
def test_stem_pool_v2_bit_identical(monkeypatch, Tk, Tu):
    """The stem + max-pool kernel's V2 epilogue and pool (ReLU on the rounded bf16 pairs, no sign masks, two pooled
    rows per item) against V1 (CBW_STEM_V1=1): the pooled stem output and hence the logits bit-identical -- LEF maps,
    two row tiles, partial tiles, odd pooled row counts (the last pair holds one row)."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=3, **hp))
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(21)
    maps = torch.rand((7, 3, Tk, Tu), generator=g, device=d) * 2 - 1
    maps[:, :, :, Tu // 3:] *= 0.05
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("CBW_STEM_V1", mode)
        out[mode] = eng.classify(maps, chunk=4)
    torch.cuda.synchronize()
    assert torch.isfinite(out["0"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("Tk,Tu", [(75, 750), (23, 61), (41, 97), (9, 40)])
def test_stem_pool_v3_bit_identical(monkeypatch, Tk, Tu):
    """Round 6's stem + max-pool kernel (per-launch index tables, masks only on the first fragment and the
    column-edge tiles, three pooled rows per pool item; full-height tiles) against V2 (CBW_STEM_V3=0): logits
    bit-identical -- LEF maps, partial column tiles, pooled row counts that are not multiples of 3."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=4, **hp))
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(22)
    maps = torch.rand((7, 3, Tk, Tu), generator=g, device=d) * 2 - 1
    maps[:, :, :, Tu // 3:] *= 0.05
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CBW_STEM_V3", mode)
        out[mode] = eng.classify(maps, chunk=4)
    torch.cuda.synchronize()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("Tk,Tu", [(75, 750), (150, 1500), (23, 61)])
def test_bottleneck_fusion_matches_three_convs(monkeypatch, Tk, Tu):
    """The fused stage-1 bottleneck kernels (reduce + 3x3 + expand + residual in one launch,
    intermediates in LDS) vs the three-conv path and both vs the torch-fp32 oracle (ResNet-50 of
    oracle/torch_ref.py); LEF maps (precomputed-mask tiles + edge tiles), LE maps (two row tiles of
    19), odd sizes (partial tiles).  Same bf16 rounding points as the three-conv path; the fused
    kernels seed the accumulators with the bias (the conv path adds it after the K loop), so the two
    agree to bf16 rounding-order noise (5e-3 of max|logit|; the diagnostic build -DBT_BIAS_EPI=1,
    bias added last, agrees within 1e-3)."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    sd = synth.synth_kws_state_dict(seed=1, **hp)
    eng = KwsEngine(hp, sd)
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(12)
    maps = torch.rand((5, 3, Tk, Tu), generator=g, device=d) * 2 - 1
    fused = eng.classify(maps, chunk=3)
    monkeypatch.setenv("CBW_NO_BOTTLENECK_FUSION", "1")
    sep = eng.classify(maps, chunk=3)
    f, s = fused.cpu().numpy(), sep.cpu().numpy()
    assert np.isfinite(f).all()
    from oracle import torch_ref
    ref = torch_ref.resnet_forward({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, maps.cpu()).numpy()
    scale = np.abs(ref).max()
    np.testing.assert_allclose(s, ref, atol=LOGIT_RTOL * scale)
    np.testing.assert_allclose(f, ref, atol=LOGIT_RTOL * scale)
    np.testing.assert_allclose(f, s, atol=5e-3 * max(1.0, np.abs(s).max()))


@pytest.mark.parametrize("N,H,W,Cin,Cout,k,s", [(625, 10, 94, 256, 256, 3, 2), (625, 3, 24, 2048, 512, 1, 1),
                                                 (256, 10, 94, 64, 256, 3, 1), (300, 10, 94, 512, 256, 1, 1),
                                                 (625, 19, 188, 128, 128, 3, 2), (625, 10, 94, 128, 128, 3, 1),
                                                 (301, 10, 94, 128, 128, 3, 1)])
def test_p8_conv_vs_torch(N, H, W, Cin, Cout, k, s):
    """conv_igemm_p8 (the 8-phase kernel cbw_conv2d takes at these shapes: 256 x 256 tiles, and 512 x 128 tiles at
    Cout 128 -- the stage-2 3x3s, stride 2 and 1, and a partial last tile at 301 pairs) against torch fp32 on 8 pairs:
    K-tiles 8 (1x1, 512 channels: the counted waits of the last K-tiles), 9 (3x3 over 64), 18 (3x3 over 128), 32, 36
    (3x3 stride 2); an all-NaN canvas checks that every output element is written."""
    from cbw import _lib
    lib = _lib.load()
    d = torch.device("cuda:0")
    g = torch.Generator(device=d)
    g.manual_seed(11)
    x = torch.randn((N, H, W, Cin), generator=g, device=d).to(torch.bfloat16)
    w = (torch.randn((Cout, k, k, Cin), generator=g, device=d) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=d)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    y = torch.full((N, Ho, Wo, Cout), float("nan"), device=d).to(torch.bfloat16)
    _lib.check(lib.cbw_conv2d(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(), N, H, W, Cin, Cout, k, k,
                              s, s, k // 2, k // 2, 1, _lib.stream_handle()), "cbw_conv2d")
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    ref = torch.nn.functional.conv2d(x[:8].permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), b,
                                     stride=s, padding=k // 2).relu().permute(0, 2, 3, 1)
    torch.testing.assert_close(y[:8].float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("N", [625, 300])
def test_conv1x1_dual_source_vs_torch(N):
    """The folded expand + shortcut conv (cbw_conv1x1_dual: K-tiles past Cin read the stride-2 shortcut input) at the
    stage-3 first block's shape, against torch fp32 on 8 pairs; every output element written."""
    from cbw import _lib
    lib = _lib.load()
    d = torch.device("cuda:0")
    g = torch.Generator(device=d)
    g.manual_seed(17)
    H, W, Cin, H2, W2, Cin2, Cout = 5, 47, 256, 10, 94, 512, 1024
    x = torch.randn((N, H, W, Cin), generator=g, device=d).to(torch.bfloat16)
    x2 = torch.randn((N, H2, W2, Cin2), generator=g, device=d).to(torch.bfloat16)
    w = (torch.randn((Cout, Cin + Cin2), generator=g, device=d) / (Cin + Cin2) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=d)
    y = torch.full((N, H, W, Cout), float("nan"), device=d).to(torch.bfloat16)
    _lib.check(lib.cbw_conv1x1_dual(x.data_ptr(), x2.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(),
                                    N, H, W, Cin, H2, W2, Cin2, 2, Cout, 1, _lib.stream_handle()), "cbw_conv1x1_dual")
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    xs = torch.cat([x[:8].float(), x2[:8, ::2, ::2].float()], dim=-1)
    ref = (xs @ w.float().t() + b).relu()
    torch.testing.assert_close(y[:8].float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("K", [400, 130])
def test_compensated_tier_on_p8_bit_identical(monkeypatch, K):
    """The compensated tier's convs on conv_igemm_p8 (CBW_P8_TIER: the expand convs with the [hi | lo] / fp32 residual
    and the fp32-output shortcuts on p8's residual epilogue, deep-K stage-4 convs from half a round of 256 x 256
    tiles) compute every output exactly as the tile kernels do: x3 logits bit-identical with the knob on and off, at
    ~400 band pairs (stage 4: 226 tiles) and at 130 (fewer tiles than half a round: the tile kernels stay), and
    within 1e-3 of the fp32 tier's."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=2, **hp))
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(5)
    kwd = torch.randn((K, 3, 150, 128), generator=g, device=d)
    km = torch.ones((K, 3, 150), device=d)
    km[::7, :, 90:] = 0
    utt = torch.randn((1, 3, 1500, 128), generator=g, device=d)
    um = torch.ones((1, 3, 1500), device=d)
    pk, pkm = eng.project(kwd, km)
    pk32, _ = eng.project_f32(kwd, km)
    pu32, pum = eng.project_f32(utt, um)
    sel = torch.arange(K, device=d)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CBW_P8_TIER", mode)
        out[mode] = eng.rescore(pu32, pum, pk32, pkm, torch.zeros((K, 2), device=d), sel, tier="x3")
    f32 = eng.rescore(pu32, pum, pk32, pkm, torch.zeros((K, 2), device=d), sel[:16], tier="fp32")
    torch.cuda.synchronize()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])
    torch.testing.assert_close(out["1"][:16], f32[:16], rtol=0, atol=1e-3)


@pytest.mark.parametrize("tier", ["bf16", "x3"])
def test_p8_n128_bit_identical(monkeypatch, tier):
    """The stage-2 3x3 convs (Cout 128) on conv_igemm_p8's 512 x 128 tiles compute every output exactly as the 4-wave
    128 x 128 kernel does (same K order, fp32 accumulation, epilogue): the classifier's bf16 logits (150 LEF pairs:
    276 tiles per 3x3) and the compensated tier's x3 logits (400 pairs, [hi | lo] inputs, split outputs) are
    bit-identical with CBW_P8_N128 on and off."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=3, **hp))
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(23)
    out = {}
    if tier == "bf16":
        maps = torch.rand((150, 3, 75, 750), generator=g, device=d) * 2 - 1
        for mode in ("0", "1"):
            monkeypatch.setenv("CBW_P8_N128", mode)
            out[mode] = eng.classify(maps, chunk=150)
    else:
        K = 400
        kwd = torch.randn((K, 3, 150, 128), generator=g, device=d)
        km = torch.ones((K, 3, 150), device=d)
        utt = torch.randn((1, 3, 1500, 128), generator=g, device=d)
        um = torch.ones((1, 3, 1500), device=d)
        pk32, pkm = eng.project_f32(kwd, km)
        pu32, pum = eng.project_f32(utt, um)
        sel = torch.arange(K, device=d)
        for mode in ("0", "1"):
            monkeypatch.setenv("CBW_P8_N128", mode)
            out[mode] = eng.rescore(pu32, pum, pk32, pkm, torch.zeros((K, 2), device=d), sel, tier="x3")
    torch.cuda.synchronize()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"]), (out["0"] - out["1"]).abs().max().item()


@pytest.mark.parametrize("Tk,Tu,K", [(75, 750, 40), (73, 741, 9), (75, 750, 1)])
def test_bottleneck_ring_bit_identical(monkeypatch, Tk, Tu, K):
    """The column-ring stage-1 identity block (bottleneck.hip bottleneck_ring_kernel: LEF-shaped maps, H = 19, ring of
    input columns shared by consecutive 4-column tiles) computes every output element exactly as bottleneck_kernel<256>
    does (same operands, k-step order, bias seeding, rounding): the classifier's logits are bit-identical with it on
    and off (CBW_BT_RING=0).  LEF maps (W = 188: 47 whole tiles), W = 186 (a partial last tile), 40 pairs (workgroup
    tile ranges start inside pairs: the ring's cold starts), one pair."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    sd = synth.synth_kws_state_dict(seed=1, **hp)
    eng = KwsEngine(hp, sd)
    g = torch.Generator(device=eng.device)
    g.manual_seed(13)
    maps = torch.rand((K, 3, Tk, Tu), generator=g, device=eng.device) * 2 - 1
    monkeypatch.setenv("CBW_BT_RING", "1")
    ring = eng.classify(maps, chunk=K)
    monkeypatch.setenv("CBW_BT_RING", "0")
    tile = eng.classify(maps, chunk=K)
    torch.cuda.synchronize()
    assert torch.isfinite(ring).all()
    assert torch.equal(ring, tile), (ring - tile).abs().max().item()


@pytest.mark.parametrize("Tk,Tu,K", [(75, 750, 40), (150, 1500, 6), (41, 97, 7), (23, 61, 5)])
def test_stage1_merged_schedule_bit_identical(monkeypatch, Tk, Tu, K):
    """The merged stage-1 schedules (bottleneck.hip: tile t-1's phase E and tile t's phase R in one barrier interval, in
    bottleneck_ring_kernel and in the first block bottleneck_kernel<64>) leave every output as the three-barrier
    schedules compute it: logits bit-identical with CBW_BT_MERGE / CBW_BT64_MERGE on and off.  LEF maps, H = 38 (two
    row tiles per pair), non-LEF H = 11 and H = 6 (ragged last tiles)."""
    from cbw.kws import KwsEngine
    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True)
    eng = KwsEngine(hp, synth.synth_kws_state_dict(seed=10, **hp))
    g = torch.Generator(device=eng.device)
    g.manual_seed(47)
    maps = torch.rand((K, 3, Tk, Tu), generator=g, device=eng.device) * 2 - 1
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CBW_BT_MERGE", mode)
        monkeypatch.setenv("CBW_BT64_MERGE", mode)
        out[mode] = eng.classify(maps, chunk=K)
    torch.cuda.synchronize()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"]), (out["0"] - out["1"]).abs().max().item()


def test_cnn12_score_resized_vs_reference_golden(golden_dir):
    """CB-Whisper's own spotter on the GPU (similarity GEMM + bilinear resize + 12-channel
    ResNet-50 in one libcbw call) vs the reference model.model.KWSModel on the same inputs
    (tests/golden/cnn12.npz); ragged keywords incl. 1 frame and > 150 frames."""
    import sys as _s
    _s.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import cnn12_inputs
    from model.model import KWSModel as CBKWSModel
    g = np.load(os.path.join(golden_dir, "cnn12.npz"))
    sd = synth.synth_kws_state_dict(seed=3, n_layers=12, embedding_dim=128, learn_features=False, proj_mlp=False)
    m = CBKWSModel()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    utt, kwd = cnn12_inputs()
    d = torch.device("cuda:0")
    logits = m.score_keywords(torch.from_numpy(utt).to(d), [torch.from_numpy(k).to(d) for k in kwd]).cpu().numpy()
    ref = g["logits"]
    np.testing.assert_allclose(logits, ref, atol=LOGIT_RTOL * np.abs(ref).max())
    # chunking does not change results (bit-identical)
    eng = m.engine(128)
    a = eng.score_resized(torch.from_numpy(utt).to(d), [torch.from_numpy(k) for k in kwd], chunk=2)
    b = eng.score_resized(torch.from_numpy(utt).to(d), [torch.from_numpy(k) for k in kwd], chunk=5)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    # forward() on caller-built maps (NCHW, 12 channels) = the same classifier
    u = torch.from_numpy(utt).to(d)
    maps = torch.stack([torch.nn.functional.interpolate(torch.matmul(torch.from_numpy(k).to(d), u.transpose(1, 2))[None],
                                                        size=(150, 750), mode="bilinear", align_corners=False)[0]
                        for k in kwd])
    out = m.forward(maps)
    np.testing.assert_allclose(out.logits.cpu().numpy(), ref, atol=LOGIT_RTOL * np.abs(ref).max())
    assert m.spot_keywords(u, [torch.from_numpy(k) for k in kwd]) == g["argmax_idx"].tolist()


EXACT_RTOL = 1e-4


@pytest.mark.parametrize("name", list(KWS_CASES))
def test_exact_rescore_matches_reference_fp32(name, golden_dir):
    """fp32 re-scoring (KWSModel.exact_band; cbw_kws_project_f32 + cbw_kws_rescore): with every pair
    re-scored, logits within 1e-4 of max|logit| of the reference's fp32 forward and the spotted indices
    identical to the reference's at every threshold -- no tolerance band."""
    from cbw.kws import spot
    from efficient_kws.model import KWSModel
    hp, bk = KWS_CASES[name]
    g = np.load(os.path.join(golden_dir, f"kws_{name}.npz"))
    m = KWSModel(features_size=(150, 1500), exact_band=1.0, **hp)
    m.load_state_dict(synth.synth_kws_state_dict(seed=0, **hp))
    b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
    out = m.forward(kwd_features=torch.from_numpy(b["kwd"]), utt_features=torch.from_numpy(b["utt"]),
                    kwd_mask=torch.from_numpy(b["kwd_mask"]), utt_mask=torch.from_numpy(b["utt_mask"]),
                    return_features=False)
    lg = out.logits.cpu().numpy()
    err = np.abs(lg - g["logits"]).max() / np.abs(g["logits"]).max()
    print(f"{name}: fp32 re-score max|dlogit|/max|logit| = {err:.2e}")
    assert err < EXACT_RTOL, f"fp32 re-score deviates {err:.2e}"
    ghost = torch.from_numpy(b["ghost_mask"]).to(out.logits.device)
    for t in THRESHOLDS:
        p, idx = spot(out.logits, ghost, t)
        np.testing.assert_allclose(p.cpu().numpy(), g["probs"], atol=1e-5)
        assert idx.cpu().tolist() == g[f"idx_{t}"].tolist()


def test_exact_band_rescores_only_near_threshold():
    """exact_band = 0.2: pairs outside the band keep the bf16 logits bit for bit, pairs inside get the
    fp32 ones; the decisions equal the oracle's (fp64) at the threshold."""
    import oracle.kws as okws
    from efficient_kws.model import KWSModel
    hp, bk = KWS_CASES["LEF"]
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
    args = dict(kwd_features=torch.from_numpy(b["kwd"]), utt_features=torch.from_numpy(b["utt"]),
                kwd_mask=torch.from_numpy(b["kwd_mask"]), utt_mask=torch.from_numpy(b["utt_mask"]),
                return_features=False)
    m0 = KWSModel(features_size=(150, 1500), exact_band=0.0, **hp)
    m0.load_state_dict(sd)
    base = m0.forward(**args).logits.cpu().numpy()
    m1 = KWSModel(features_size=(150, 1500), exact_band=0.2, **hp)
    m1.load_state_dict(sd)
    mixed = m1.forward(**args).logits.cpu().numpy()
    p0 = np.exp(base[:, 1]) / np.exp(base).sum(1)
    inside = np.abs(p0 - 0.5) <= 0.2
    np.testing.assert_array_equal(mixed[~inside], base[~inside])
    ref, _ = okws.kws_forward(sd, hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], return_features=False)
    if inside.any():
        assert np.abs(mixed[inside] - ref[inside]).max() < EXACT_RTOL * np.abs(ref).max()


def test_checksum_matches_host_restatement_and_keys_the_keyword_cache():
    """cbw_checksum (the keyword-database cache key of KWSModel.test_step, kwd_cache="content") equals its host
    restatement (tests/test_host.py::checksum_host) on random byte ranges with tails, changes with any one bit; and
    KWSModel re-projects a database whose content changed at an element a sampled fingerprint would miss, even when
    the write bypasses torch's version counter."""
    from cbw import _lib
    from efficient_kws.model import KWSModel
    from test_host import checksum_host
    lib = _lib.load()
    dev = torch.device("cuda:0")
    ws = torch.empty(int(lib.cbw_checksum_workspace_bytes()), dtype=torch.uint8, device=dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(3)

    def dev_sum(buf):
        t = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy()).to(dev) if buf else torch.empty(16, dtype=torch.uint8, device=dev)
        _lib.check(lib.cbw_checksum(t.data_ptr(), len(buf), out.data_ptr(), ws.data_ptr(), ws.numel(),
                                    _lib.stream_handle()), "cbw_checksum")
        return int(out.cpu().item()) & ((1 << 64) - 1)

    for n in (0, 1, 15, 16, 17, 4096 * 16 + 5, 300_001):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert dev_sum(b) == checksum_host(b), n
        if n:
            c = bytearray(b)
            c[n // 2] ^= 0x10
            assert dev_sum(bytes(c)) != dev_sum(b)
    t = bytearray(16 + 12)     # tail bytes 8-15 no longer fold onto bytes 0-7
    t[18] = 0x80
    u = bytearray(t)
    u[26] = 0x80
    assert dev_sum(bytes(u)) == checksum_host(bytes(u)) and dev_sum(bytes(u)) != dev_sum(bytes(t))

    hp = dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True, exact_band=0.0)
    sd = synth.synth_kws_state_dict(seed=0, **{k: v for k, v in hp.items() if k != "exact_band"})
    b = synth.synth_kws_batch(seed=5, K=6, n_layers=3, D=128, plant=(1,), utt_len=1300)
    kwd = torch.from_numpy(b["kwd"]).to(dev)
    km = torch.from_numpy(b["kwd_mask"]).to(dev)
    batch = {"kwd": [kwd[:3].contiguous(), kwd[3:].contiguous()], "kwd_mask": [km[:3].contiguous(), km[3:].contiguous()],
             "utt": torch.from_numpy(b["utt"][0]).to(dev), "utt_mask": torch.from_numpy(b["utt_mask"][0]).to(dev)}
    m = KWSModel(**hp)
    m.load_state_dict(sd)
    assert m.kwd_cache == "content"
    p0 = m.test_step(batch)["preds"].clone()
    assert torch.equal(m.test_step(batch)["preds"], p0)   # cache hit, same result
    g = batch["kwd"][0]
    v0 = g._version
    g.data[1, 0, 1, 5] += 0.5    # an element a 4096-sample fingerprint of this tensor would not read; no version bump
    assert g._version == v0
    p1 = m.test_step(batch)["preds"]
    fresh = KWSModel(**hp)
    fresh.load_state_dict(sd)
    fresh.kwd_cache = "off"
    torch.testing.assert_close(p1, fresh.test_step(batch)["preds"], rtol=0, atol=0)
