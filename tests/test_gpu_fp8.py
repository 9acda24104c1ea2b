"""The fp8 first tier (conv_fp8.hip, cbw_kws_score_fp8; BASELINE C5 "fp8 MFMA"):

* the operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 the kernel assumes, found with exact integers;
* the e4m3 conversions (OCP e4m3fn, round to nearest even, saturating at 448) against a host encoder;
* the e4m3 conv kernels against a float64 conv of the decoded operands (1x1 / 3x3, stride 1 / 2, residual,
  ReLU, e4m3 and bf16 outputs; the shapes cover the 4-wave tile kernel, the 8-wave schedule (Cout % 256, >= 8
  K-tiles) and the streaming 1x1 kernel (stride 1, Cin 128 / 256 / 512, one and several weight slices)): exact
  products, fp32 accumulation, so within fp32 rounding before the output rounding (bf16: 2^-8 relative; e4m3: one
  e4m3 step);
* the calibrated network against the fp32 network on held-out pairs (error bounded), and the cascade fp8 ->
  bf16 -> compensated -> fp32 reproducing every all-pairs fp32 decision.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def e4m3_table():
    v = np.zeros(256)
    for c in range(256):
        s = -1.0 if c & 0x80 else 1.0
        e, m = (c >> 3) & 15, c & 7
        if e == 15 and m == 7:
            v[c] = np.nan
        elif e == 0:
            v[c] = s * m / 8 * 2.0 ** -6
        else:
            v[c] = s * (1 + m / 8) * 2.0 ** (e - 7)
    return v


TAB = e4m3_table()


def encode(x):
    """nearest e4m3 code (ties to even mantissa), saturating at +-448"""
    x = np.clip(np.asarray(x, np.float64), -448, 448)
    finite = np.where(np.isnan(TAB), np.inf, TAB)
    out = np.zeros(x.shape, np.uint8)
    for i, v in np.ndenumerate(x):
        d = np.abs(finite - v)
        best = np.flatnonzero(d == d.min())
        if len(best) > 1:   # tie: even code (mantissa LSB 0), prefer the sign of v
            best = [b for b in best if (b & 1) == 0 and (np.sign(TAB[b]) == np.sign(v) or TAB[b] == 0)] or best
        out[i] = best[0]
    return out


def lib():
    from cbw import _lib
    return _lib, _lib.load()


def test_mfma_fp8_operand_map_exact_integers():
    _lib, L = lib()
    rng = np.random.default_rng(0)
    ints = [c for c in range(256) if not np.isnan(TAB[c]) and TAB[c] == int(TAB[c]) and abs(TAB[c]) <= 4]
    A = rng.choice(ints, (16, 128)).astype(np.uint8)
    Bt = rng.choice(ints, (16, 128)).astype(np.uint8)
    Bt[3, 5] = ints[-1]   # asymmetric
    want = TAB[A] @ TAB[Bt].T
    d = torch.device("cuda:0")
    a, b = torch.from_numpy(A).to(d), torch.from_numpy(Bt).to(d)
    match = []
    for mode in range(4):
        c = torch.zeros((16, 16), device=d)
        _lib.check(L.cbw_fp8_probe(mode, a.data_ptr(), b.data_ptr(), c.data_ptr(), None, 0, _lib.stream_handle()), "probe")
        if np.array_equal(c.cpu().numpy().astype(np.float64), want):
            match.append(mode)
    # the product is invariant under any k-permutation shared by A and B (the hardware pairs A's and B's k slots
    # alike), so every mode that puts row / column l & 15 on lane l must match; the kernel's is mode 0
    print("operand maps matching exactly:", match)
    assert match == [0, 1, 2, 3], f"rows / columns not on lane & 15, or the scales are not unit: {match}"


def test_fp8_conversions_match_host_encoder():
    _lib, L = lib()
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.standard_normal(4000) * 3, rng.standard_normal(1000) * 200, rng.standard_normal(1000) * 1e-3,
                        [0.0, -0.0, 448, 449, 470, 1e6, -1e6, 2 ** -9, 2 ** -10, 3 * 2 ** -10, 2 ** -6, 0.0625 * 1.0625,
                         1.0 + 1 / 16, 1.0 + 3 / 16, 240.0, 248.0]]).astype(np.float32)
    x = x[: len(x) // 8 * 8]
    d = torch.device("cuda:0")
    xt = torch.from_numpy(x).to(d)
    q = torch.zeros(len(x), dtype=torch.uint8, device=d)
    back = torch.zeros(len(x), device=d)
    _lib.check(L.cbw_fp8_probe(4, xt.data_ptr(), None, q.data_ptr(), back.data_ptr(), len(x), _lib.stream_handle()),
               "probe")
    got = q.cpu().numpy()
    want = encode(x)
    bad = np.flatnonzero((got != want) & ~((TAB[got] == 0) & (TAB[want] == 0)))
    assert bad.size == 0, [(float(x[i]), int(got[i]), int(want[i])) for i in bad[:10]]
    np.testing.assert_array_equal(back.cpu().numpy(), TAB[got].astype(np.float32))


def ref_conv(x, w, alpha, bias, res, res_scale, k, stride, relu):
    """float64 NHWC conv of decoded e4m3 operands, pad k // 2"""
    N, H, W, C = x.shape
    Co = w.shape[0]
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // stride + 1, (W + 2 * p - k) // stride + 1
    xp = np.zeros((N, H + 2 * p, W + 2 * p, C))
    xp[:, p:p + H, p:p + W] = x
    out = np.zeros((N, Ho, Wo, Co))
    for kh in range(k):
        for kw in range(k):
            patch = xp[:, kh:kh + stride * Ho:stride, kw:kw + stride * Wo:stride, :]
            out += patch @ w[:, kh, kw, :].T
    out = out * alpha + bias
    if res is not None:
        out = out + res.reshape(out.shape) * res_scale
    return np.maximum(out, 0) if relu else out


@pytest.mark.parametrize("k,stride,Cin,Cout,res,out_bf16", [
    (1, 1, 256, 128, False, False), (3, 1, 128, 128, False, False), (3, 2, 128, 256, False, True),
    (1, 1, 128, 512, True, False), (1, 2, 256, 512, False, True), (3, 1, 512, 512, True, True),
    (1, 1, 512, 2048, True, True), (1, 1, 512, 256, False, False), (1, 1, 1024, 256, False, False),
    (3, 2, 256, 256, False, False)])
def test_conv_fp8_vs_float64(k, stride, Cin, Cout, res, out_bf16):
    _lib, L = lib()
    rng = np.random.default_rng(k * 100 + stride * 10 + Cin // 128 + Cout)
    N, H, W = 3, 11, 13
    codes = [c for c in range(256) if not np.isnan(TAB[c]) and abs(TAB[c]) <= 8]
    xq = rng.choice(codes, (N, H, W, Cin)).astype(np.uint8)
    wq = rng.choice(codes, (Cout, k, k, Cin)).astype(np.uint8)
    alpha = rng.uniform(0.5, 2.0, Cout).astype(np.float32) * 1e-3
    bias = rng.standard_normal(Cout).astype(np.float32)
    Ho, Wo = (H + 2 * (k // 2) - k) // stride + 1, (W + 2 * (k // 2) - k) // stride + 1
    rq = rng.choice(codes, (N * Ho * Wo, Cout)).astype(np.uint8) if res else None
    rs, ys = 0.25, 0.125
    d = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d)   # noqa: E731
    y = torch.zeros((N * Ho * Wo, Cout), dtype=torch.bfloat16 if out_bf16 else torch.uint8, device=d)
    xt, wt, at, bt = t(xq), t(wq), t(alpha), t(bias)
    rt = t(rq) if res else None
    _lib.check(L.cbw_conv2d_fp8(xt.data_ptr(), wt.data_ptr(), at.data_ptr(), bt.data_ptr(), _lib.ptr(rt), rs,
                                y.data_ptr(), ys, int(out_bf16), 1, N, H, W, Cin, Cout, k, stride, _lib.stream_handle()),
               "cbw_conv2d_fp8")
    want = ref_conv(TAB[xq], TAB[wq], alpha.astype(np.float64), bias.astype(np.float64), TAB[rq] if res else None, rs,
                    k, stride, True).reshape(-1, Cout)
    if out_bf16:
        got = y.float().cpu().numpy()
        # bf16 output: fp32 accumulation (exact e4m3 products, a different summation order) then bf16 rounding
        np.testing.assert_allclose(got, want, rtol=2 ** -7, atol=2e-3 * np.abs(want).max())
    else:
        got = TAB[y.cpu().numpy()]
        wq_out = TAB[encode(want / ys)]

        def step(v):   # the e4m3 spacing at |v| (subnormals: 2^-9)
            e = np.floor(np.log2(np.maximum(np.abs(v), 2.0 ** -6)))
            return 2.0 ** (e - 3)
        # exact apart from fp32-vs-float64 differences at an e4m3 rounding boundary: then one e4m3 step apart
        d = np.abs(got - wq_out)
        bad = d > np.maximum(step(got), step(wq_out)) + 1e-12
        mis = got != wq_out
        info = [(tuple(int(v) for v in i), float(want[tuple(i)] / ys), float(got[tuple(i)]), float(wq_out[tuple(i)]))
                for i in np.argwhere(bad | mis)[:8]]
        assert not bad.any() and mis.mean() < 2e-3, (int(bad.sum()), float(mis.mean()), info)


@pytest.fixture(scope="module")
def lef_setup():
    """large-v3 LEF widths (D 1280), the bench's seeds, 1536 keywords; the utterance of bench clip 0."""
    import bench
    from cbw import synth
    from cbw.kws import KwsEngine
    dev = torch.device("cuda:0")
    D = 1280
    hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True,
              proj_mlp_units=64, resnet_version="resnet-50", threshold=0.5)
    kws = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp), dev)
    K = 1536
    db, dbm, db32 = bench.build_keyword_db(kws, K, D, f32=True)
    g = torch.Generator(device=dev).manual_seed(77)
    hs = torch.randn((1, 3, 1500, D), generator=g, device=dev)
    hs = hs / hs.norm(dim=-1, keepdim=True)
    um = torch.ones((1, 3, 1500), device=dev)
    pu, pum = kws.project(hs, um)
    pu32, _ = kws.project_f32(hs, um)
    cal = torch.arange(512, dtype=torch.int32, device=dev)
    kws.calibrate_fp8(pu32[0], pum[0], db32, dbm, sel=cal, margin=1.0, utt=pu[0], kwd=db)
    return dict(kws=kws, db=db, dbm=dbm, db32=db32, pu=pu[0], pum=pum[0], pu32=pu32[0], dev=dev, K=K)


def _p(lg):
    return torch.softmax(lg.double(), -1)[:, 1].cpu().numpy()


def test_fp8_network_error_and_cascade_decisions(lef_setup):
    s = lef_setup
    kws, K = s["kws"], s["K"]
    ho = slice(512, K)   # held out from the calibration
    db, dbm, db32 = s["db"][ho].contiguous(), s["dbm"][ho].contiguous(), s["db32"][ho].contiguous()
    n = db.shape[0]
    l8 = kws.score_fp8(s["pu"], s["pum"], db, dbm, chunk=512)
    l16 = kws.score(s["pu"], s["pum"], db, dbm, chunk=512)
    l32 = torch.empty_like(l8)
    kws.rescore(s["pu32"], s["pum"], db32, dbm, l32, torch.arange(n, dtype=torch.int32, device=s["dev"]))
    p8, p16, p32 = _p(l8), _p(l16), _p(l32)
    e8, e16 = np.abs(p8 - p32), np.abs(p16 - p32)
    print(f"fp8 |p - p32| max {e8.max():.4f} p99 {np.quantile(e8, 0.99):.4f}; bf16 max {e16.max():.4f}; "
          f"corr(l8, l32) {np.corrcoef((l8[:, 1] - l8[:, 0]).cpu(), (l32[:, 1] - l32[:, 0]).cpu())[0, 1]:.4f}")
    assert np.isfinite(p8).all() and e8.max() < 0.35 and np.corrcoef(p8, p32)[0, 1] > 0.9
    fp8_band = min(0.49, 1.5 * float(e8.max()))
    ex, st = kws.score_exact(s["pu"], s["pum"], db, dbm, s["pu32"], db32, 0.5, 0.03, chunk=512, band_x3=1e-4,
                             fp8_band=fp8_band)
    flips = np.flatnonzero((_p(ex) >= 0.5) != (p32 >= 0.5))
    assert flips.size == 0, flips[:20]
    assert 0 < st["bf16"] < n


def test_fp8_tier_stage1_output_quantized_in_the_block(lef_setup, monkeypatch):
    """(CBW_FP8_Q8=1) The last stage-1 block stores its output in e4m3 itself (bottleneck.hip, Q8: conv_fp8.hip's pack
    on the bf16 values the block would store) instead of a bf16 tensor quantized by a separate pass (cbw_quant_fp8).
    Both quantize the same bf16 values with the same pack, so the fp8 tier's logits are bit-identical (a wrong e4m3
    pack or layout moves them by O(1)); against stage 1 as three convs + the pass (CBW_NO_BOTTLENECK_FUSION=1, bf16
    rounding order differs, then amplified by e4m3 rounding) the probabilities stay well inside the fp8 band."""
    s = lef_setup
    kws = s["kws"]
    db, dbm = s["db"][:640].contiguous(), s["dbm"][:640].contiguous()
    monkeypatch.setenv("CBW_FP8_Q8", "1")
    fused = kws.score_fp8(s["pu"], s["pum"], db, dbm, chunk=320)
    monkeypatch.setenv("CBW_FP8_Q8", "0")
    passq = kws.score_fp8(s["pu"], s["pum"], db, dbm, chunk=320)
    monkeypatch.setenv("CBW_NO_BOTTLENECK_FUSION", "1")
    unfused = kws.score_fp8(s["pu"], s["pum"], db, dbm, chunk=320)
    torch.cuda.synchronize()
    assert torch.isfinite(fused).all()
    d = np.abs(_p(fused) - _p(unfused))
    print(f"fp8 tier, fused e4m3 stage-1 output: max |logit diff| vs the quantization pass "
          f"{(fused - passq).abs().max().item():.2e}; max |dp| vs convs + pass {d.max():.2e}")
    assert torch.equal(fused, passq)
    assert d.max() < 0.15
