"""Encoder parity at the sizes the bench runs (VERDICT r01 "what's weak" 1).

* The split-K GEMM (``cbw_gemm`` with S in {2, 4}: conv_igemm_kernel over K-slices into fp32 partials +
  splitk_epilogue_kernel) against a float64 torch matmul of the same bf16 operands, with and without
  bias / fp32 residual (in place, as the encoder's residual stream uses it) / GELU / bf16 output, at
  M = 1500 (a partial 128-row tile) and the small / large-v3 out-projection and fc2 shapes.
* ``cbw_encoder_hs`` at Whisper-small (D 768, 12 heads, 12 layers, 80 mel: S = 2 / 4 on out-proj / fc2) and
  at a 2-layer slice of large-v3 (D 1280, 20 heads, ffn 5120, 128 mel: S = 4) against the float64 oracle
  (oracle/encoder.py, restating HF WhisperEncoder as called at src/model/cb_whisper.py:100-106 and
  src/utils.py:188-195), fed the oracle's own log-mel of the same clip.

Tolerances (stated here): split-K GEMM with f32 output 2e-3 of max|y| (bf16 operands are
exact in the float64 reference; the only error is fp32 accumulation order), bf16 output 1e-2 of max|y|;
encoder hidden states 2e-2 of max|hs| per state and relative Frobenius error <= 1e-2 (bf16 weights and
GEMM operands against fp32 weights evaluated in float64); normalised selected states 2.5e-2 absolute.
"""
import numpy as np
import pytest
import torch

from cbw import synth

pytestmark = pytest.mark.gpu

FLAG_GELU, FLAG_RES_F32, FLAG_OUT_F32 = 2, 4, 8


def _bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16)


@pytest.mark.parametrize("M,K,N,S", [(1500, 1280, 1280, 4), (1500, 5120, 1280, 4), (1500, 768, 768, 2),
                                     (1500, 3072, 768, 4)])
def test_splitk_factor_at_encoder_shapes(M, K, N, S):
    """The production shapes really take split-K (large-v3 out-proj / fc2: S = 4; small out-proj 2, fc2 4)."""
    from cbw import _lib
    assert _lib.load().cbw_gemm_splitk_factor(M, K, N) == S


@pytest.mark.parametrize("case", [
    # M, K, N, S, bias, residual (None | "f32_inplace" | "bf16"), flags
    (1500, 1280, 1280, 4, True, "f32_inplace", FLAG_RES_F32 | FLAG_OUT_F32),   # large-v3 out-proj
    (1500, 5120, 1280, 4, True, "f32_inplace", FLAG_RES_F32 | FLAG_OUT_F32),   # large-v3 fc2
    (1500, 768, 768, 2, True, "f32_inplace", FLAG_RES_F32 | FLAG_OUT_F32),     # small out-proj
    (1500, 3072, 768, 4, True, "f32_inplace", FLAG_RES_F32 | FLAG_OUT_F32),    # small fc2
    (1500, 1280, 1280, 2, True, None, FLAG_GELU),                              # GELU, bf16 out, no residual
    (1500, 1280, 1280, 4, False, "bf16", 0),                                   # bf16 residual, no bias
    (3000, 2048, 256, 8, True, None, FLAG_OUT_F32),                            # 2 clips, S = 8
    (1500, 1280, 1280, 1, True, "f32_inplace", FLAG_RES_F32 | FLAG_OUT_F32),   # unsplit reference path
])
def test_gemm_splitk_vs_float64(case):
    from cbw import _lib
    M, K, N, S, with_bias, res_kind, flags = case
    lib = _lib.load()
    d = torch.device("cuda:0")
    rng = np.random.default_rng(abs(hash(case)) % 2**32)
    x = _bf(rng.standard_normal((M, K)))
    w = _bf(rng.standard_normal((N, K)) / np.sqrt(K))
    b = torch.from_numpy(rng.standard_normal(N).astype(np.float32)) if with_bias else None
    r32 = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32))
    out_f32 = bool(flags & FLAG_OUT_F32)
    if res_kind == "f32_inplace":           # the encoder's residual stream: y aliases res (hbuf)
        y = r32.to(d).clone()
        res = y
    else:
        y = torch.full((M, N), float("nan"), dtype=torch.float32 if out_f32 else torch.bfloat16, device=d)
        res = None if res_kind is None else r32.to(torch.bfloat16).to(d)
    part = torch.empty((max(S, 1) * M * N,), dtype=torch.float32, device=d)
    xd, wd = x.to(d), w.to(d)
    bd = b.to(d) if b is not None else None
    _lib.check(lib.cbw_gemm(xd.data_ptr(), wd.data_ptr(), _lib.ptr(bd), _lib.ptr(res), y.data_ptr(), M, K, N, flags,
                            S, part.data_ptr(), part.numel(), _lib.stream_handle()), "cbw_gemm")
    torch.cuda.synchronize()
    ref = x.double() @ w.double().T
    if b is not None:
        ref = ref + b.double()
    if res_kind == "f32_inplace":
        ref = ref + r32.double()
    elif res_kind == "bf16":
        ref = ref + r32.to(torch.bfloat16).double()
    if flags & FLAG_GELU:
        ref = torch.nn.functional.gelu(ref)
    got = y.double().cpu()
    tol = (2e-3 if out_f32 else 1e-2) * ref.abs().max().item()
    err = (got - ref).abs().max().item()
    assert err <= tol, f"split-K S={S}: max err {err:.3g} > {tol:.3g}"


def test_gemm_splitk_deterministic():
    """Fixed-order reduction of the K-slices: two runs give identical bits."""
    from cbw import _lib
    lib = _lib.load()
    d = torch.device("cuda:0")
    g = torch.Generator(device=d)
    g.manual_seed(3)
    M, K, N, S = 1500, 5120, 1280, 4
    x = torch.randn((M, K), generator=g, device=d).to(torch.bfloat16)
    w = (torch.randn((N, K), generator=g, device=d) / K ** 0.5).to(torch.bfloat16)
    part = torch.empty((S * M * N,), dtype=torch.float32, device=d)
    outs = []
    for _ in range(2):
        y = torch.empty((M, N), dtype=torch.float32, device=d)
        _lib.check(lib.cbw_gemm(x.data_ptr(), w.data_ptr(), None, None, y.data_ptr(), M, K, N, FLAG_OUT_F32, S,
                                part.data_ptr(), part.numel(), _lib.stream_handle()), "cbw_gemm")
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_gemm_rejects_small_partial_buffer():
    from cbw import _lib
    lib = _lib.load()
    d = torch.device("cuda:0")
    x = torch.zeros((1500, 1280), dtype=torch.bfloat16, device=d)
    w = torch.zeros((1280, 1280), dtype=torch.bfloat16, device=d)
    y = torch.zeros((1500, 1280), dtype=torch.float32, device=d)
    part = torch.empty((1500 * 1280,), dtype=torch.float32, device=d)
    rc = lib.cbw_gemm(x.data_ptr(), w.data_ptr(), None, None, y.data_ptr(), 1500, 1280, 1280, FLAG_OUT_F32, 4,
                      part.data_ptr(), part.numel(), _lib.stream_handle())
    assert rc == -3


def _encoder_vs_oracle(name, n_layers, ids_raw, ids_sel, clip_seed):
    import oracle.encoder as oenc
    import oracle.mel as omel
    from cbw.whisper import EncoderEngine
    n_mel, D, full, H, F = synth.WHISPER_CONFIGS[name]
    cfg = (n_mel, D, n_layers, H, F)
    sd = synth.synth_whisper_encoder_state_dict(name, seed=0, n_layers=n_layers)
    mel = omel.log_mel(synth.synth_clip(clip_seed), n_mel)                      # [n_mel, 3000] float64
    ref = oenc.encoder_hidden_states({k: v.astype(np.float64) for k, v in sd.items()}, mel, H)
    eng = EncoderEngine(cfg, sd)
    dev = eng.device
    pk = torch.zeros((3000, eng.cpad), dtype=torch.bfloat16, device=dev)
    pk[:, :n_mel] = torch.from_numpy(mel.T.astype(np.float32)).to(dev).to(torch.bfloat16)
    hs = eng.hidden_states(pk, ids_raw, normalize=False)[0].double().cpu().numpy()
    for j, i in enumerate(ids_raw):
        r = ref[i]
        err = np.abs(hs[j] - r).max()
        fro = np.linalg.norm(hs[j] - r) / np.linalg.norm(r)
        assert err <= 2e-2 * np.abs(r).max(), f"{name} hidden_states[{i}]: max err {err:.3g} (max|hs| {np.abs(r).max():.3g})"
        assert fro <= 1e-2, f"{name} hidden_states[{i}]: relative Frobenius error {fro:.3g}"
    sel = eng.hidden_states(pk, ids_sel, normalize=True)[0].double().cpu().numpy()
    rs = oenc.select_and_normalise(ref, ids_sel)
    np.testing.assert_allclose(sel, rs, atol=2.5e-2)
    np.testing.assert_allclose(np.linalg.norm(sel, axis=-1), 1.0, atol=1e-4)


def test_encoder_small_vs_oracle():
    """Whisper-small (C2): all 12 layers; hidden_states[10:22] = states 10, 11, 12 (12 post-LN)."""
    _encoder_vs_oracle("small", 12, [0, 1, 6, 10, 11, 12], [10, 11, 12], clip_seed=3)


def test_encoder_large_v3_slice_vs_oracle():
    """Two layers of large-v3 (C3 widths: D 1280, 20 heads, ffn 5120, 128 mel)."""
    _encoder_vs_oracle("large-v3", 2, [0, 1, 2], [1, 2], clip_seed=4)


def test_encoder_splitk_matches_unsplit_within_tolerance(monkeypatch):
    """CBW_ENC_SPLITK=0 (unsplit GEMMs) and the default split-K path agree at large-v3 widths."""
    from cbw.whisper import EncoderEngine, log_mel
    name = "large-v3"
    n_mel, D, _, H, F = synth.WHISPER_CONFIGS[name]
    sd = synth.synth_whisper_encoder_state_dict(name, seed=0, n_layers=2)
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("CBW_ENC_SPLITK", mode)
        eng = EncoderEngine((n_mel, D, 2, H, F), sd)
        _, pk = log_mel(torch.from_numpy(synth.synth_clip(4)).to(eng.device), n_mel, packed=True)
        outs.append(eng.hidden_states(pk, [1, 2], normalize=False))
    torch.cuda.synchronize()
    a, b = outs
    assert (a - b).abs().max().item() <= 1e-3 * b.abs().max().item()


@pytest.mark.parametrize("T", [1500, 100, 37])
def test_encoder_attention_vs_fp32(T):
    """cbw_encoder_attention against a float32 softmax(q k^T) v of the same bf16 operands, with scores spread wide
    enough that each query attends to a few keys: a key / value mis-pairing inside an MFMA k-slot, which near-uniform
    attention (the synthetic encoders) would average away, shows here as an O(1) error (a round-6 pipelined variant
    with transposing LDS reads failed exactly so: 1.2-1.6 of max|out|, and was not kept).  Within 1e-2 of max|out|
    (bf16 P and output rounding); full, partial-tile and sub-tile lengths."""
    from cbw import _lib
    lib = _lib.load()
    d = torch.device("cuda:0")
    g = torch.Generator(device=d)
    g.manual_seed(T)
    B, H = 2, 3
    scale = torch.tensor([2.0, 2.0, 1.0], device=d)[None, None, :, None, None]
    qkv = (torch.randn((B, T, 3, H, 64), generator=g, device=d) * scale).to(torch.bfloat16)
    q, k, v = (qkv[:, :, i].float().permute(0, 2, 1, 3) for i in range(3))
    ref = torch.softmax(q @ k.transpose(-1, -2), dim=-1) @ v                 # [B, H, T, 64]
    ref = ref.permute(0, 2, 1, 3).reshape(B, T, H * 64)
    y = torch.full((B, T, H * 64), float("nan"), dtype=torch.bfloat16, device=d)
    _lib.check(lib.cbw_encoder_attention(qkv.data_ptr(), y.data_ptr(), B, T, H, _lib.stream_handle()),
               "cbw_encoder_attention")
    torch.cuda.synchronize()
    torch.testing.assert_close(y.float(), ref, rtol=0, atol=1e-2 * ref.abs().max().item())
