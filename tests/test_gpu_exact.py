"""Exact decisions at the bench operating point (VERDICT r01 "what's weak" 2/3, "next" 2 and 8).

Large-v3 LEF widths (D 1280, ResNet-50), K = 720 keywords scored in chunks of 625 over the two scoring
streams (the bench's configuration), with the fp32 re-scoring band (``KwsEngine.score_exact``:
cbw_kws_band + cbw_kws_rescore from the cached fp32 keyword projections) at the bench's 0.03:

* every one of the 720 spotted-or-not decisions equals the all-pairs fp32 decision (the fp32 path is pinned
  to the reference's own fp32 forward by test_gpu_kws.py::test_exact_rescore_matches_reference_fp32);
* 16 random pairs plus the 16 pairs nearest the threshold against the float64 oracle (oracle/kws.py):
  identical decisions; logits within 2e-2 of max|logit| (bf16 pairs) / 1e-4 (re-scored pairs);
* pairs outside the band keep their bf16 logits bit for bit;
* the compensated-bf16 tier (cbw_kws_rescore_x3) on all 720 pairs within 1e-4 of the fp32 probabilities,
  and the two-tier schedule (band 0.03 -> x3, then 1e-4 -> fp32) giving the fp32 decisions;
* a single-GPU sharding simulation: the 720 keywords split into 8 contiguous shards (cbw.parallel.shard_range)
  scored separately and concatenated equal the unsharded scores bit for bit (bf16 and banded).
"""
import numpy as np
import pytest
import torch

from cbw import synth

pytestmark = pytest.mark.gpu

K, D, THR, BAND, CHUNK = 720, 1280, 0.5, 0.03, 625
BAND_X3 = 1e-4   # compensated-bf16 tier: measured max |p_x3 - p_fp32| 2.5e-5 at the bench point (tools/band_stats.py)
HP = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True, proj_mlp_units=64,
          resnet_version="resnet-50", threshold=THR)


@pytest.fixture(scope="module")
def setup():
    from cbw.kws import KwsEngine
    sd = synth.synth_kws_state_dict(seed=0, **HP)
    eng = KwsEngine(HP, sd)
    d = eng.device
    g = torch.Generator(device=d)
    g.manual_seed(77)
    kwd = torch.randn((K, 3, 150, D), generator=g, device=d)
    kwd = kwd / kwd.norm(dim=-1, keepdim=True)
    lens = torch.randint(8, 151, (K,), generator=g, device=d)
    km = (torch.arange(150, device=d)[None, :] < lens[:, None]).float()[:, None, :].expand(K, 3, 150).contiguous()
    kwd = kwd * km[..., None]
    utt = torch.randn((1, 3, 1500, D), generator=g, device=d)
    utt = utt / utt.norm(dim=-1, keepdim=True)
    um = torch.ones((1, 3, 1500), device=d)
    um[:, :, 1350:] = 0
    utt = utt * um[..., None]
    pk, pkm = eng.project(kwd, km)
    pk32, _ = eng.project_f32(kwd, km)
    pu, pum = eng.project(utt, um)
    pu32, _ = eng.project_f32(utt, um)
    return dict(sd=sd, eng=eng, kwd=kwd, km=km, utt=utt, um=um, pk=pk, pkm=pkm, pk32=pk32, pu=pu[0], pum=pum[0],
                pu32=pu32[0])


def _prob(lg):
    return torch.softmax(lg.double(), -1)[:, 1].cpu().numpy()


def test_band_decisions_equal_fp32_decisions_at_bench_point(setup):
    s = setup
    eng = s["eng"]
    bf = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
    banded, st = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, BAND, chunk=CHUNK)
    n = st["band"]
    full = bf.clone()
    eng.rescore(s["pu32"], s["pum"], s["pk32"], s["pkm"], full, torch.arange(K, dtype=torch.int32, device=bf.device))
    torch.cuda.synchronize()
    p_bf, p_band, p_fp32 = _prob(bf), _prob(banded), _prob(full)
    inside = np.abs(p_bf - THR) <= BAND
    assert n == int(inside.sum()) and n > 0
    # outside the band: bf16 logits untouched, bit for bit
    np.testing.assert_array_equal(banded.cpu().numpy()[~inside], bf.cpu().numpy()[~inside])
    # inside: the fp32 logits, bit for bit the all-pairs fp32 result
    np.testing.assert_array_equal(banded.cpu().numpy()[inside], full.cpu().numpy()[inside])
    flips_bf16 = int(((p_bf >= THR) != (p_fp32 >= THR)).sum())
    print(f"K={K}: band pairs {n}, bf16 decision flips vs fp32 {flips_bf16}, max |p_bf16 - p_fp32| "
          f"{np.abs(p_bf - p_fp32).max():.4f}")
    assert np.abs(p_bf - p_fp32).max() < BAND, "bf16 error exceeds the band: widen exact_band"
    np.testing.assert_array_equal(p_band >= THR, p_fp32 >= THR)
    # the spot kernel's index list on the banded logits is the fp32 decision set
    from cbw.kws import spot
    _, idx = spot(banded, None, THR)
    assert idx.cpu().tolist() == np.nonzero(p_fp32 >= THR)[0].tolist()


def test_band_pairs_vs_oracle_sampled(setup):
    import oracle.kws as okws
    s = setup
    eng = s["eng"]
    banded, _ = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, BAND, chunk=CHUNK)
    bf = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
    torch.cuda.synchronize()
    p_bf = _prob(bf)
    rng = np.random.default_rng(5)
    near = np.argsort(np.abs(p_bf - THR))[:16]
    pick = np.unique(np.concatenate([rng.choice(K, 16, replace=False), near]))
    kwd = s["kwd"][torch.from_numpy(pick).to(bf.device)].cpu().numpy()
    km = s["km"][torch.from_numpy(pick).to(bf.device)].cpu().numpy()
    ref, _ = okws.kws_forward(s["sd"], HP, kwd, s["utt"].cpu().numpy(), km, s["um"].cpu().numpy(),
                              return_features=False)
    got = banded.cpu().numpy()[pick]
    inside = np.abs(p_bf[pick] - THR) <= BAND
    scale = np.abs(ref).max()
    assert np.abs(got[inside] - ref[inside]).max(initial=0) < 1e-4 * scale
    assert np.abs(got[~inside] - ref[~inside]).max(initial=0) < 2e-2 * scale
    p_ref, _ = okws.decide(ref, None, THR)
    p_got = torch.softmax(torch.from_numpy(got).double(), -1)[:, 1].numpy()
    np.testing.assert_array_equal(p_got >= THR, p_ref >= THR)


def test_x3_tier_close_to_fp32_and_two_tier_decisions(setup):
    s = setup
    eng = s["eng"]
    bf = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
    everyone = torch.arange(K, dtype=torch.int32, device=bf.device)
    full, x3 = bf.clone(), bf.clone()
    eng.rescore(s["pu32"], s["pum"], s["pk32"], s["pkm"], full, everyone)
    eng.rescore(s["pu32"], s["pum"], s["pk32"], s["pkm"], x3, everyone, tier="x3")
    two, st = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, BAND, chunk=CHUNK,
                              band_x3=BAND_X3)
    torch.cuda.synchronize()
    p32, px3, p2 = _prob(full), _prob(x3), _prob(two)
    err = np.abs(px3 - p32).max()
    print(f"x3 tier: max |p_x3 - p_fp32| = {err:.2e}, max |dlogit| = {(x3 - full).abs().max().item():.2e}; "
          f"two-tier: {st['band']} band pairs, {st['fp32']} in fp32")
    assert err < BAND_X3
    assert st["fp32"] < st["band"]
    np.testing.assert_array_equal(p2 >= THR, p32 >= THR)


@pytest.mark.parametrize("band", [0.0, BAND])
def test_sharding_simulation_bit_exact(setup, band):
    """8 contiguous keyword shards scored one by one and concatenated == the unsharded call."""
    from cbw.parallel import shard_range
    s = setup
    eng = s["eng"]
    whole, _ = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, band, chunk=CHUNK)
    parts = []
    for r in range(8):
        lo, hi = shard_range(K, r, 8)
        lg, _ = eng.score_exact(s["pu"], s["pum"], s["pk"][lo:hi], s["pkm"][lo:hi], s["pu32"], s["pk32"][lo:hi],
                                THR, band, chunk=CHUNK)
        parts.append(lg)
    torch.cuda.synchronize()
    torch.testing.assert_close(torch.cat(parts), whole, rtol=0, atol=0)


BAND_CAL = 0.015   # calibrated bf16 scoring (bias correction + logit offset): the band bench.py runs with
BAND_SCALE = 3.0e-3  # ... and the per-pair band (bench.py --band-scale 3e-3): |p - thr| <= c max(|l0|, |l1|)
N_CAL = 256


def test_bias_correction_narrows_bf16_error(setup):
    """KwsEngine.calibrate_bias (cbw_kws_calibrate_bias) on the first 256 keywords; on the other 464 the
    bias-corrected bf16 logits are closer to the fp32 ones (rms and max), their decisions after the two-tier
    schedule at the narrower band equal the fp32 decisions, and calibrate_bias() restores the folded biases
    bit for bit."""
    s = setup
    eng = s["eng"]
    dev = s["pu"].device
    bf = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
    full = bf.clone()
    eng.rescore(s["pu32"], s["pum"], s["pk32"], s["pkm"], full, torch.arange(K, dtype=torch.int32, device=dev))
    try:
        off = eng.calibrate_bias(s["pu32"], s["pum"], s["pk32"], s["pkm"], torch.arange(N_CAL, dtype=torch.int32, device=dev),
                                 utt=s["pu"], kwd=s["pk"])
        print(f"calibrated logit offset {off}")
        cal = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
        two, st = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, BAND_CAL,
                                  chunk=CHUNK, band_x3=BAND_X3)
        sc, st_sc = eng.score_exact(s["pu"], s["pum"], s["pk"], s["pkm"], s["pu32"], s["pk32"], THR, BAND_SCALE,
                                    chunk=CHUNK, band_x3=BAND_X3, band_scaled=True)
        torch.cuda.synchronize()
    finally:
        eng.calibrate_bias()
    p32, pbf, pcal, ptwo = _prob(full)[N_CAL:], _prob(bf)[N_CAL:], _prob(cal)[N_CAL:], _prob(two)
    d32 = (full[:, 1] - full[:, 0]).double()[N_CAL:]
    e_bf = ((bf[:, 1] - bf[:, 0]).double()[N_CAL:] - d32).abs()
    e_cal = ((cal[:, 1] - cal[:, 0]).double()[N_CAL:] - d32).abs()
    print(f"l1-l0 error vs fp32 ({K - N_CAL} held-out keywords): folded max {e_bf.max():.3e} rms {e_bf.pow(2).mean().sqrt():.3e}; "
          f"bias-corrected max {e_cal.max():.3e} rms {e_cal.pow(2).mean().sqrt():.3e}; max |p - p32| "
          f"{np.abs(pbf - p32).max():.4f} -> {np.abs(pcal - p32).max():.4f}; band {BAND_CAL}: {st['band']} pairs")
    assert e_cal.pow(2).mean() < 0.6 * e_bf.pow(2).mean()
    assert e_cal.max() < e_bf.max()
    assert np.abs(pcal - p32).max() < BAND_CAL, "bias-corrected bf16 error exceeds the narrower band"
    np.testing.assert_array_equal(ptwo >= THR, _prob(full) >= THR)
    # the scaled band: every held-out pair's error within its own half-width, fp32 decisions after the tiers
    lmax = cal.abs().max(dim=1).values.double().cpu().numpy()[N_CAL:]
    ratio = np.abs(pcal - p32) / lmax
    print(f"scaled band {BAND_SCALE}: max |p - p32| / max|l| = {ratio.max():.3e}, {st_sc['band']} pairs")
    assert ratio.max() < BAND_SCALE
    np.testing.assert_array_equal(_prob(sc) >= THR, _prob(full) >= THR)
    again = eng.score(s["pu"], s["pum"], s["pk"], s["pkm"], chunk=CHUNK)
    torch.cuda.synchronize()
    torch.testing.assert_close(again, bf, rtol=0, atol=0)
