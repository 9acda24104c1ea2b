"""Every decision of the bench's timed clips equals the all-pairs fp32 decision, at the bench's own operating point;
and C4's keyword count (100 000) sharded over 8 ranks is bit-equal to the unsharded call.

bench.py's default configuration (large-v3 encoder and LEF/ResNet-50 with the bench's seeds, the bench's seeded
10 000-keyword database, the setup-time bias / logit-offset calibration on the database's first 512 keywords,
bf16 scoring in chunks of 1112, the 0.015 band through the compensated tier and 1e-4 into the fp32 tier) against all
10 000 pairs re-scored on the fp32 tier -- the path test_gpu_kws.py::test_exact_rescore_matches_reference_fp32 pins
to the reference's own fp32 forward.  The band is an empirical bound; this checks it on the clips
the bench line is measured on.  bench.py runs ``run_steps(0, warmup)`` on clips 0..warmup-1 and times clips
warmup..warmup+steps-1 (rank 0: clip ids 1000 * rank + i), so the timed clips are 2-11 for the defaults
(--warmup 2 --steps 10) and 5-24 for the driver's run (--warmup 5 --steps 20): clips 2-24 are checked, every one
of their 10 000 decisions and the bf16 error of every pair.  (bench.py also audits its last timed clip itself,
``audit_flips`` in its JSON line.)
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TIMED_CLIPS = list(range(2, 25))   # union of the default (2-11) and driver (5-24) timed clips
GROUPS = [TIMED_CLIPS[i:i + 6] for i in range(0, len(TIMED_CLIPS), 6)]


def _prob(lg):
    return torch.softmax(lg.double(), -1)[:, 1].cpu().numpy()


@pytest.fixture(scope="module")
def bench_setup():
    import bench
    from cbw import synth
    from cbw.kws import KwsEngine
    from cbw.whisper import EncoderEngine, default_layer_ids
    dev = torch.device("cuda:0")
    cfg = synth.WHISPER_CONFIGS["large-v3"]
    n_mel, D, n_layers = cfg[0], cfg[1], cfg[2]
    enc = EncoderEngine(cfg, synth.synth_whisper_encoder_state_dict("large-v3", seed=0), dev)
    ids = default_layer_ids(n_layers)
    hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True,
              proj_mlp_units=64, resnet_version="resnet-50", threshold=0.5)
    kws = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp), dev)
    return dict(bench=bench, enc=enc, ids=ids, kws=kws, n_mel=n_mel, D=D, dev=dev)


@pytest.fixture(scope="module")
def db10k(bench_setup):
    s = bench_setup
    db, dbm, db32 = s["bench"].build_keyword_db(s["kws"], 10000, s["D"], f32=True)
    s["bench"].calibrate_kws(s["kws"], s["enc"], s["ids"], s["n_mel"], 10000, s["D"], 512, s["dev"])
    return db, dbm, db32


def _utterance(s, clip):
    from cbw import synth
    from cbw.whisper import log_mel
    um = torch.ones((1, 3, 1500), device=s["dev"])
    _, mel = log_mel(torch.from_numpy(synth.synth_clip(clip)).to(s["dev"]), s["n_mel"], packed=True)
    hs = s["enc"].hidden_states(mel, s["ids"], normalize=True)
    pu, pum = s["kws"].project(hs, um)
    pu32, _ = s["kws"].project_f32(hs, um)
    return pu[0], pum[0], pu32[0]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("clips", GROUPS, ids=[f"clips{g[0]}-{g[-1]}" for g in GROUPS])
def test_bench_timed_clip_decisions_equal_all_pairs_fp32(bench_setup, db10k, clips):
    s = bench_setup
    kws, dev = s["kws"], s["dev"]
    db, dbm, db32 = db10k
    K, band, band_x3 = db.shape[0], 0.015, 1e-4
    for clip in clips:
        u, um, u32 = _utterance(s, clip)
        bf = kws.score(u, um, db, dbm, chunk=1112)
        ex, stats = kws.score_exact(u, um, db, dbm, u32, db32, 0.5, band, chunk=1112, band_x3=band_x3)
        full = torch.empty_like(ex)
        kws.rescore(u32, um, db32, dbm, full, torch.arange(K, dtype=torch.int32, device=dev))
        torch.cuda.synchronize()
        p_bf, p_ex, p32 = _prob(bf), _prob(ex), _prob(full)
        assert np.isfinite(p32).all()
        err = np.abs(p_bf - p32)
        assert err.max() < band, f"clip {clip}: bf16 error {err.max():.4f} reaches the band {band}"
        flips = np.nonzero((p_ex >= 0.5) != (p32 >= 0.5))[0]
        assert flips.size == 0, f"clip {clip}: decisions differing from the all-pairs fp32 ones: {flips.tolist()[:20]}"
        n_band = int(np.sum(np.abs(p_bf - 0.5) <= band))
        assert abs(stats["band"] - n_band) <= 2 and 100 <= n_band <= 1000   # (fp32 vs float64 softmax at the edge)


@pytest.mark.timeout(900)
def test_c4_100k_eight_shards_bit_equal_and_fp32_decisions(bench_setup):
    """C4 (BASELINE configs[3]): the bench's seeded 100 000-keyword database cut into 8 contiguous shards
    (cbw.parallel.shard_range, what --mode kwshard gives each rank) and each shard scored with score_exact; the
    concatenated logits are bit-equal to the unsharded call, and every one of the 100 000 decisions of the clip
    equals the all-pairs fp32 decision."""
    from cbw.parallel import shard_range
    s = bench_setup
    kws, dev = s["kws"], s["dev"]
    K, band, band_x3 = 100000, 0.015, 1e-4
    db, dbm, db32 = s["bench"].build_keyword_db(kws, K, s["D"], f32=True)
    s["bench"].calibrate_kws(kws, s["enc"], s["ids"], s["n_mel"], K, s["D"], 512, dev)
    u, um, u32 = _utterance(s, 5)
    whole, st = kws.score_exact(u, um, db, dbm, u32, db32, 0.5, band, chunk=1112, band_x3=band_x3)
    parts, n_band = [], 0
    for r in range(8):
        lo, hi = shard_range(K, r, 8)
        lg, st_r = kws.score_exact(u, um, db[lo:hi], dbm[lo:hi], u32, db32[lo:hi], 0.5, band, chunk=1112,
                                   band_x3=band_x3)
        parts.append(lg)
        n_band += st_r["band"]
    sharded = torch.cat(parts, 0)
    assert torch.equal(sharded, whole), "8-shard logits differ from the unsharded call"
    assert n_band == st["band"]
    full = torch.empty_like(whole)
    kws.rescore(u32, um, db32, dbm, full, torch.arange(K, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    p_bf = _prob(kws.score(u, um, db, dbm, chunk=1112))
    p_ex, p32 = _prob(whole), _prob(full)
    assert np.abs(p_bf - p32).max() < band
    flips = np.nonzero((p_ex >= 0.5) != (p32 >= 0.5))[0]
    assert flips.size == 0, f"{flips.size} of {K} decisions differ from fp32: {flips.tolist()[:20]}"
    del db, dbm, db32
    torch.cuda.empty_cache()
