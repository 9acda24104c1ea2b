"""Every decision of a bench clip equals the all-pairs fp32 decision, at the bench's own operating point.

bench.py's default configuration (large-v3 encoder and LEF/ResNet-50 with the bench's seeds, the bench's seeded
10 000-keyword database, the setup-time bias / logit-offset calibration on the database's first 512 keywords,
bf16 scoring in chunks of 625 over two streams, the 0.015 band through the compensated tier and 1e-4 into the fp32
tier) against all 10 000 pairs re-scored on the fp32 tier -- the path
test_gpu_kws.py::test_exact_rescore_matches_reference_fp32 pins to the reference's own fp32 forward.  The band is
an empirical bound; this checks it where the bench line is measured: the timed clips 0-3 (rank 0,
steps 0-3), every one of their 10 000 spotted-or-not decisions, and the bf16 error of every pair inside the band.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bench_clip_decisions_equal_all_pairs_fp32():
    import bench
    from cbw import synth
    from cbw.kws import KwsEngine
    from cbw.whisper import EncoderEngine, default_layer_ids, log_mel
    dev = torch.device("cuda:0")
    cfg = synth.WHISPER_CONFIGS["large-v3"]
    n_mel, D, n_layers = cfg[0], cfg[1], cfg[2]
    enc = EncoderEngine(cfg, synth.synth_whisper_encoder_state_dict("large-v3", seed=0), dev)
    ids = default_layer_ids(n_layers)
    hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True,
              proj_mlp_units=64, resnet_version="resnet-50", threshold=0.5)
    kws = KwsEngine(hp, synth.synth_kws_state_dict(seed=0, **hp), dev)
    K, band, band_x3 = 10000, 0.015, 1e-4
    db, dbm, db32 = bench.build_keyword_db(kws, K, D, f32=True)
    bench.calibrate_kws(kws, enc, ids, n_mel, K, D, 512, dev)
    um = torch.ones((1, 3, 1500), device=dev)

    def prob(lg):
        return torch.softmax(lg.double(), -1)[:, 1].cpu().numpy()
    for clip in range(4):   # the bench's first timed clips of rank 0 (ids 1000 rank + i)
        _, mel = log_mel(torch.from_numpy(synth.synth_clip(clip)).to(dev), n_mel, packed=True)
        hs = enc.hidden_states(mel, ids, normalize=True)
        pu, pum = kws.project(hs, um)
        pu32, _ = kws.project_f32(hs, um)
        bf = kws.score(pu[0], pum[0], db, dbm, chunk=625)
        ex, stats = kws.score_exact(pu[0], pum[0], db, dbm, pu32[0], db32, 0.5, band, chunk=625, band_x3=band_x3)
        full = torch.empty_like(ex)
        kws.rescore(pu32[0], pum[0], db32, dbm, full, torch.arange(K, dtype=torch.int32, device=dev))
        torch.cuda.synchronize()
        p_bf, p_ex, p32 = prob(bf), prob(ex), prob(full)
        assert np.isfinite(p32).all()
        err = np.abs(p_bf - p32)
        assert err.max() < band, f"clip {clip}: bf16 error {err.max():.4f} reaches the band {band}"
        flips = np.nonzero((p_ex >= 0.5) != (p32 >= 0.5))[0]
        assert flips.size == 0, f"clip {clip}: decisions differing from the all-pairs fp32 ones: {flips.tolist()[:20]}"
        n_band = int(np.sum(np.abs(p_bf - 0.5) <= band))
        assert abs(stats["band"] - n_band) <= 2 and 100 <= n_band <= 1000   # (fp32 vs float64 softmax at the edge)
