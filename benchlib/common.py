"""Shared setup of bench.py's modes: the spotter's hyper-parameters, the seeded synthetic keyword database, the
one-process-per-GPU device / process-group plumbing and the setup-time calibrations (bf16 bias, operating point,
fp8 tier).  Imported by bench.py and benchlib.modes; tests and tools reach these through ``bench`` (re-exported)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch


# efficient_kws variants (efficient_kws/model.py:71-124): L = ResNet on raw-hs
# similarities (learn_features False, the reference's working L form), LE = per-layer MLP
# projector, LEF = LE + the time projector (conv1d + BN + max-pool: maps 75 x 750 instead of 150 x 1500)
VARIANTS = {"L": dict(learn_features=False, proj_mlp=False, frames_conv=False),
            "LE": dict(learn_features=True, proj_mlp=True, frames_conv=False),
            "LEF": dict(learn_features=True, proj_mlp=True, frames_conv=True)}


def kws_hparams(variant: str, D: int, threshold: float, **extra) -> dict:
    """KWSModel init_args of the bench's spotter (train-LEF.yaml:168-209 with the variant's switches)."""
    return dict(n_layers=3, embedding_dim=D, proj_mlp_units=64, resnet_version="resnet-50", threshold=threshold,
                **VARIANTS[variant], **extra)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def keyword_hs(K: int, D: int, dev, Tk: int = 150, seed: int = 1234, chunk: int = 250):
    """The seeded synthetic keyword database in chunks: per-frame L2-normalised N(0,1) hs [kc, 3, Tk, D], ragged
    lengths U{8..150}, zero padding and 0/1 masks [kc, 3, Tk] as efficient_kws/dataset.py:1767-1796.  Yields
    (first keyword, generator of the chunk) so callers can skip chunks outside a shard without drawing them
    differently: the random stream is the same for every K and shard."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    for k0 in range(0, K, chunk):
        kc = min(chunk, K - k0)
        x = torch.randn((kc, 3, Tk, D), generator=g, device=dev)
        x = x / x.norm(dim=-1, keepdim=True)
        lens = torch.randint(8, Tk + 1, (kc,), generator=g, device=dev)
        m = (torch.arange(Tk, device=dev)[None, :] < lens[:, None]).float()
        m = m[:, None, :].expand(kc, 3, Tk).contiguous()
        yield k0, x * m[..., None], m


def build_keyword_db(kws, K: int, D: int, Tk: int = 150, seed: int = 1234, chunk: int = 250, lo: int = 0,
                     hi: int | None = None, f32: bool = False):
    """keyword_hs projected once through the LEF projector -> bf16 [K, 3, 75, 64], masks [K, 3, 75]
    (+ the fp32 projection [K, 3, 75, 64] the exact re-scoring band reads, when ``f32``).
    The database is always the same seeded K keywords; [lo, hi) selects a shard of it
    (keyword-sharded ranks), so a sharded run scores exactly the keywords of N = 1."""
    hi = K if hi is None else hi
    feats, masks, f32s = [], [], []
    for k0, x, m in keyword_hs(K, D, kws.device, Tk, seed, chunk):
        if k0 >= hi:
            break
        a, b = max(lo, k0), min(hi, k0 + x.shape[0])
        if a >= b:
            continue
        x = x[a - k0:b - k0].contiguous()
        m = m[a - k0:b - k0].contiguous()
        pk, pm = kws.project(x, m)
        feats.append(pk)
        masks.append(pm)
        if f32:
            f32s.append(kws.project_f32(x, m)[0])
        del x
    out = (torch.cat(feats, 0), torch.cat(masks, 0))
    return out + (torch.cat(f32s, 0),) if f32 else out


def _rank_device(local_rank: int) -> torch.device:
    """One GPU per rank (LOCAL_RANK).  CBW_BENCH_DEVICE=i pins every rank to GPU i: a rehearsal of the N-rank code
    path on a one-GPU box (with CBW_BENCH_DIST=gloo; RCCL refuses two ranks on one device) -- never for numbers."""
    pin = os.environ.get("CBW_BENCH_DEVICE")
    idx = int(pin) if pin is not None else local_rank
    torch.cuda.set_device(idx)
    return torch.device(f"cuda:{idx}")


def _init_dist(dist, dev):
    """RCCL ("nccl") process group, one process per GPU; CBW_BENCH_DIST=gloo only for the one-GPU rehearsal."""
    backend = os.environ.get("CBW_BENCH_DIST", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)


def rank_times(dist, elapsed: float, dev) -> tuple:
    """The timed region's length on every rank (all-gather) and its max, the job's time (every rank has started
    after the common barrier and the job ends with the slowest rank)."""
    if dist is None:
        return elapsed, [elapsed]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    allt = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(allt, t)
    per = [float(x.item()) for x in allt]
    return max(per), per


def calibrate_kws(kws, enc, ids, n_mel: int, K: int, D: int, n_cal: int, dev):
    """Setup-time bias / logit-offset calibration of the bf16 scoring pass (KwsEngine.calibrate_bias):
    a clip outside the timed ones (id 999 999) against the database's first ``n_cal`` keywords, so every rank
    (keyword-sharded or not, clip-parallel or long-form) calibrates on the same pairs."""
    from cbw.whisper import log_mel
    from cbw import synth
    _, mel_pk = log_mel(torch.from_numpy(synth.synth_clip(999_999)).to(dev), n_mel, packed=True)
    hs = enc.hidden_states(mel_pk, ids, normalize=True)
    um = torch.ones((1, len(ids), hs.shape[-2]), device=dev)
    cu32, _ = kws.project_f32(hs, um)
    cu, cum = kws.project(hs, um)
    cdb, cdbm, cdb32 = build_keyword_db(kws, K, D, lo=0, hi=min(n_cal, K), f32=True)
    kws.calibrate_bias(cu32[0], cum[0], cdb32, cdbm, utt=cu[0], kwd=cdb)
    torch.cuda.synchronize()


def _calibration_pairs(kws, enc, ids, n_mel: int, K: int, D: int, lo: int, hi: int, dev):
    """The calibration clip (id 999 999, never timed) projected in bf16 and fp32, and keywords [lo, hi) of the
    database (bf16 + fp32 projections): (cu, cum, cu32, cdb, cdbm, cdb32)."""
    from cbw.whisper import log_mel
    from cbw import synth
    _, mel_pk = log_mel(torch.from_numpy(synth.synth_clip(999_999)).to(dev), n_mel, packed=True)
    hs = enc.hidden_states(mel_pk, ids, normalize=True)
    um = torch.ones((1, len(ids), hs.shape[-2]), device=dev)
    cu32, _ = kws.project_f32(hs, um)
    cu, cum = kws.project(hs, um)
    cdb, cdbm, cdb32 = build_keyword_db(kws, K, D, lo=lo, hi=min(hi, K), f32=True)
    return cu[0], cum[0], cu32[0], cdb, cdbm, cdb32


def _probs(lg):
    return torch.softmax(lg.double(), -1)[:, 1]


OP_POSITIVE_FRAC = {"realistic": 0.01, "sparse": 0.0015}   # operating point -> fraction of calibration pairs spotted


def realistic_bias_shift(kws, enc, ids, n_mel: int, K: int, D: int, dev, positive_frac: float = 0.01) -> float:
    """The realistic operating point: the seeded classifier puts probabilities around 0.5 (a
    third of all keywords spotted per clip); a trained spotter on a real keyword list spots few.  The shift
    delta = the (1 - positive_frac) quantile of the fp32 logit difference l1 - l0 over the calibration pairs
    (the database's first 512 keywords vs the calibration clip); subtracting it from the classifier's class-1 bias
    leaves ~positive_frac of the pairs above the 0.5 threshold."""
    cu, cum, cu32, cdb, cdbm, cdb32 = _calibration_pairs(kws, enc, ids, n_mel, K, D, 0, 512, dev)
    l32 = torch.empty((cdb.shape[0], 2), dtype=torch.float32, device=dev)
    kws.rescore(cu32, cum, cdb32, cdbm, l32, torch.arange(cdb.shape[0], dtype=torch.int32, device=dev))
    d = (l32[:, 1] - l32[:, 0]).double().cpu().numpy()
    return float(np.quantile(d, 1.0 - positive_frac))


def calibrate_fp8_tier(kws, enc, ids, n_mel: int, K: int, D: int, dev, margin: float = 1.0):
    """The fp8 first tier's setup: scales + weights from the fp32 network over the calibration pairs (first 512
    keywords vs the calibration clip) and its logit offset, then its band: 1.5 x the largest |p_fp8 - p_fp32| over
    held-out pairs (keywords 512..1535 vs the same clip).  Returns (band, measured max error, held-out pairs)."""
    cu, cum, cu32, cdb, cdbm, cdb32 = _calibration_pairs(kws, enc, ids, n_mel, K, D, 0, 512, dev)
    kws.calibrate_fp8(cu32, cum, cdb32, cdbm, margin=margin, utt=cu, kwd=cdb)
    if K <= 512:
        hu, hum, hu32, hdb, hdbm, hdb32 = cu, cum, cu32, cdb, cdbm, cdb32
    else:
        hu, hum, hu32, hdb, hdbm, hdb32 = _calibration_pairs(kws, enc, ids, n_mel, K, D, 512, 1536, dev)
    l8 = kws.score_fp8(hu, hum, hdb, hdbm)
    l32 = torch.empty_like(l8)
    kws.rescore(hu32, hum, hdb32, hdbm, l32, torch.arange(hdb.shape[0], dtype=torch.int32, device=dev))
    err = float((_probs(l8) - _probs(l32)).abs().max())
    torch.cuda.synchronize()
    return min(0.49, 1.5 * err), err, int(hdb.shape[0])
