#!/usr/bin/env python
"""bench.py — CB-Whisper keyword-spotting path on MI355X (BASELINE.json metric).

One step = one synthetic 30 s clip through the whole hot path, inputs resident
in HBM: log-mel (128 bins) -> Whisper-large-v3 encoder (all 32 layers,
hidden_states[10:22][-3:] = states 19..21, per-frame L2 norm) -> LEF utterance
projection -> masked cosine-similarity maps against a 10 000-keyword LEF
database -> ResNet-50 classifier -> spotted-keyword decision.  The keyword
database is projected once before timing (keyword-side
projections are amortised per database).  Weights are seeded random
(cbw.synth; no checkpoints offline), data synthetic.

Clip pipeline (default; --no-pipeline turns it off): clip i+1's front end (mel, encoder,
utterance projection) runs on a second HIP stream while clip i is scored; every timed
step still carries one whole clip through the whole path.

Multi-GPU (torchrun, one process per GPU): clip-parallel — every rank scores its
own clips against the full keyword database; no data-path collective, only the
timing barrier and a max-reduce of the elapsed time ("scaling": "weak").

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "utterances/sec (30 s clips) + keywords/sec matched, Whisper-large-v3 LEF 10k kw"
RESNET50_GFLOP_LEF = 10.08   # per pair at [3, 75, 750] (FlopCounterMode)
SIM_GFLOP_LEF = 0.0216


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def build_keyword_db(kws, K: int, D: int, Tk: int = 150, seed: int = 1234, chunk: int = 250, lo: int = 0,
                     hi: int | None = None, f32: bool = False):
    """Synthetic keyword hs (per-frame L2-normalised N(0,1), ragged lengths
    U{8..150}, zero padding + 0/1 masks as efficient_kws/dataset.py:1767-1796)
    projected once through the LEF projector -> bf16 [K, 3, 75, 64], masks [K, 3, 75]
    (+ the fp32 projection [K, 3, 75, 64] the exact re-scoring band reads, when ``f32``).
    The database is always the same seeded K keywords; [lo, hi) selects a shard of it
    (keyword-sharded ranks), so a sharded run scores exactly the keywords of N = 1."""
    hi = K if hi is None else hi
    dev = kws.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    feats, masks, f32s = [], [], []
    for k0 in range(0, K, chunk):
        kc = min(chunk, K - k0)
        x = torch.randn((kc, 3, Tk, D), generator=g, device=dev)
        x = x / x.norm(dim=-1, keepdim=True)
        lens = torch.randint(8, Tk + 1, (kc,), generator=g, device=dev)
        a, b = max(lo, k0), min(hi, k0 + kc)
        if a >= b:
            del x
            continue
        m = (torch.arange(Tk, device=dev)[None, :] < lens[:, None]).float()
        m = m[:, None, :].expand(kc, 3, Tk).contiguous()
        x = (x * m[..., None])[a - k0:b - k0].contiguous()
        m = m[a - k0:b - k0].contiguous()
        pk, pm = kws.project(x, m)
        feats.append(pk)
        masks.append(pm)
        if f32:
            f32s.append(kws.project_f32(x, m)[0])
        del x
    out = (torch.cat(feats, 0), torch.cat(masks, 0))
    return out + (torch.cat(f32s, 0),) if f32 else out


def cpu_baseline(enc_sd, kws_sd, kws_hp, clip: np.ndarray, K: int, enc_cfg):
    """Oracle (numpy port of the reference path, oracle/) on this host's cores, on a
    bounded sample (~10 s): mel of one clip, encoder front + 1 and 5 layers (per-layer
    cost by difference, extrapolated to 32), LEF forward for 4 and 32 keywords (per-pair
    cost by difference, extrapolated to K)."""
    import oracle.encoder as oenc
    import oracle.kws as okws
    import oracle.mel as omel
    from cbw import synth
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n_mel, D, n_layers, n_heads, _ = enc_cfg
    t0 = time.perf_counter()
    mel = omel.log_mel(clip, n_mel)
    t_mel = time.perf_counter() - t0

    def enc_time(nl):
        sd = {k: v for k, v in enc_sd.items() if not k.startswith("layers.") or int(k.split(".")[1]) < nl}
        t = time.perf_counter()
        oenc.encoder_hidden_states(sd, mel, n_heads)
        return time.perf_counter() - t

    t1, t5 = enc_time(1), enc_time(5)
    per_layer = max(0.0, (t5 - t1) / 4)
    t_enc = (t1 - per_layer) + n_layers * per_layer

    def kws_time(k):
        b = synth.synth_kws_batch(seed=7, K=k, n_layers=3, D=D, utt_len=1500)
        t = time.perf_counter()
        okws.kws_forward(kws_sd, kws_hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], return_features=False)
        return time.perf_counter() - t

    k4, k32 = kws_time(4), kws_time(32)
    per_pair = max(1e-9, (k32 - k4) / 28)
    t_utt_proj = max(0.0, k4 - 4 * per_pair)
    total = t_mel + t_enc + t_utt_proj + K * per_pair
    wall = time.perf_counter() - t0
    return {"value": 1.0 / total, "unit": "utterances/s", "cores": int(threads), "kind": "port",
            "sample": (f"numpy oracle (oracle/), {wall:.1f} s of CPU work: mel of 1 clip ({t_mel:.2f} s); encoder front "
                       f"+1 and +5 layers -> {per_layer:.2f} s/layer x {n_layers} ({t_enc:.1f} s); LEF forward of 4 and 32 "
                       f"keywords -> {per_pair*1e3:.0f} ms/pair x {K} ({K*per_pair:.0f} s); per-utterance total "
                       f"{total:.1f} s"),
            "pairs_per_s": K / total}


def _pmc_traffic():
    """Fabric-side bytes per conv launch from the last committed PMC pass (profiles/pmc_conv_latest.json:
    rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes of this bench, FETCH_SIZE doubled per the
    gfx950 correction).  bench.py cannot collect counters itself; None when no summary is committed."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_conv_latest.json")) as f:
            return round(json.load(f)["bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--keywords", type=int, default=10000)
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--chunk", type=int, default=625,
                    help="keyword pairs per ResNet chunk (625 = 16 even chunks of the 10k database: 5.75 vs 5.71 "
                         "utt/s at 500, 5.54 at 400, 5.72 at 1000)")
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--exact-band", type=float, default=0.03,
                    help="re-score in fp32 every pair whose bf16 probability lies within this distance of the "
                         "threshold (inside the timed step), so the spotted indices are those of the reference's "
                         "fp32 evaluation; 0 = bf16 decisions only.  0.03 > the largest bf16-vs-fp32 probability "
                         "error measured at this operating point (0.024, tools/band_stats.py)")
    ap.add_argument("--x3-band", type=float, default=1e-4,
                    help="two-tier re-scoring: the pairs within --exact-band go through the compensated-bf16 tier "
                         "(cbw_kws_rescore_x3, max |p - p_fp32| 2.5e-5 measured) and only those then within this "
                         "distance of the threshold through fp32; <= 0: every band pair in fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-launch HIP-event roofline timing")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="run each clip's front end (mel, encoder, utterance projection) on the main stream before its "
                         "scoring; by default clip i+1's front end runs on a second stream while clip i is scored "
                         "(+1.8 %% utt/s: the encoder's few-tile GEMMs leave CUs the scoring convs use)")
    ap.add_argument("--mode", choices=["clip", "kwshard"], default="clip",
                    help="clip: every rank scores its own clips vs all keywords (weak scaling); kwshard: one clip "
                         "per step, keywords sharded over ranks, RCCL broadcast + all-gather (strong scaling, C4)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from cbw import synth, _lib
    from cbw.kws import KwsEngine
    from cbw.whisper import EncoderEngine, default_layer_ids, log_mel

    t_setup = time.time()
    enc_cfg = synth.WHISPER_CONFIGS[args.model]
    n_mel, D, n_layers, _, _ = enc_cfg
    enc_sd = synth.synth_whisper_encoder_state_dict(args.model, seed=0)
    enc = EncoderEngine(enc_cfg, enc_sd, dev)
    ids = default_layer_ids(n_layers)
    kws_hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True,
                  proj_mlp_units=64, resnet_version="resnet-50", threshold=args.threshold)
    kws_sd = synth.synth_kws_state_dict(seed=0, **kws_hp)
    kws = KwsEngine(kws_hp, kws_sd, dev)
    K = args.keywords
    sharded = args.mode == "kwshard" and world > 1
    band = float(args.exact_band)
    exact = band > 0
    rescored = [0, 0]
    x3_band = args.x3_band if args.x3_band and args.x3_band > 0 else None

    def score_db(u, um, u32, kd, km, kd32, out=None):
        """bf16 scores of every pair + the fp32 re-score of the near-threshold band (cbw_kws_band/rescore)."""
        if not exact:
            return kws.score(u, um, kd, km, chunk=args.chunk, logits_out=out)
        lg, st = kws.score_exact(u, um, kd, km, u32, kd32, args.threshold, band, chunk=args.chunk, logits_out=out,
                                 band_x3=x3_band)
        rescored[0] += st["band"]
        rescored[1] += st["fp32"]
        return lg

    if sharded:
        from cbw.parallel import KeywordShardedSpotter, shard_range
        lo, hi = shard_range(K, rank, world)
        db, dbm, *db32 = build_keyword_db(kws, K, D, lo=lo, hi=hi, f32=exact)   # this rank's slice of the same DB
        db32 = db32[0] if exact else None
        spotter = KeywordShardedSpotter(K, db, dbm, lambda u, um, kd, km: score_db(u, um, u32_shared[0], kd, km, db32))
    else:
        db, dbm, *db32 = build_keyword_db(kws, K, D, f32=exact)
        db32 = db32[0] if exact else None
    u32_shared = [None]
    n_clips = args.warmup + args.steps
    clips = [torch.from_numpy(synth.synth_clip(1000 * rank + i)).to(dev) for i in range(n_clips)]
    utt_mask = torch.ones((1, 3, 1500), device=dev)
    hs = torch.empty((1, 3, 1500, D), dtype=torch.float32, device=dev)
    logits = torch.empty((K, 2), dtype=torch.float32, device=dev)
    prob = torch.empty((K,), dtype=torch.float32, device=dev)
    idx = torch.empty((K,), dtype=torch.int32, device=dev)
    nspot = torch.zeros((1,), dtype=torch.int32, device=dev)
    lib = _lib.load()
    torch.cuda.synchronize()
    log(f"[bench] setup {time.time() - t_setup:.1f} s: {args.model} encoder + LEF/resnet-50, K={K}, db "
        f"{tuple(db.shape)}")

    def project_utt(h):
        pu, pum = kws.project(h, utt_mask)
        pu32 = kws.project_f32(h, utt_mask)[0][0] if exact else None
        return pu, pum, pu32

    def step(i):
        if sharded:
            pu = pum = pu32 = None
            if rank == 0:
                _, mel_pk = log_mel(clips[i], n_mel, packed=True)
                enc.hidden_states(mel_pk, ids, normalize=True, out=hs)
                pu, pum, pu32 = project_utt(hs)
                pu, pum = pu[0], pum[0]
            u, um = spotter.broadcast_utterance(pu, pum, (3, 750, 64), (3, 750), torch.bfloat16, dev)
            if exact:   # the fp32 utterance projection travels with the bf16 one (576 KB)
                u32_shared[0] = spotter.broadcast_tensor(pu32, (3, 750, 64), torch.float32, dev)
            logits.copy_(spotter.score(u, um))
        else:
            _, mel_pk = log_mel(clips[i], n_mel, packed=True)
            enc.hidden_states(mel_pk, ids, normalize=True, out=hs)
            pu, pum, pu32 = project_utt(hs)
            score_db(pu[0], pum[0], pu32, db, dbm, db32, out=logits)
        _lib.check(lib.cbw_kws_spot(logits.data_ptr(), None, K, float(args.threshold), 0, prob.data_ptr(),
                                    idx.data_ptr(), nspot.data_ptr(), _lib.stream_handle()), "cbw_kws_spot")

    # clip pipeline (clip-parallel mode): clip i+1's front end (mel -> encoder -> utterance projection,
    # few-tile GEMMs) runs on its own stream while clip i's keyword scoring runs on the main stream;
    # every clip still passes through the whole path, the GPU's idle slots of one overlap the other
    pipeline = args.pipeline and not sharded
    front_stream = torch.cuda.Stream(device=dev) if pipeline else None
    hs_buf = [hs, torch.empty_like(hs)]

    def front(i):
        main = torch.cuda.current_stream()
        front_stream.wait_stream(main)
        with torch.cuda.stream(front_stream):
            _, mel_pk = log_mel(clips[i], n_mel, packed=True)
            h = hs_buf[i % 2]
            enc.hidden_states(mel_pk, ids, normalize=True, out=h)
            pu, pum, pu32 = project_utt(h)
            ev = torch.cuda.Event()
            ev.record(front_stream)
        for t in (pu, pum, pu32):
            if t is not None:
                t.record_stream(main)
        return pu, pum, pu32, ev

    def run_steps(first, n):
        if not pipeline:
            for i in range(first, first + n):
                step(i)
            return
        nxt = front(first)
        for i in range(first, first + n):
            pu, pum, pu32, ev = nxt
            if i + 1 < first + n:
                nxt = front(i + 1)
            torch.cuda.current_stream().wait_event(ev)
            score_db(pu[0], pum[0], pu32, db, dbm, db32, out=logits)
            _lib.check(lib.cbw_kws_spot(logits.data_ptr(), None, K, float(args.threshold), 0, prob.data_ptr(),
                                        idx.data_ptr(), nspot.data_ptr(), _lib.stream_handle()), "cbw_kws_spot")

    run_steps(0, args.warmup)
    # phase breakdown on one warm step (torch events: libcbw launches on torch's current stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    ev[0].record()
    _, mel_pk = log_mel(clips[0], n_mel, packed=True)
    ev[1].record()
    enc.hidden_states(mel_pk, ids, normalize=True, out=hs)
    ev[2].record()
    pu, pum, pu32 = project_utt(hs)
    ev[3].record()
    kws.score(pu[0], pum[0], db, dbm, chunk=args.chunk, logits_out=logits)
    ev[4].record()
    n_band = 0
    if exact:
        _, st = kws.score_exact(pu[0], pum[0], db, dbm, pu32, db32, args.threshold, band, chunk=args.chunk,
                                logits_out=logits, band_x3=x3_band)
        n_band = st["band"]
    ev[5].record()
    torch.cuda.synchronize()
    breakdown = {"mel": ev[0].elapsed_time(ev[1]), "encoder": ev[1].elapsed_time(ev[2]),
                 "utt_projection": ev[2].elapsed_time(ev[3]), "kws_score": ev[3].elapsed_time(ev[4]),
                 "band_rescore": ev[4].elapsed_time(ev[5]) - ev[3].elapsed_time(ev[4]), "band_pairs": n_band}

    n_conv_per_step = ((K + args.chunk - 1) // args.chunk) * 53
    if not args.no_profile:
        _lib.check(lib.cbw_kws_profile(kws.h, n_conv_per_step * args.steps + 16), "cbw_kws_profile")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    rescored[0] = rescored[1] = 0
    t0 = time.perf_counter()
    run_steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    conv_ms = ctypes.c_double()
    conv_flop = ctypes.c_double()
    conv_n = ctypes.c_int()
    if not args.no_profile:
        _lib.check(lib.cbw_kws_profile_read(kws.h, ctypes.byref(conv_ms), ctypes.byref(conv_flop),
                                            ctypes.byref(conv_n)), "cbw_kws_profile_read")
        lib.cbw_kws_profile(kws.h, 0)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    utts = args.steps * (1 if sharded else world)
    value = utts / elapsed
    n_spotted = int(nspot.item())

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 4), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded 30 s clips, seeded random weights, 10k synthetic keyword hs)",
            "config": {"workload": f"whisper-{args.model} encoder + efficient_kws LEF (resnet-50) vs {K} keywords, "
                                   f"one 30 s clip per step per GPU",
                       "keywords": K, "clips_per_step": 1 if sharded else world, "utterance_frames": 1500, "keyword_frames": 150,
                       "hs_layers": ids, "chunk": args.chunk, "parallelism": (f"keyword-sharded x{world} (RCCL broadcast + all-gather)" if sharded
                                       else f"clip-parallel x{world}"),
                       "clip_pipeline": pipeline},
            "pairs_per_s": round(value * K, 1),
            "breakdown_ms": {k: round(v, 3) for k, v in breakdown.items()},
            "spotted_last_clip": n_spotted,
            "exact_band": band, "x3_band": x3_band,
            "rescored_pairs_per_step": round(rescored[0] / args.steps, 1),
            "fp32_rescored_pairs_per_step": round(rescored[1] / args.steps, 1),
            "decisions": ("bf16 scores; pairs within exact_band of the threshold re-scored inside the timed step "
                          "(compensated-bf16 tier, then those within x3_band in fp32-input MFMA), so spotted indices "
                          "follow the reference's fp32 evaluation"
                          if exact else "bf16 scores only (decisions within ~0.03 of the threshold may differ "
                                        "from fp32)"),
        }
        if not args.no_profile and conv_n.value > 0:
            achieved = conv_flop.value / (conv_ms.value * 1e-3) / 1e12
            rec["roofline"] = {"bound": "mfma", "achieved": round(achieved, 2), "peak": 2500.0, "unit": "TFLOP/s",
                               "frac": round(achieved / 2500.0, 4), "traffic": _pmc_traffic(),
                               "kernel": "ResNet-50 conv family: conv_igemm* + conv_ring + conv_stream + bottleneck_s1 (bf16 MFMA 16x16x32); "
                                         "achieved = algorithmic FLOPs / union of launch intervals",
                               "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                               "profiles/pmc_conv_latest.json)",
                               "launches": conv_n.value, "kernel_ms_per_step": round(conv_ms.value / args.steps, 3),
                               "algorithmic_tflop_per_step": round(conv_flop.value / args.steps / 1e12, 3)}
        if world == 1 and not args.no_cpu_baseline:
            try:
                rec["cpu_baseline"] = cpu_baseline(enc_sd, kws_sd, kws_hp, synth.synth_clip(0), K, enc_cfg)
            except Exception as e:  # the GPU result stands on its own
                rec["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
