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
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "utterances/sec (30 s clips) + keywords/sec matched, Whisper-large-v3 LEF 10k kw"
# efficient_kws variants (efficient_kws/model.py:71-124): L = ResNet on raw-hs
# similarities (learn_features False, the reference's working L form), LE = per-layer MLP
# projector, LEF = LE + the time projector (conv1d + BN + max-pool: maps 75 x 750 instead of 150 x 1500)
VARIANTS = {"L": dict(learn_features=False, proj_mlp=False, frames_conv=False),
            "LE": dict(learn_features=True, proj_mlp=True, frames_conv=False),
            "LEF": dict(learn_features=True, proj_mlp=True, frames_conv=True)}
# ResNet-50 GFLOP per pair (BASELINE.md / SURVEY §6, FlopCounterMode): LEF maps [3, 75, 750], L / LE [3, 150, 1500]
RESNET50_GFLOP = {"L": 38.25, "LE": 38.25, "LEF": 10.08}


def kws_hparams(variant: str, D: int, threshold: float, **extra) -> dict:
    """KWSModel init_args of the bench's spotter (train-LEF.yaml:168-209 with the variant's switches)."""
    return dict(n_layers=3, embedding_dim=D, proj_mlp_units=64, resnet_version="resnet-50", threshold=threshold,
                **VARIANTS[variant], **extra)


def workload_metric(model: str, variant: str, K: int) -> str:
    """BASELINE.json's metric for the headline config; the same metric named for the other configs"""
    if (model, variant, K) == ("large-v3", "LEF", 10000):
        return METRIC
    return f"utterances/sec (30 s clips) + keywords/sec matched, Whisper-{model} {variant} {K} kw"


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


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(enc_sd, kws_sd, kws_hp, clip: np.ndarray, K: int, enc_cfg):
    """The reference path in torch fp32 on this host's cores (oracle/torch_ref.py: the torch ops the reference
    calls -- torch.stft mel, HF-eager encoder, efficient_kws KWSModel.forward with F.conv2d / BN-eval ResNet-50,
    groups of 50 keywords), on a bounded sample: mel of one clip, encoder front + 1 and + 3 layers (per-layer
    cost by difference, extrapolated to all layers), LEF forward of 8 and 108 keywords (per-pair cost by
    difference, extrapolated to K)."""
    import oracle.torch_ref as tref
    from cbw import synth
    threads = torch.get_num_threads()
    n_mel, D, n_layers, n_heads, _ = enc_cfg
    t0 = time.perf_counter()
    with torch.inference_mode():
        mel = tref.log_mel(clip, n_mel)
        t_mel = time.perf_counter() - t0

        def enc_time(nl):
            t = time.perf_counter()
            tref.encoder_hidden_states(enc_sd, mel, n_heads, n_layers=nl)
            return time.perf_counter() - t

        enc_time(1)   # warm-up (first-call allocations)
        t1, t3 = enc_time(1), enc_time(3)
    per_layer = max(0.0, (t3 - t1) / 2)
    t_enc = (t1 - per_layer) + n_layers * per_layer

    def kws_time(k):
        b = synth.synth_kws_batch(seed=7, K=k, n_layers=3, D=D, utt_len=1500)
        t = time.perf_counter()
        tref.kws_forward(kws_sd, kws_hp, b["kwd"], b["utt"], b["kwd_mask"], b["utt_mask"], group=50)
        return time.perf_counter() - t

    k_lo, k_hi = 8, 108
    kws_time(2)   # warm-up
    a, b = kws_time(k_lo), kws_time(k_hi)
    per_pair = max(1e-9, (b - a) / (k_hi - k_lo))
    t_utt_proj = max(0.0, a - k_lo * per_pair)
    total = t_mel + t_enc + t_utt_proj + K * per_pair
    wall = time.perf_counter() - t0
    return {"value": 1.0 / total, "unit": "utterances/s", "cores": int(threads), "kind": "port",
            "cpu": _cpu_model(),
            "sample": (f"torch fp32 restatement of the reference path (oracle/torch_ref.py), {torch.get_num_threads()} "
                       f"intra-op threads, {wall:.1f} s of CPU work: mel of 1 clip ({t_mel:.2f} s); encoder front +1 "
                       f"and +3 layers -> {per_layer:.3f} s/layer x {n_layers} ({t_enc:.1f} s); LEF forward of {k_lo} "
                       f"and {k_hi} keywords in groups of 50 -> {per_pair * 1e3:.1f} ms/pair x {K} ({K * per_pair:.0f} "
                       f"s); per-utterance total {total:.1f} s"),
            "pairs_per_s": K / total}


def _union_ms(starts, ends):
    """Total length of the union of [start, end] intervals."""
    tot, cs, ce = 0.0, None, None
    for a, b in sorted(zip(starts.tolist(), ends.tolist())):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + (ce - cs if ce is not None else 0.0)


def _pmc_traffic():
    """Fabric-side bytes per conv launch and per step from the last committed PMC passes
    (profiles/pmc_conv_latest.json: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes of this bench,
    cut to the timed region and to the KWS conv family by tools/roofline_from_trace.py, FETCH_SIZE doubled per
    the gfx950 correction).  bench.py cannot collect counters itself; (None, None) when no summary is committed."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_conv_latest.json")) as f:
            d = json.load(f)
        return round(d["bytes_per_launch"]), round(d.get("bytes_per_step", 0)) or None
    except (OSError, ValueError, KeyError):
        return None, None


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


def launch_ranks(gpus: int, argv: list) -> int | None:
    """--gpus N against the launched world.  Under torchrun (WORLD_SIZE set) the world must be
    N.  Without it and N > 1 this process starts the N ranks itself -- one torchrun child (127.0.0.1 rendezvous, a free
    port) running this script with the same arguments -- before anything touches the GPU, waits for it and returns its
    exit code; N = 1 (or a world set by the caller) returns None: run here."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return None
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if gpus == 1:
        return None
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    log(f"[bench] --gpus {gpus}: starting {gpus} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.run(cmd).returncode


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


def run_plumbing(args):
    """--plumbing (test only, no GPU): the multi-rank envelope of the clip bench on the CPU -- gloo group, barrier,
    K timed steps, barrier, all-gather of every rank's elapsed time, max over ranks, rank 0's JSON line.  A step is a
    sleep of (rank + 1) x --plumbing-ms, so the slowest rank is known; nothing here measures the hot path."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch.distributed as dist
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29543")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("gloo")
    dev = torch.device("cpu")
    step_s = (rank + 1) * args.plumbing_ms * 1e-3
    for _ in range(args.warmup):
        time.sleep(step_s)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(step_s)
    dist.barrier()
    elapsed, per = rank_times(dist, time.perf_counter() - t0, dev)
    if rank == 0:
        print(json.dumps({"metric": "plumbing (no hot path)", "value": round(world * args.steps / elapsed, 4),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "none", "data": "none",
                          "config": {"workload": "plumbing"},
                          "rank_elapsed_s": [round(x, 6) for x in per]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


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


TRACE_TAG = "r06n"  # the committed in-bench trace of this commit (tools/roofline_from_trace.py input)


def per_kernel_table(names, start_ms, end_ms, flop, tier, steps: int, peak_tflops: float = 2500.0) -> list:
    """In-bench per-kernel roofline table from the runtime's per-launch records (hipEvents on the launch's stream,
    cbw_kws_profile_kernels' kernel names): per (tier, kernel) the launches per step, the
    average launch duration, the algorithmic GFLOP per launch (2 M N K of the conv it ran) and the fraction of
    the dense bf16 MFMA peak that rate is (algorithmic FLOP / average duration / 2.5 PFLOP/s), sorted by time."""
    tiers = {0: "bf16_scoring", 1: "compensated_rescoring", 2: "fp8_first_tier"}
    acc = {}
    for nm, a, b, f, t in zip(names, start_ms, end_ms, flop, tier):
        k = (int(t), nm)
        e = acc.setdefault(k, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += float(b - a)
        e[2] += float(f)
    rows = []
    for (t, nm), (c, ms, f) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        avg_us = ms / c * 1e3
        gf = f / c / 1e9
        rows.append({"tier": tiers.get(t, str(t)), "kernel": nm, "launches_per_step": round(c / steps, 2),
                     "ms_per_step": round(ms / steps, 3), "avg_us": round(avg_us, 1), "gflop_per_launch": round(gf, 2),
                     "frac": round(gf * 1e9 / (avg_us * 1e-6) / 1e12 / peak_tflops, 4) if avg_us > 0 else None})
    return rows


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


def _isolated_per_kernel(dominant):
    """The committed profile set's per-kernel table with each launch alone on the GPU (profiles/{TRACE_TAG}_roofline.json
    per_kernel_isolated: the FETCH_SIZE pass serialises the kernels) beside the in-bench one, where three scoring
    streams share the CUs: the dominant kernel's isolated fraction and the bf16 tier's top rows."""
    try:   # profiles/isolated_latest.json: that table, written by tools/pmc_latest.py (profiles/r0* stays off the box)
        with open(os.path.join(REPO, "profiles", "isolated_latest.json")) as f:
            rows = json.load(f).get("per_kernel_isolated") or []
    except (OSError, ValueError):
        return None
    bf = [r for r in rows if r.get("tier") == "bf16_scoring"]
    if not bf:
        return None
    dom = next((r for r in bf if dominant and r.get("kernel") == dominant.get("kernel")), None)
    return {"dominant_kernel_isolated": dom, "per_kernel_isolated": bf[:10],
            "per_kernel_isolated_source": f"profiles/{TRACE_TAG}_roofline.json (rocprofv3 --pmc FETCH_SIZE pass of "
                                          "this configuration: durations with the kernels serialised)"}


def _child_bench(extra: list, timeout: int = 420, steps: int = 5, warmup: int = 1):
    """This bench as a child process (its own GPU setup, 5 timed steps) -> (its JSON line or None, error text)."""
    import subprocess
    import threading
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(steps), "--warmup", str(warmup),
           "--no-cpu-baseline", "--no-companions", *extra]
    log(f"[bench] companion: {' '.join(extra)}")
    t0 = time.time()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    err_lines = []

    def relay():   # the child's progress lines as they come (a silent parent for minutes looks hung)
        for line in p.stderr:
            err_lines.append(line)
            if line.startswith("[bench]"):
                log("    " + line.rstrip())
    out_parts = []
    readers = [threading.Thread(target=relay, daemon=True),
               threading.Thread(target=lambda: out_parts.append(p.stdout.read()), daemon=True)]
    for t in readers:
        t.start()
    try:
        p.wait(timeout=timeout)
    except subprocess.TimeoutExpired as e:
        p.kill()
        p.wait()
        return None, type(e).__name__
    for t in readers:
        t.join(timeout=10)
    log(f"[bench] companion done in {time.time() - t0:.0f} s (rc {p.returncode})")
    try:
        if p.returncode == 0:
            return json.loads("".join(out_parts).strip().splitlines()[-1]), None
        tail = "".join(err_lines).strip()
        return None, f"rc {p.returncode}: {tail.splitlines()[-1] if tail else ''}"
    except (ValueError, IndexError) as e:
        return None, type(e).__name__


def companion_runs(args) -> dict:
    """The fp8 first tier (C5) beside the headline line: this bench at the realistic operating point with and
    without --fp8-first (same clips, same K, 5 timed steps each), as child processes (each its own GPU setup), and
    the fp8-first run at this (synthetic) point.  Their values are not the headline `value`."""
    out = {}
    base = ["--keywords", str(args.keywords), "--model", args.model, "--chunk", str(args.chunk)]
    for tag, extra in (("realistic_bf16", ["--operating-point", "realistic"]),
                       ("realistic_fp8_first", ["--operating-point", "realistic", "--fp8-first"]),
                       ("synthetic_fp8_first", ["--fp8-first"])):
        d, err = _child_bench(base + extra)
        if d is None:
            out[tag] = {"error": err}
            continue
        out[tag] = {k: d.get(k) for k in ("value", "ms_per_step", "spotted_last_clip", "spotted_digest",
                                          "bf16_pairs_per_step", "rescored_pairs_per_step", "audit_flips",
                                          "audit_max_bf16_err", "audit_max_fp8_err", "audit_fp8_band_margin",
                                          "fp8_first", "operating_point")}
        out[tag]["fp8_tier_union_ms_per_step"] = ((d.get("roofline") or {}).get("tiers") or {}).get(
            "fp8_first_tier", {}).get("union_ms_per_step")
    return out


# BASELINE.json configs[1] and configs[0]: the bench's own path at those models / variants /
# keyword counts, reported beside the headline (C1 is the reference's CPU plumbing config; here on the GPU)
CONFIG_COMPANIONS = (("C2", ["--model", "small", "--variant", "LE", "--keywords", "1000", "--chunk", "250"]),
                     ("C1", ["--model", "tiny.en", "--variant", "L", "--keywords", "32", "--chunk", "32"]))


def config_runs() -> dict:
    out = {}
    for tag, extra in CONFIG_COMPANIONS:
        d, err = _child_bench(extra)
        if d is None:
            out[tag] = {"error": err, "args": " ".join(extra)}
            continue
        rf = d.get("roofline") or {}
        out[tag] = {"metric": d.get("metric"), "args": " ".join(extra), "value": d.get("value"), "unit": d.get("unit"),
                    "ms_per_step": d.get("ms_per_step"), "pairs_per_s": d.get("pairs_per_s"),
                    "map_shape": (d.get("config") or {}).get("map_shape"),
                    "roofline": {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac",
                                                        "algorithmic_tflop_per_step", "kernel_ms_per_step")},
                    "breakdown_ms": d.get("breakdown_ms"), "spotted_last_clip": d.get("spotted_last_clip"),
                    "rescored_pairs_per_step": d.get("rescored_pairs_per_step"), "audit_flips": d.get("audit_flips"),
                    "audit_index_lists_equal": d.get("audit_index_lists_equal"),
                    "audit_max_bf16_err": d.get("audit_max_bf16_err"), "audit_band_margin": d.get("audit_band_margin")}
    return out


# end to end and C5 beside the headline: one 30 s clip through CBWhisper.forward (spotting ->
# keyword prompt -> 5-beam decode) in utt/s, and C5's long-form at 300 s (fp8-first spotting, realistic point) as four
# lanes of one audio each and as one lane of batched generate calls over the same four 300 s audios
E2E_COMPANIONS = (
    ("e2e_realistic", ["--mode", "e2e", "--operating-point", "realistic"], 5, 1),
    # ~15 keywords per clip, so the keyword prompt stays under the 224-token cut and the returned
    # transcript (pba_whisper.py:338's slice by the prompt length) is the decoded text, not empty
    ("e2e_short_prompt", ["--mode", "e2e", "--operating-point", "sparse"], 5, 1),
    # serving form: four clips in flight (a lane = stream + host thread + engines per clip), so one clip's spotting
    # fills the CUs another clip's latency-bound decode leaves idle (r06c: 1 / 2 / 4 in flight = 1.44 / 2.07 / 2.55)
    ("e2e_realistic_inflight4", ["--mode", "e2e", "--operating-point", "realistic", "--audios-in-flight", "4"], 5, 1),
    ("C5_longform_lanes4", ["--mode", "longform", "--audio-seconds", "300", "--audios-in-flight", "4", "--fp8-first",
                            "--operating-point", "realistic"], 1, 1),
    ("C5_longform_generate_batch4", ["--mode", "longform", "--audio-seconds", "300", "--generate-batch", "4",
                                     "--batch-length-step", "0", "--fp8-first", "--operating-point", "realistic"], 1, 1))


def end_to_end_runs() -> dict:
    out = {}
    for tag, extra, steps, warmup in E2E_COMPANIONS:
        d, err = _child_bench(extra, timeout=300, steps=steps, warmup=warmup)
        if d is None:
            out[tag] = {"error": err, "args": " ".join(extra)}
            continue
        keep = ("metric", "value", "unit", "ms_per_step", "ms_per_clip", "ms_per_window", "windows", "tokens_generated",
                "transcript_tokens", "spotted_keywords_per_clip", "spotted_keywords_per_window", "spotting_ms_per_clip",
                "spotting_ms_per_window", "transcript_digests")
        out[tag] = {"args": " ".join(extra), **{k: d[k] for k in keep if k in d}}
    a, b = out.get("C5_longform_lanes4", {}), out.get("C5_longform_generate_batch4", {})
    if "transcript_digests" in a and "transcript_digests" in b:
        # the same four 300 s audios; a batched call hands every window the union of its batch's spotted keywords
        # (the reference's aliased list, cb_whisper.py:89,129; CBWhisper segment_keywords="union") and left-pads the
        # prompts to the longest, pads attended (4.37.2), so its transcripts may differ from four separate
        # calls by design: this is reported, not asserted
        out["C5_lanes_vs_batch_digests_equal"] = sorted(a["transcript_digests"].values()) == \
            sorted(b["transcript_digests"].values())
    return out


def run_longform(args):
    """C5 (BASELINE.json configs[4]): PBAWhisper long-form + LEF keyword spotting, clip-parallel across audios.
    One step = one synthetic audio of --audio-seconds per rank through the whole path: long-form log-mel of the
    audio (cbw_mel_long), then PBAWhisper.generate's seek loop (pba_whisper.py:343-475; return_timestamps,
    condition_on_prev_tokens, num_beams 5 -- CBWhisper.forward's long-form arguments, cb_whisper.py:166-178):
    per 30 s window the CB-Whisper keyword spotter (large-v3 hs[19..21] -> LEF -> ResNet-50 against K keywords,
    exact-decision tiers) builds the <|startofprev|> prompt, the window is encoded and decoded with the
    timestamp rules, and the seek moves to the last closed segment.  The windows of one audio are sequential
    (the seek depends on the decoded timestamps); ranks process independent audios, no collective but the
    timing max.  value = audio seconds transcribed per second (whole job)."""
    import tempfile
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = _rank_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        _init_dist(dist, dev)
    from cbw import synth
    from cbw.kws import KwsEngine
    from cbw.tokenizer import WhisperTokenizerLite
    from cbw.whisper import log_mel_long
    from model.cb_whisper import CBWhisper
    from model.pba_whisper import PBAWhisper
    import threading
    t_setup = time.time()
    enc_cfg, dec_cfg = synth.WHISPER_CONFIGS[args.model], synth.WHISPER_DECODERS[args.model]
    n_mel, D = enc_cfg[0], enc_cfg[1]
    tokdir = tempfile.mkdtemp(prefix="cbw_tok_")
    synth.write_synth_tokenizer(tokdir, dec_cfg[0])
    K = args.keywords
    exact = args.exact_band > 0
    e2e = args.mode == "e2e"
    if e2e:   # one 30 s clip per step and lane: the short-form path CBWhisper.forward takes
        args.audio_seconds, args.generate_batch = 30.0, 1
    A = max(1, args.audios_in_flight)
    G = max(1, args.generate_batch)   # audios per PBAWhisper.generate call (pba_whisper.py:351-475, batch_size > 1)
    words = [synth.TOKENIZER_WORDS[i % len(synth.TOKENIZER_WORDS)] + str(i) for i in range(K)]
    gen_kw = dict(task="transcribe", language="english", return_timestamps=True, condition_on_prev_tokens=True,
                  return_segments=True, num_beams=args.beams, do_sample=False, temperature=0)
    if args.max_new_tokens:
        gen_kw["max_new_tokens"] = args.max_new_tokens

    class Lane:
        """One audio in flight: its own PBAWhisper + spotter engines (the decoder state, the KWS workspace and the
        calibrated biases are per engine), HIP stream and host thread.  The lanes of a rank share the GPU: the
        decode steps are latency-bound chains of small launches that leave most CUs idle, which another lane's
        launches (spotting, encoder or decode) fill."""

        def __init__(self, j):
            self.whisper = PBAWhisper(enc_cfg, dec_cfg, wsd, suppress_tokens=[1, 2, 7], device=dev,
                                      tokenizer=WhisperTokenizerLite.from_dir(tokdir))
            kws_hp = kws_hparams(args.variant, D, args.threshold)
            from cbw.whisper import default_layer_ids
            ids = default_layer_ids(enc_cfg[2])
            kws_sd = synth.synth_kws_state_dict(seed=0, **kws_hp)
            self.kws = KwsEngine(kws_hp, kws_sd, dev)
            if args.operating_point != "synthetic":   # the clip bench's realistic / sparse point (class-1 bias lowered)
                if op_shift[0] is None:
                    op_shift[0] = realistic_bias_shift(self.kws, self.whisper.encoder, ids, n_mel, K, D, dev,
                                                       OP_POSITIVE_FRAC[args.operating_point])
                kws_sd = dict(kws_sd)
                b = np.array(kws_sd["model.classifier.1.bias"], dtype=np.float32).copy()
                b[1] -= op_shift[0]
                kws_sd["model.classifier.1.bias"] = b
                del self.kws
                self.kws = KwsEngine(kws_hp, kws_sd, dev)
            db, dbm, *db32 = build_keyword_db(self.kws, K, D, f32=exact)
            if exact and args.bias_calibrate > 0:   # the same calibration as the clip bench (the spotter's hs[19..21])
                calibrate_kws(self.kws, self.whisper.encoder, ids, n_mel, K, D, args.bias_calibrate, dev)
            fp8_band = None
            if args.fp8_first:   # the e4m3 first tier in front of the bf16 pass (C5 "fp8 MFMA")
                if not exact:
                    raise SystemExit("--fp8-first runs the exact tiers after it (--exact-band > 0)")
                fp8_band, self.fp8_err, _ = calibrate_fp8_tier(self.kws, self.whisper.encoder, ids, n_mel, K, D, dev)
                fp8_cal[0] = {"fp8_band": round(fp8_band, 5), "fp8_max_err_held_out": round(self.fp8_err, 5)}
            self.cb = CBWhisper.from_components(self.whisper, self.kws, self.whisper.encoder, words, db, dbm,
                                                num_beams=args.beams, keyword_feats32=db32[0] if exact else None,
                                                exact_band=args.exact_band, fp8_band=fp8_band,
                                                keyword_prompt_prepend="The topic of today's speech is, ah, ",
                                                keyword_prompt_append=". Okay, then I'll continue.",
                                                keyword_separator=", ")
            # --lane-priority (with lanes): the lane's decode runs on a high-priority stream and its spotting on a
            # normal-priority one, so another lane's compute-bound spotting does not delay the latency-bound decode
            prio = args.lane_priority and A > 1
            self.stream = torch.cuda.Stream(device=dev, priority=-1 if prio else 0)
            self.spot_stream = torch.cuda.Stream(device=dev, priority=0) if prio else None
            self.stats = {"windows": 0, "tokens": 0, "spotted": 0, "spot_s": 0.0, "transcript_tokens": 0}
            self.digests = {}   # audio index -> sha1 of its transcript's token ids
            self.error = None
            spot0 = self.cb.keyword_spotting

            def spotting(input_features, start_of_prev=False):
                t = time.perf_counter()
                if self.spot_stream is not None:
                    self.spot_stream.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(self.spot_stream):
                        out = spot0(input_features, start_of_prev)
                    torch.cuda.current_stream().wait_stream(self.spot_stream)
                else:
                    out = spot0(input_features, start_of_prev)   # ends on the host (prompt ids): its wall time is its cost
                self.stats["spot_s"] += time.perf_counter() - t
                self.stats["windows"] += input_features.shape[0]
                self.stats["spotted"] += sum(len(k) for k in self.cb.last_spotted)
                if self.stats["windows"] % 10 == 0:   # progress (a 30 min audio is ~60 windows)
                    log(f"[bench] longform lane {j}: {self.stats['windows']} windows")
                return out
            self.gen_kw = dict(gen_kw, keyword_spotting=spotting)
            if e2e:   # CBWhisper.forward calls its own keyword_spotting: the counting wrapper stands in for it
                self.cb.keyword_spotting = spotting
                tok = self.whisper.tokenizer
                self.last_ids = []

                def detok(ids):   # forward's detokenize hook: the transcript's token ids (special tokens dropped, as
                    self.last_ids = list(ids)   # skip_special_tokens)
                    return tok.decode(ids)
                self.cb.detokenize = detok
                self.decoded = []
                dw0 = self.whisper.decode_window

                def dw(enc_out, prefix, *a, **k):   # the decoded tokens after the forced prefix: the digest and count
                    out = dw0(enc_out, prefix, *a, **k)   # source (the returned transcript is sliced by the untruncated
                    seq = out[0] if isinstance(out, tuple) else out   # keyword prompt's length, pba_whisper.py:338,
                    self.decoded.append([int(t) for t in seq[len(prefix):]])   # so a long prompt leaves it empty)
                    return out
                self.whisper.decode_window = dw

        def transcribe(self, idxs):
            """one generate call over the audios idxs (several: padded features + attention_mask, the reference's
            batched long-form); each audio's transcript = its segments' tokens.  --mode e2e: each 30 s clip through
            CBWhisper.forward (short-form: no timestamps, 5 beams, the keyword prompt; cb_whisper.py:151-187), its
            transcript = the decoded text"""
            with torch.cuda.device(dev), torch.cuda.stream(self.stream):
                feats = [log_mel_long(audios[i], n_mel) for i in idxs]
                if e2e:
                    for f, i in zip(feats, idxs):
                        self.decoded.clear()
                        self.cb.forward(f[None], torch.ones((1, f.shape[-1]), dtype=torch.long, device=dev))
                        gen = [t for d in self.decoded for t in d]
                        self.stats["tokens"] += len(gen)
                        self.stats["transcript_tokens"] += len(self.last_ids)
                        self.digests[i] = hashlib.sha1(np.asarray(gen, dtype=np.int64).tobytes()).hexdigest()[:16]
                    self.stream.synchronize()
                    return None
                if len(feats) == 1:
                    res = self.whisper.generate(input_features=feats[0][None], **self.gen_kw)
                else:
                    T = max(f.shape[-1] for f in feats)
                    x = torch.zeros((len(feats), n_mel, T), dtype=torch.float32, device=dev)
                    mask = torch.zeros((len(feats), T), dtype=torch.long, device=dev)
                    for b, f in enumerate(feats):
                        x[b, :, :f.shape[-1]] = f
                        mask[b, :f.shape[-1]] = 1
                    res = self.whisper.generate(input_features=x, attention_mask=mask, **self.gen_kw)
                for b, i in enumerate(idxs):
                    toks = [int(t) for s_ in res["segments"][b] for t in s_["tokens"].tolist()]
                    self.stats["tokens"] += len(toks)
                    self.digests[i] = hashlib.sha1(np.asarray(toks, dtype=np.int64).tobytes()).hexdigest()[:16]
                self.stream.synchronize()
            return res

        def run(self, calls):
            try:
                for idxs in calls:
                    self.transcribe(idxs)
            except BaseException as e:   # re-raised by the main thread
                self.error = e

    op_shift = [None]   # the realistic point's class-1 bias shift (computed once, every lane the same network)
    fp8_cal = [None]
    wsd = {"model.encoder." + k: v for k, v in synth.synth_whisper_encoder_state_dict(args.model, seed=0).items()}
    wsd.update({"model.decoder." + k: v for k, v in synth.synth_whisper_decoder_state_dict(args.model, seed=0).items()})
    lanes = [Lane(j) for j in range(A)]
    del wsd
    n = int(args.audio_seconds * 16000)
    audios = []   # audio u = (i * A + j) * G + g (step i, lane j, g-th of its generate call): seed 100000 * rank +
    # 1000 * u; a generate call's audios differ in length by 17 s steps; warm-up audios cut to <= 60 s
    for i in range(args.warmup + args.steps):
        for j in range(A):
            for g in range(G):
                u = (i * A + j) * G + g
                ni = max(16000, n - int(g * args.batch_length_step * 16000))
                ni = ni if i >= args.warmup else min(ni, 60 * 16000)
                a = np.concatenate([synth.synth_clip(100000 * rank + 1000 * u + q) for q in range(ni // 480000 + 1)])[:ni]
                audios.append(torch.from_numpy(a).to(dev))

    def run_lanes(first, count):
        """lane j transcribes audios (i * A + j) for i in [first, first + count), all lanes concurrently"""
        def calls(j):
            return [[(i * A + j) * G + g for g in range(G)] for i in range(first, first + count)]
        if A == 1:
            lanes[0].run(calls(0))
        else:
            th = [threading.Thread(target=ln.run, args=(calls(j),)) for j, ln in enumerate(lanes)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        for ln in lanes:
            if ln.error is not None:
                raise ln.error

    log(f"[bench] longform setup {time.time() - t_setup:.1f} s: {args.model} + LEF/resnet-50 vs {K} keywords, "
        f"{args.audio_seconds:.0f} s audio per lane per step, {A} lane(s), {args.beams} beams")
    run_lanes(0, args.warmup)
    torch.cuda.synchronize()
    for ln in lanes:
        for k in ln.stats:
            ln.stats[k] = 0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_lanes(args.warmup, args.steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = {k: sum(ln.stats[k] for ln in lanes) for k in lanes[0].stats}
    timed = range(args.warmup * A * G, (args.warmup + args.steps) * A * G)
    digests = {i: d for ln in lanes for i, d in ln.digests.items() if i in timed}
    elapsed, rank_elapsed = rank_times(dist, elapsed, dev)
    if dist is not None:
        tot = torch.tensor([stats["windows"], stats["tokens"]], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        stats["windows"], stats["tokens"] = int(tot[0]), int(tot[1])
    audio_s = sum(len(audios[u]) for u in timed) / 16000 * world
    if rank == 0 and e2e:
        clips = len(timed) * world
        rec = {"metric": f"utterances/sec end to end (30 s clips: {args.model} encoder hs -> CB-Whisper LEF spotting vs "
                         f"{K} keywords -> keyword prompt -> PBAWhisper {args.beams}-beam decode)",
               "value": round(clips / elapsed, 4), "unit": "utterances/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 1), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "e4m3+bf16" if args.fp8_first else "bf16",
               "data": "synthetic (seeded clips, seeded random weights, synthetic keyword hs and tokenizer)",
               "config": {"workload": f"CBWhisper.forward (cb_whisper.py:151-187): short-form generate, {args.beams} "
                                      f"beams, keyword prompt from LEF spotting vs {K} keywords (exact band "
                                      f"{args.exact_band})",
                          "parallelism": f"clip-parallel x{world}, {A} clip(s) in flight per GPU",
                          "operating_point": {"name": args.operating_point,
                                              **({"class1_bias_shift": round(-op_shift[0], 4)} if op_shift[0] else {})},
                          "spotting_first_tier": "fp8 (e4m3 MFMA)" if args.fp8_first else "bf16",
                          "max_new_tokens": args.max_new_tokens},
               "rank_elapsed_s": [round(x, 4) for x in rank_elapsed],
               "ms_per_clip": round(elapsed * world * A / max(1, clips) * 1e3, 1),
               "tokens_generated": stats["tokens"],
               "transcript_tokens": stats["transcript_tokens"],
               "note": "tokens_generated / transcript_digests: the decoded tokens after the forced prefix; the returned "
                       "transcript drops the first len(keyword prompt) tokens (pba_whisper.py:338 slices by the "
                       "untruncated prompt, which the decoder sees cut to its last 225 tokens)",
               "spotted_keywords_per_clip": round(stats["spotted"] / max(1, stats["windows"]), 1),
               "spotting_ms_per_clip": round(stats["spot_s"] / max(1, stats["windows"]) * 1e3, 1),
               "transcript_digests": {str(i): digests[i] for i in sorted(digests)}}
        print(json.dumps(rec), flush=True)
    elif rank == 0:
        rec = {"metric": f"audio seconds/sec (long-form PBAWhisper-{args.model} + CB-Whisper LEF spotting vs {K} "
                         f"keywords, clip-parallel)",
               "value": round(audio_s / elapsed, 3), "unit": "audio s/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 1), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "e4m3+bf16" if args.fp8_first else "bf16",
               "data": "synthetic (seeded audio, seeded random weights, synthetic keyword hs and tokenizer)",
               "config": {"workload": f"PBAWhisper.generate long-form ({args.audio_seconds:.0f} s per audio, "
                                      f"{args.beams} beams, timestamps, condition_on_prev_tokens) + CB-Whisper LEF "
                                      f"spotting per 30 s window vs {K} keywords (exact band {args.exact_band})",
                          "parallelism": f"clip-parallel x{world} (independent audios), {A} audio(s) in flight per GPU",
                          "audios_in_flight": A, "lane_priority": bool(args.lane_priority and A > 1),
                          "generate_batch": G,
                          "operating_point": {"name": args.operating_point,
                                              **({"class1_bias_shift": round(-op_shift[0], 4)} if op_shift[0] else {})},
                          "spotting_first_tier": "fp8 (e4m3 MFMA)" if args.fp8_first else "bf16",
                          "fp8_first": fp8_cal[0],
                          "max_new_tokens": args.max_new_tokens},
               "rank_elapsed_s": [round(x, 4) for x in rank_elapsed],
               "windows_per_s": round(stats["windows"] / elapsed, 3), "windows": stats["windows"],
               "tokens_generated": stats["tokens"],
               "ms_per_window": round(elapsed * world * A / max(1, stats["windows"]) * 1e3, 1),
               "spotted_keywords_per_window": round(stats["spotted"] / max(1, stats["windows"]), 1),
               "spotting_ms_per_window": round(stats["spot_s"] / max(1, stats["windows"]) * 1e3, 1),
               "transcript_digests": {str(i): digests[i] for i in sorted(digests)}}
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_api(args):
    """--mode api: the drop-in API path (efficient_kws.model.KWSModel.test_step, the call run_efficient_kws.py test
    makes per utterance; reference model.py:748-802) on the bench's workload.  One step = one synthetic 30 s clip:
    mel -> large-v3 encoder -> hs[19..21] (the utterance features the dataset would hand over) -> test_step with
    the bench's 10 000 seeded keywords as the dataset groups them (raw hs [50, 3, 150, D] fp32 + masks per group of
    hotwords_per_group = 50, eval-LEF-comp-acl.yaml:121; device-resident, the same tensor objects every step as a
    cached dataset hands them).  KWSModel keeps the groups' projections across calls and scores all groups in one
    chunked call; exact_band "auto" (calibrated at the first call, a warm-up step).  No pipelining: test_step is
    synchronous.  The spotted digest of the last timed clip equals the engine path's (both exact)."""
    from cbw import synth
    from cbw.whisper import EncoderEngine, default_layer_ids, log_mel
    from efficient_kws.model import KWSModel
    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--mode api is the one-GPU drop-in path (--gpus 1)")
    dev = _rank_device(int(os.environ.get("LOCAL_RANK", "0")))
    t_setup = time.time()
    enc_cfg = synth.WHISPER_CONFIGS[args.model]
    n_mel, D, n_layers, _, _ = enc_cfg
    enc = EncoderEngine(enc_cfg, synth.synth_whisper_encoder_state_dict(args.model, seed=0), dev)
    ids = default_layer_ids(n_layers)
    kws_hp = kws_hparams(args.variant, D, args.threshold, features_size=[150, 1500])
    model = KWSModel(**kws_hp)
    model.load_state_dict(synth.synth_kws_state_dict(seed=0, **kws_hp))
    model.engine()
    K = args.keywords
    groups, gmasks = [], []
    for _, x, m in keyword_hs(K, D, dev):
        for a in range(0, x.shape[0], 50):
            groups.append(x[a:a + 50].contiguous())
            gmasks.append(m[a:a + 50].contiguous())
    ghost = [torch.ones(g.shape[0], device=dev) for g in groups]
    clips = [torch.from_numpy(synth.synth_clip(i)).to(dev) for i in range(args.warmup + args.steps)]
    utt_mask = torch.ones((3, 1500), device=dev)
    log(f"[bench] api setup {time.time() - t_setup:.1f} s: {len(groups)} groups of 50 raw keyword hs")
    last = [None]

    def step(i):
        _, mel_pk = log_mel(clips[i], n_mel, packed=True)
        hs = enc.hidden_states(mel_pk, ids, normalize=True)
        out = model.test_step({"kwd": groups, "kwd_mask": gmasks, "utt": hs[0], "utt_mask": utt_mask,
                               "hotword_mask": ghost}, i)
        last[0] = out["preds"]

    t_w = time.perf_counter()
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - t_w
    model.test_step_outputs = []
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
        model.test_step_outputs = []
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    spotted = torch.nonzero(last[0] >= args.threshold).flatten().to(torch.int32)
    digest = hashlib.sha1(spotted.cpu().numpy().tobytes()).hexdigest()[:16]
    rec = {"metric": "utterances/sec (30 s clips) via efficient_kws.model.KWSModel.test_step (drop-in API), "
                     "Whisper-large-v3 LEF 10k kw",
           "value": round(args.steps / elapsed, 4), "unit": "utterances/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (seeded 30 s clips, seeded random weights, 10k synthetic keyword hs in groups of 50)",
           "config": {"workload": f"whisper-{args.model} encoder + KWSModel.test_step (LEF, resnet-50) vs {K} "
                                  f"keywords in {len(groups)} groups of 50, one 30 s clip per step",
                      "keywords": K, "kwd_cache": model.kwd_cache},
           "pairs_per_s": round(args.steps / elapsed * K, 1), "warmup_s": round(warm_s, 2),
           "band_calibration": model.band_calibration, "exact_band": model.exact_band,
           "spotted_last_clip": int(spotted.numel()), "spotted_digest": digest}
    print(json.dumps(rec), flush=True)


def main():
    # a fatal signal (e.g. the r03 SIGSEGV under rocprofv3 --pmc) writes every Python thread's stack to stderr;
    # a thread with no Python frames there is a native one (the runtime's or the profiler's)
    import faulthandler
    faulthandler.enable(all_threads=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--keywords", type=int, default=10000)
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--variant", choices=sorted(VARIANTS), default="LEF",
                    help="efficient_kws spotter: LEF (C3-C5, default), LE (C2: Whisper-small + LE, 1k keywords), L (C1: "
                         "tiny.en + L, 32 keywords)")
    ap.add_argument("--chunk", type=int, default=1112,
                    help="keyword pairs per ResNet chunk (1112 = 9 chunks of the 10k database, 3 per scoring stream; "
                         "profiles/r06c_chunk_sweep.txt: 6.14-6.16 utt/s vs 6.10-6.13 at 834 and 6.00-6.02 at 556 "
                         "on three streams, 6.04-6.05 at the former 625 on two)")
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--exact-band", type=float, default=None,
                    help="re-score every pair whose bf16 probability lies within this distance of the threshold "
                         "(inside the timed step), so the spotted indices are those of the reference's fp32 "
                         "evaluation; 0 = bf16 decisions only.  Default 0.015 with --bias-calibrate (largest "
                         "calibrated bf16-vs-fp32 probability error measured at this operating point 0.0109 over "
                         "16384 held-out pairs), else 0.03 (folded biases: 0.0254; tools/band_stats.py)")
    ap.add_argument("--x3-band", type=float, default=1e-4,
                    help="two-tier re-scoring: the pairs within --exact-band go through the compensated-bf16 tier "
                         "(cbw_kws_rescore_x3, max |p - p_fp32| 2.5e-5 measured) and only those then within this "
                         "distance of the threshold through fp32; <= 0: every band pair in fp32")
    ap.add_argument("--band-scale", type=float, default=None,
                    help="select the re-scored pairs by |p - threshold| <= band_scale x max(|l0|, |l1|) (cbw_kws_band_scaled: "
                         "the bf16 error of a pair's decision variable scales with its logit magnitude) instead of the "
                         "uniform --exact-band (0 = uniform, the default: after the calibrated logit offset the error "
                         "no longer grows with the logits; 3.0e-3 = 1.34 x the largest error / max|l| ratio, 2.2e-3, "
                         "over 16384 held-out pairs, selects 10 %% more pairs than the uniform 0.015)")
    ap.add_argument("--bias-calibrate", type=int, default=512,
                    help="setup: bias-correct the bf16 scoring network (KwsEngine.calibrate_bias) from the fp32 "
                         "network's conv-input means over the database's first N keywords vs a calibration clip that "
                         "is not timed (0.24 s at 512); 0 = the folded biases")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prof-dump", default=None,
                    help="write every timed conv launch (start/end ms from the hipEvents, algorithmic FLOPs) and the "
                         "timed region's CLOCK_MONOTONIC bounds to this JSON file, so the roofline's union-of-intervals "
                         "figure can be recomputed from it or from a rocprofv3 trace (tools/roofline_from_trace.py)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-launch HIP-event roofline timing")
    ap.add_argument("--fp8-first", action="store_true",
                    help="the fp8 first tier (C5): every pair scored by the e4m3 ResNet (stages 2-4 on "
                         "v_mfma_scale_f32_16x16x128_f8f6f4), only the pairs within the calibrated fp8 band re-scored "
                         "in bf16, then the exact tiers; the band is 1.5 x the largest fp8 error over held-out "
                         "calibration pairs (or --fp8-band)")
    ap.add_argument("--fp8-band", type=float, default=None, help="fp8 tier band (default: calibrated)")
    ap.add_argument("--no-companions", dest="companions", action="store_false",
                    help="skip the fp8-first companion runs (child processes after the headline measurement: the "
                         "realistic operating point with and without --fp8-first, and --fp8-first at this point)")
    ap.add_argument("--operating-point", choices=["synthetic", "realistic", "sparse"], default="synthetic",
                    help="synthetic: the seeded classifier as is (probabilities straddle 0.5, ~1/3 of the keywords "
                         "spotted); realistic: its class-1 bias lowered so ~1%% of the calibration pairs are positive "
                         "(a trained spotter on a real keyword list); sparse: ~0.15%% positive (~15 of 10 000 "
                         "keywords per clip: a keyword prompt short enough that the decoded transcript survives the "
                         "reference's outputs[:, len(prompt_ids):] slice, pba_whisper.py:338)")
    ap.add_argument("--no-audit", dest="audit", action="store_false",
                    help="skip the post-run audit (every pair of the last timed clip re-scored in fp32 and compared "
                         "with the timed step's decisions: audit_flips, audit_max_bf16_err, audit_band_margin)")
    ap.add_argument("--audit-pass", type=int, default=512,
                    help="audit: re-score the pairs in host-synchronised passes of this many pairs (0: one call, "
                         "~19k conv_f32 dispatches enqueued at once, which crashes the process under rocprofv3 --pmc: "
                         "DESIGN.md §5, profiles/r05b_pmc_f32_*)")
    ap.add_argument("--x3-overlap", dest="x3_overlap", action="store_true", default=True,
                    help="run clip i's re-scoring tiers on their own stream beside clip i+1's bf16 scoring (default)")
    ap.add_argument("--no-x3-overlap", dest="x3_overlap", action="store_false")
    ap.add_argument("--scoring-priority", choices=("normal", "high"), default="normal",
                    help="high: the bf16 scoring pass (main stream and libcbw's side streams, CBW_KWS_PRIO=-1) on "
                         "high-priority streams, the re-scoring tier and the front end on normal ones")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="run each clip's front end (mel, encoder, utterance projection) on the main stream before its "
                         "scoring; by default clip i+1's front end runs on a second stream while clip i is scored "
                         "(+1.8 %% utt/s: the encoder's few-tile GEMMs leave CUs the scoring convs use)")
    ap.add_argument("--mode", choices=["clip", "kwshard", "longform", "api", "e2e"], default="clip",
                    help="clip: every rank scores its own clips vs all keywords (weak scaling); kwshard: one clip "
                         "per step, keywords sharded over ranks, RCCL broadcast + all-gather (strong scaling, C4); "
                         "longform: every rank transcribes its own long audio with PBAWhisper.generate's seek loop, "
                         "CB-Whisper keyword spotting per 30 s window (C5, clip-parallel across audios); api: the drop-in "
                         "efficient_kws KWSModel.test_step path on the clip workload (one GPU); e2e: one 30 s clip per "
                         "step through CBWhisper.forward (spotting -> keyword prompt -> 5-beam decode, cb_whisper.py:151-187)")
    ap.add_argument("--batch-length-step", type=float, default=17.0,
                    help="longform --generate-batch: the audios of one generate call are this many seconds apart in "
                         "length (0: all --audio-seconds long, the lanes' audios)")
    ap.add_argument("--shard-sim", default=None, metavar="R/N",
                    help="kwshard at world 1: run rank R's workload of an N-rank keyword-sharded run (its front ends "
                         "are the clips i with i mod N == R; the other clips' projected utterances, which the other "
                         "ranks would broadcast, are computed before the timed region); pass the shard size as "
                         "--keywords (e.g. 12500 for C4's 100k over 8)")
    ap.add_argument("--audio-seconds", type=float, default=120.0,
                    help="longform: seconds of synthetic audio per rank per step (C5 names 30 min = 1800)")
    ap.add_argument("--beams", type=int, default=5, help="longform: beam width (cb_whisper.py:174)")
    ap.add_argument("--lane-priority", dest="lane_priority", action="store_true", default=True,
                    help="longform with lanes: decode on high-priority streams, spotting on normal-priority ones")
    ap.add_argument("--no-lane-priority", dest="lane_priority", action="store_false")
    ap.add_argument("--audios-in-flight", type=int, default=1,
                    help="longform: independent audios transcribed concurrently per GPU (one engine set, HIP stream "
                         "and host thread each)")
    ap.add_argument("--generate-batch", type=int, default=1,
                    help="longform: audios per PBAWhisper.generate call (the reference's batched long-form with an "
                         "attention mask: their windows spotted in one call and decoded together on one decoder "
                         "state); the g-th audio of a call is 17 g s shorter")
    ap.add_argument("--max-new-tokens", type=int, default=None,
                    help="longform: cap on the tokens generated per window (default: the reference's max_length)")
    ap.add_argument("--plumbing", action="store_true",
                    help="test only, no GPU: the multi-rank launch / barrier / max-over-ranks envelope with a CPU sleep "
                         "as the step (gloo); measures nothing of the hot path")
    ap.add_argument("--plumbing-ms", type=float, default=20.0, help="--plumbing: rank r's step sleeps (r + 1) x this")
    args = ap.parse_args()
    rc = launch_ranks(args.gpus, sys.argv[1:])
    if rc is not None:
        raise SystemExit(rc)
    if args.plumbing:
        return run_plumbing(args)
    if args.exact_band is not None and args.exact_band <= 0:
        args.bias_calibrate = 0   # bf16 decisions only: no fp32 keyword projections to calibrate from
    if args.band_scale is None:
        args.band_scale = 0.0
    if args.exact_band is None:
        args.exact_band = 0.015 if args.bias_calibrate > 0 else 0.03
    if args.mode in ("longform", "e2e"):
        if args.audios_in_flight > 1:   # one HIP hardware queue per lane stream (+ its spotting and side streams), so
            # the lanes' launches are not serialised behind each other in a shared queue (HIP's default: 4)
            os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, 4 + 3 * args.audios_in_flight))
        if args.audios_in_flight > 1 or args.generate_batch > 1:
            # several spotters / windows share the GPU: two scoring streams per spotter instead of the single-clip
            # default of three (r06, profiles/r06k_c5_streams_ab.txt: C5 lanes4 67.6 vs 62.9 audio s/s, batched
            # generate 45.9 vs 45.2, e2e with 4 clips in flight 2.70 vs 2.59 utt/s)
            os.environ.setdefault("CBW_KWS_STREAMS", "2")
        return run_longform(args)
    if args.mode == "api":
        return run_api(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = _rank_device(local_rank)
    if args.scoring_priority == "high":
        os.environ["CBW_KWS_PRIO"] = "-1"   # read when the engine creates its scoring side streams
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    dist = None
    if world > 1 or args.mode == "kwshard":
        # kwshard at world 1: the sharded code path (broadcast / all-gather over a one-rank group) on one GPU --
        # one rank's workload of a keyword-sharded run (e.g. --keywords 12500 = rank 0 of C4's 100k over 8 GPUs)
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29541")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        _init_dist(dist, dev)

    from cbw import synth, _lib
    from cbw.kws import KwsEngine
    from cbw.whisper import EncoderEngine, default_layer_ids, log_mel

    t_setup = time.time()
    enc_cfg = synth.WHISPER_CONFIGS[args.model]
    n_mel, D, n_layers, _, _ = enc_cfg
    enc_sd = synth.synth_whisper_encoder_state_dict(args.model, seed=0)
    enc = EncoderEngine(enc_cfg, enc_sd, dev)
    ids = default_layer_ids(n_layers)
    kws_hp = kws_hparams(args.variant, D, args.threshold)
    kws_sd = synth.synth_kws_state_dict(seed=0, **kws_hp)
    kws = KwsEngine(kws_hp, kws_sd, dev)
    K = args.keywords
    op_point = {"name": args.operating_point}
    if args.operating_point != "synthetic":   # lower the class-1 bias so ~1 % (sparse: 0.15 %) of the calibration
        delta = realistic_bias_shift(kws, enc, ids, n_mel, K, D, dev, OP_POSITIVE_FRAC[args.operating_point])   # pairs
        # are positive
        kws_sd = dict(kws_sd)
        b = np.array(kws_sd["model.classifier.1.bias"], dtype=np.float32).copy()
        b[1] -= delta
        kws_sd["model.classifier.1.bias"] = b
        del kws
        kws = KwsEngine(kws_hp, kws_sd, dev)
        op_point["class1_bias_shift"] = round(-delta, 4)
    sharded = args.mode == "kwshard"
    exact = float(args.exact_band) > 0
    band_scaled = exact and args.band_scale > 0
    band = float(args.band_scale) if band_scaled else float(args.exact_band)   # the first band's half-width / coefficient
    rescored = [0, 0]
    x3_band = args.x3_band if args.x3_band and args.x3_band > 0 else None

    def score_db(u, um, u32, kd, km, kd32, out=None):
        """bf16 scores of every pair + the fp32 re-score of the near-threshold band (cbw_kws_band/rescore)."""
        if not exact:
            n_bf16[0] += kd.shape[0]
            return kws.score(u, um, kd, km, chunk=args.chunk, logits_out=out)
        lg, st = kws.score_exact(u, um, kd, km, u32, kd32, args.threshold, band, chunk=args.chunk, logits_out=out,
                                 band_x3=x3_band, band_scaled=band_scaled, fp8_band=fp8_band)
        rescored[0] += st["band"]
        rescored[1] += st["fp32"]
        n_bf16[0] += st["bf16"]
        return lg

    # per-clip timing of the timed steps (hipEvents on the streams the work runs on, not subtraction): the first
    # scoring pass on the main stream, the re-scoring tiers (+ gather + spot) on the tier stream
    tspan = {"on": False, "score": [], "tiers": []}

    def first_pass(u, um, out):
        """every pair's first scores into ``out``: bf16, or (--fp8-first) fp8 and then bf16 for the pairs within
        the fp8 band (the host waits for the fp8 scores to select them)"""
        if tspan["on"]:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = _first_pass(u, um, out)
            b.record()
            tspan["score"].append((a, b))
            return r
        return _first_pass(u, um, out)

    def _first_pass(u, um, out):
        if fp8_band is None:
            n_bf16[0] += db.shape[0]
            return kws.score(u, um, db, dbm, chunk=args.chunk, logits_out=out)
        kws.score_fp8(u, um, db, dbm, chunk=args.chunk, logits_out=out)
        sel8, n8 = kws.band(out, args.threshold, fp8_band)
        n_bf16[0] += n8
        if n8:
            s_l = sel8.long()
            sub = kws.score(u, um, db.index_select(0, s_l), dbm.index_select(0, s_l), chunk=args.chunk)
            out.index_copy_(0, s_l, sub)
        return out

    sim = None
    if args.shard_sim:
        if not sharded or world != 1:
            raise SystemExit("--shard-sim simulates one rank of a keyword-sharded run on one process (--mode kwshard)")
        sr, sn = (int(v) for v in args.shard_sim.split("/"))
        if not 0 <= sr < sn:
            raise SystemExit("--shard-sim R/N needs 0 <= R < N")
        sim = (sr, sn)

    def owner(i):
        """the rank that runs clip i's front end and broadcasts it (cbw.parallel.front_owner: round robin)"""
        from cbw.parallel import front_owner
        return front_owner(i, sim[1] if sim else world)

    my_rank = sim[0] if sim else rank   # the rank whose workload this process runs
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
    # clip-parallel: every rank its own clips; keyword-sharded: clip i is the same audio on every rank (its front-end
    # rank, i mod N, broadcasts it), so N-rank decisions equal N = 1's clip by clip
    clips = [torch.from_numpy(synth.synth_clip((0 if sharded else 1000 * rank) + i)).to(dev) for i in range(n_clips)]
    utt_mask = torch.ones((1, 3, 1500), device=dev)
    hs = torch.empty((1, 3, 1500, D), dtype=torch.float32, device=dev)
    u_shape = (3, kws.out_frames(1500), kws.feat_dim)   # the projected utterance: [3, 750, 64] at LEF
    logits = torch.empty((K, 2), dtype=torch.float32, device=dev)
    prob = torch.empty((K,), dtype=torch.float32, device=dev)
    idx = torch.empty((K,), dtype=torch.int32, device=dev)
    nspot = torch.zeros((1,), dtype=torch.int32, device=dev)
    lib = _lib.load()
    if args.bias_calibrate > 0:
        if db32 is None:
            raise SystemExit("--bias-calibrate needs the fp32 keyword projections (--exact-band > 0)")
        calibrate_kws(kws, enc, ids, n_mel, K, D, args.bias_calibrate, dev)
    fp8_band, fp8_cal = None, None
    if args.fp8_first:
        if not exact:
            raise SystemExit("--fp8-first runs the exact tiers after it (--exact-band > 0)")
        b8, err8, n_ho = calibrate_fp8_tier(kws, enc, ids, n_mel, K, D, dev)
        fp8_band = float(args.fp8_band) if args.fp8_band else b8
        fp8_cal = {"fp8_max_err_held_out": round(err8, 5), "held_out_pairs": n_ho, "fp8_band": round(fp8_band, 5)}
        if fp8_band <= band:
            raise SystemExit(f"fp8 band {fp8_band} must exceed the bf16 band {band}")
    n_bf16 = [0]   # pairs scored in bf16 (all of them without the fp8 tier)
    torch.cuda.synchronize()
    log(f"[bench] setup {time.time() - t_setup:.1f} s: {args.model} encoder + {args.variant}/resnet-50, K={K}, db "
        f"{tuple(db.shape)}")

    def project_utt(h):
        pu, pum = kws.project(h, utt_mask)
        pu32 = kws.project_f32(h, utt_mask)[0][0] if exact else None
        return pu, pum, pu32

    last_utt = [None, None, None, None]   # (clip id, bf16 utterance, mask, fp32 utterance) of the latest scored clip
    sim_recv = {}
    if sim:   # the utterances the other ranks' front ends would broadcast to this rank, computed before timing
        for i in range(n_clips):
            if owner(i) != my_rank:
                _, mel_pk = log_mel(clips[i], n_mel, packed=True)
                h_ = enc.hidden_states(mel_pk, ids, normalize=True)
                pu_, pum_, pu32_ = project_utt(h_)
                sim_recv[i] = (pu_, pum_, pu32_)

    def step(i):
        if sharded:
            pu = pum = pu32 = None
            src = 0 if sim else owner(i)
            if my_rank == owner(i):
                _, mel_pk = log_mel(clips[i], n_mel, packed=True)
                enc.hidden_states(mel_pk, ids, normalize=True, out=hs)
                pu, pum, pu32 = project_utt(hs)
                pu, pum = pu[0], pum[0]
            elif sim:   # what another rank would have broadcast
                pu, pum, pu32 = sim_recv[i]
                pu, pum = pu[0], pum[0]
            u, um = spotter.broadcast_utterance(pu, pum, u_shape, u_shape[:2], torch.bfloat16, dev, src=src)
            if exact:   # the fp32 utterance projection travels with the bf16 one (576 KB at LEF)
                u32_shared[0] = spotter.broadcast_tensor(pu32, u_shape, torch.float32, dev, src=src)
            last_utt[:] = [i, u, um, u32_shared[0]]
            logits.copy_(spotter.score(u, um))
        else:
            _, mel_pk = log_mel(clips[i], n_mel, packed=True)
            enc.hidden_states(mel_pk, ids, normalize=True, out=hs)
            pu, pum, pu32 = project_utt(hs)
            last_utt[:] = [i, pu[0], pum[0], pu32]
            score_db(pu[0], pum[0], pu32, db, dbm, db32, out=logits)
        _lib.check(lib.cbw_kws_spot(logits.data_ptr(), None, K, float(args.threshold), 0, prob.data_ptr(),
                                    idx.data_ptr(), nspot.data_ptr(), _lib.stream_handle()), "cbw_kws_spot")

    # clip pipeline: clip i+1's front end (mel -> encoder -> utterance projection, few-tile GEMMs) runs on its
    # own stream while clip i's keyword scoring runs on the main stream; every clip still passes through the
    # whole path, the GPU's idle slots of one overlap the other.  Keyword-sharded: only rank 0 runs the front
    # end, and clip i+1's broadcast follows clip i's scoring on every rank.
    pipeline = args.pipeline
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

    # re-scoring overlap (--x3-overlap, clip-parallel mode with the exact tiers): clip i's compensated / fp32
    # tiers run on their own stream while clip i+1's bf16 scoring runs on the main stream.  Every clip still
    # passes through every tier before its spot; logits / spot buffers alternate between two clips.
    overlap = pipeline and exact and (args.x3_overlap or sharded)
    tier_stream = torch.cuda.Stream(device=dev) if overlap else None
    lg_buf = [logits, torch.empty_like(logits)]
    idx_buf = [idx, torch.empty_like(idx)]
    nspot_buf = [nspot, torch.zeros_like(nspot)]
    last_spot = [idx, nspot]   # the buffers holding the most recent clip's spotted indices

    # keyword-sharded: the local shard's logits alternate between two clips, the gathered full logits too
    K_loc = db.shape[0]
    loc_buf = [torch.empty((K_loc, 2), dtype=torch.float32, device=dev) for _ in range(2)] if sharded else lg_buf
    final_lg = [logits]   # the full logits of the most recent clip (what its spot read)

    def tiers_launch(j, pum, pu32):
        """band selection of clip j (host waits for its bf16 scores), then its compensated tier on tier_stream."""
        main = torch.cuda.current_stream()
        lg = loc_buf[j % 2]
        sel, n = kws.band(lg, args.threshold, band, scaled=band_scaled)
        rescored[0] += n
        um = pum[0].reshape(pum.shape[-2:]) if pum.dim() == 3 and pum.shape[0] == 1 else pum
        tier_stream.wait_stream(main)
        ev0 = None
        if tspan["on"]:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(tier_stream)
        for t in (sel, pu32, um):
            t.record_stream(tier_stream)
        if n:
            with torch.cuda.stream(tier_stream):
                kws.rescore(pu32, um, db32, dbm, lg, sel, trusted=True, tier="x3" if x3_band else "fp32")
        return (j, um, pu32, n, ev0)

    def tiers_finish(pending):
        """the fp32 tier of the pairs still within x3_band (host waits for the compensated tier), then (sharded:
        the all-gather of the shards' logits, on the tier stream) the spot."""
        j, um, pu32, n, ev0 = pending
        lg = loc_buf[j % 2]
        with torch.cuda.stream(tier_stream):
            if n and x3_band:
                sel2, n2 = kws.band(lg, args.threshold, x3_band)
                if n2:
                    kws.rescore(pu32, um, db32, dbm, lg, sel2, trusted=True)
                rescored[1] += n2
            if sharded:
                lg = spotter.gather(lg)
                lg_buf[j % 2].copy_(lg)
                lg = lg_buf[j % 2]
            _lib.check(lib.cbw_kws_spot(lg.data_ptr(), None, K, float(args.threshold), 0, prob.data_ptr(),
                                        idx_buf[j % 2].data_ptr(), nspot_buf[j % 2].data_ptr(), _lib.stream_handle()),
                       "cbw_kws_spot")
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(tier_stream)
            tspan["tiers"].append((ev0, ev1))
        last_spot[:] = [idx_buf[j % 2], nspot_buf[j % 2]]
        final_lg[0] = lg
        torch.cuda.current_stream().wait_stream(tier_stream)   # the next clip may reuse this clip's buffers

    def sh_front(i):
        """keyword-sharded: clip i's front-end rank (round robin) launches it on the front stream; the other ranks
        have none (under --shard-sim: the projection computed before the timed region)."""
        if my_rank == owner(i):
            return front(i)
        return (*sim_recv[i], None) if sim else None

    def sh_bcast(i, fr):
        """keyword-sharded: the front-end rank's projected clip i (bf16 + mask, and the fp32 projection the band
        re-scoring reads) to every rank; that rank's main stream first waits for the front end's event."""
        pu = pum = pu32 = None
        if fr is not None:
            pu, pum, pu32, ev = fr
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            pu, pum = pu[0], pum[0]
        src = 0 if sim else owner(i)
        u, um = spotter.broadcast_utterance(pu, pum, u_shape, u_shape[:2], torch.bfloat16, dev, src=src)
        u32 = spotter.broadcast_tensor(pu32, u_shape, torch.float32, dev, src=src) if exact else None
        last_utt[:] = [i, u, um, u32]
        return u, um, u32

    def run_sharded(first, n):
        """keyword-sharded pipeline: clip i+1's front end (rank 0, front stream) and clip i-1's re-scoring tiers
        + all-gather + spot (every rank, tier stream) run beside clip i's bf16 scoring of the local shard."""
        fr, pending = sh_front(first), None
        for i in range(first, first + n):
            u, um, u32 = sh_bcast(i, fr)
            if i + 1 < first + n:
                fr = sh_front(i + 1)
            first_pass(u, um, loc_buf[i % 2])
            if not exact:
                lg = spotter.gather(loc_buf[i % 2])
                _lib.check(lib.cbw_kws_spot(lg.data_ptr(), None, K, float(args.threshold), 0, prob.data_ptr(),
                                            idx.data_ptr(), nspot.data_ptr(), _lib.stream_handle()), "cbw_kws_spot")
                final_lg[0] = lg
                continue
            if pending is not None:
                tiers_finish(pending)
            pending = tiers_launch(i, um, u32)
        if pending is not None:
            tiers_finish(pending)

    def run_steps(first, n):
        if n <= 0:   # (--warmup 0)
            return
        if not pipeline:
            for i in range(first, first + n):
                step(i)
            return
        if sharded:
            return run_sharded(first, n)
        if overlap:
            nxt, pending = front(first), None
            for i in range(first, first + n):
                pu, pum, pu32, ev = nxt
                if i + 1 < first + n:
                    nxt = front(i + 1)
                torch.cuda.current_stream().wait_event(ev)
                last_utt[:] = [i, pu[0], pum[0], pu32]
                first_pass(pu[0], pum[0], lg_buf[i % 2])
                if pending is not None:
                    tiers_finish(pending)   # clip i-1's tiers ran beside clip i's bf16 scoring
                pending = tiers_launch(i, pum, pu32)
            tiers_finish(pending)
            return
        nxt = front(first)
        for i in range(first, first + n):
            pu, pum, pu32, ev = nxt
            if i + 1 < first + n:
                nxt = front(i + 1)
            torch.cuda.current_stream().wait_event(ev)
            last_utt[:] = [i, pu[0], pum[0], pu32]
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
    lg_loc = logits[:db.shape[0]]   # this rank's keywords (the shard when keyword-sharded)
    first_pass(pu[0], pum[0], lg_loc)
    ev[4].record()
    n_band = 0
    if exact:
        _, st = kws.score_exact(pu[0], pum[0], db, dbm, pu32, db32, args.threshold, band, chunk=args.chunk,
                                logits_out=lg_loc, band_x3=x3_band, band_scaled=band_scaled, fp8_band=fp8_band)
        n_band = st["band"]
    ev[5].record()
    torch.cuda.synchronize()
    breakdown = {"mel": ev[0].elapsed_time(ev[1]), "encoder": ev[1].elapsed_time(ev[2]),
                 "utt_projection": ev[2].elapsed_time(ev[3]), "kws_score": ev[3].elapsed_time(ev[4]),
                 "kws_score_with_tiers_in_place": ev[4].elapsed_time(ev[5]), "band_pairs": n_band}

    # conv launches per step: 53 per scoring chunk, and up to 53 per compensated-tier pass of 512 pairs
    n_conv_per_step = ((K_loc + args.chunk - 1) // args.chunk) * 53 + (53 * (K_loc // 512 + 2) if exact else 0)
    if fp8_band is not None:   # the fp8 pass's launches besides the bf16 ones of its band
        n_conv_per_step *= 2
    if not args.no_profile:
        _lib.check(lib.cbw_kws_profile(kws.h, n_conv_per_step * args.steps + 16), "cbw_kws_profile")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    rescored[0] = rescored[1] = 0
    n_bf16[0] = 0
    region_ns = [time.clock_gettime_ns(time.CLOCK_MONOTONIC)]   # rocprofv3 timestamps share this clock
    tspan["on"] = True
    t0 = time.perf_counter()
    run_steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    region_ns.append(time.clock_gettime_ns(time.CLOCK_MONOTONIC))
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tspan["on"] = False
    timed_ms = {k: (sum(a.elapsed_time(b) for a, b in tspan[k]) / len(tspan[k]) if tspan[k] else None)
                for k in ("score", "tiers")}
    conv_ms = ctypes.c_double()
    conv_flop = ctypes.c_double()
    conv_n = ctypes.c_int()
    tiers = {}
    per_kernel = []
    alg_flop_raw = None
    if not args.no_profile:
        nmax = n_conv_per_step * args.steps + 16
        st_, en_, fl_ = (np.zeros(nmax) for _ in range(3))
        tr_ = np.zeros(nmax, dtype=np.int32)
        n = lib.cbw_kws_profile_records(kws.h, st_.ctypes.data, en_.ctypes.data, fl_.ctypes.data, nmax)
        n = min(max(n, 0), nmax)
        lib.cbw_kws_profile_tiers(kws.h, tr_.ctypes.data, nmax)
        kn_ = (ctypes.c_char_p * nmax)()
        lib.cbw_kws_profile_kernels(kws.h, kn_, nmax)
        kern_names = [(kn_[i] or b"?").decode() for i in range(n)]
        per_kernel = per_kernel_table(kern_names, st_[:n], en_[:n], fl_[:n], tr_[:n], args.steps)
        alg_flop_raw = float(fl_[:n][tr_[:n] == (2 if fp8_band is not None else 0)].sum())
        for name, t in (("bf16_scoring", 0), ("compensated_rescoring", 1), ("fp8_first_tier", 2)):
            sel_t = tr_[:n] == t
            if sel_t.any():
                u = _union_ms(st_[:n][sel_t], en_[:n][sel_t])
                tiers[name] = {"launches": int(sel_t.sum()), "union_ms_per_step": round(u / args.steps, 3),
                               "tflop_per_step": round(fl_[:n][sel_t].sum() / args.steps / 1e12, 3),
                               "achieved": round(fl_[:n][sel_t].sum() / (u * 1e-3) / 1e12, 2)}
        if args.prof_dump and rank == 0:
            with open(args.prof_dump, "w") as f:
                json.dump({"steps": args.steps, "launches": int(n), "region_ns": region_ns,
                           "start_ms": st_[:n].round(4).tolist(), "end_ms": en_[:n].round(4).tolist(),
                           "flop": fl_[:n].tolist(), "tier": tr_[:n].tolist(), "kernel": kern_names}, f)
        _lib.check(lib.cbw_kws_profile_read(kws.h, ctypes.byref(conv_ms), ctypes.byref(conv_flop),
                                            ctypes.byref(conv_n)), "cbw_kws_profile_read")
        lib.cbw_kws_profile(kws.h, 0)
    elapsed_local = elapsed
    elapsed, rank_elapsed = rank_times(dist, elapsed, dev)
    utts = args.steps * (1 if sharded else world)
    value = utts / elapsed
    n_spotted = int(last_spot[1].item())
    # digest of the last clip's spotted index list (equal across scheduling modes: --x3-overlap / --no-x3-overlap)
    spot_digest = hashlib.sha1(last_spot[0][:n_spotted].cpu().numpy().tobytes()).hexdigest()[:16]

    def audit_last_clip():
        """After the timed region: every pair of the last timed clip (this rank's shard when keyword-sharded)
        re-scored on the fp32 tier -- the path test_exact_rescore_matches_reference_fp32 pins to the reference's
        own fp32 forward -- against the logits the timed step's tiers left, decision by decision
        (prob >= threshold, the reference's rule, model.py:782-813).  The bf16 pass is re-run (deterministic:
        bit-identical to the timed one) for the bf16 error and the band's margin over it."""
        t_a = time.perf_counter()
        j, u, um, u32 = last_utt
        torch.cuda.synchronize()
        Kl = db.shape[0]
        lo = spotter.lo if sharded else 0
        fin = final_lg[0][lo:lo + Kl].clone()
        bf = kws.score(u, um, db, dbm, chunk=args.chunk)
        full = torch.empty((Kl, 2), dtype=torch.float32, device=dev)
        sel_all = torch.arange(Kl, dtype=torch.int32, device=dev)
        step_ = args.audit_pass if args.audit_pass > 0 else Kl
        for a0 in range(0, Kl, step_):
            kws.rescore(u32, um, db32, dbm, full, sel_all[a0:a0 + step_], trusted=True)
            if args.audit_pass > 0:
                torch.cuda.synchronize()
        p_fin, i_fin = kws.spot(fin, None, args.threshold)
        p32, i32 = kws.spot(full, None, args.threshold)
        p_bf, _ = kws.spot(bf, None, args.threshold)
        flips = int(((p_fin >= args.threshold) != (p32 >= args.threshold)).sum().item())
        same_list = bool(torch.equal(i_fin, i32))
        if not sharded:   # the index list the timed step's spot produced
            same_list = same_list and bool(torch.equal(last_spot[0][:n_spotted].long(), i32))
        err = (p_bf.double() - p32.double()).abs()
        ratio = err / bf.abs().amax(1).double().clamp_min(1e-30)
        if fp8_band is not None:
            p8, _ = kws.spot(kws.score_fp8(u, um, db, dbm, chunk=args.chunk), None, args.threshold)
            e8 = torch.tensor([(p8.double() - p32.double()).abs().max().item()], dtype=torch.float64, device=dev)
            if dist is not None:
                dist.all_reduce(e8, op=dist.ReduceOp.MAX)
            fp8_audit = {"audit_max_fp8_err": round(float(e8.item()), 6),
                         "audit_fp8_band_margin": round(fp8_band / max(float(e8.item()), 1e-12), 3)}
        else:
            fp8_audit = {}
        vals = torch.tensor([flips, 0 if same_list else 1, err.max().item(), ratio.max().item(),
                             (p_fin.double() - p32.double()).abs().max().item(),
                             int(i32.numel())], dtype=torch.float64, device=dev)
        if dist is not None:
            s_ = vals[[0, 1, 5]].clone()
            m_ = vals[[2, 3, 4]].clone()
            dist.all_reduce(s_)
            dist.all_reduce(m_, op=dist.ReduceOp.MAX)
            vals[[0, 1, 5]], vals[[2, 3, 4]] = s_, m_
        v = vals.tolist()
        max_err, max_ratio = v[2], v[3]
        margin = (band / max_ratio if band_scaled else band / max_err) if max_err > 0 else None
        return {"audit_clip": j, "audit_pairs": K, "audit_flips": int(v[0]), "audit_index_lists_equal": v[1] == 0,
                "audit_spotted_fp32": int(v[5]), "audit_max_bf16_err": round(max_err, 6),
                "audit_max_bf16_err_over_max_logit": round(max_ratio, 7),
                "audit_band_margin": round(margin, 3) if margin else None,
                "audit_max_final_err": float(f"{v[4]:.3g}"), "audit_s": round(time.perf_counter() - t_a, 2),
                **fp8_audit}

    audit = audit_last_clip() if (exact and args.audit and last_utt[0] is not None) else None
    per_rank = None
    if sharded:   # per-rank breakdown: the serial part of a step = step time - the rank's own scoring time
        # the rank's own scoring and re-scoring times, measured over the timed steps on their streams
        mine = torch.tensor([timed_ms["score"] or breakdown["kws_score"], timed_ms["tiers"] or 0.0,
                             elapsed_local * 1e3 / args.steps,
                             db.shape[0]], dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [{"rank": r, "keywords": int(a[3]), "kws_score_ms": round(float(a[0]), 3),
                     "band_rescore_ms": round(float(a[1]), 3), "ms_per_step": round(float(a[2]), 3),
                     "serial_ms_per_step": round(float(a[2] - a[0]), 3),
                     "serial_frac_of_scoring": round(float((a[2] - a[0]) / a[0]), 4),
                     # the part that does not shrink with the shard: the step minus the rank's own bf16 scoring and
                     # its band re-scoring (both proportional to its keywords) = front-end share, collectives, waits
                     "nonparallel_ms_per_step": round(float(a[2] - a[0] - a[1]), 3),
                     "nonparallel_frac_of_scoring": round(float((a[2] - a[0] - a[1]) / a[0]), 4)}
                    for r, a in enumerate(allr)]

    if rank == 0:
        rec = {
            "metric": workload_metric(args.model, args.variant, K), "value": round(value, 4), "unit": "utterances/s",
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded 30 s clips, seeded random weights, 10k synthetic keyword hs)",
            "config": {"workload": f"whisper-{args.model} encoder + efficient_kws {args.variant} (resnet-50) vs {K} keywords, "
                                   f"one 30 s clip per step per GPU",
                       "keywords": K, "variant": args.variant, "clips_per_step": 1 if sharded else world,
                       "utterance_frames": 1500, "keyword_frames": 150, "map_shape": [3, db.shape[2], u_shape[1]],
                       "hs_layers": ids, "chunk": args.chunk, "parallelism": (
                           f"rank {sim[0]} of a keyword-sharded x{sim[1]} run, simulated on one GPU (its front ends: "
                           f"clips i with i mod {sim[1]} == {sim[0]}; the others' projections computed before timing)"
                           if sim else f"keyword-sharded x{world} (round-robin front end, RCCL broadcast + all-gather)"
                           if sharded else f"clip-parallel x{world}"),
                       "clip_pipeline": pipeline},
            "pairs_per_s": round(value * K, 1),
            "rank_elapsed_s": [round(x, 4) for x in rank_elapsed],
            "breakdown_ms": {k: round(v, 3) for k, v in breakdown.items()},
            "timed_ms_per_clip": {"first_scoring_pass": None if timed_ms["score"] is None else round(timed_ms["score"], 3),
                                  "rescoring_tiers_on_tier_stream": None if timed_ms["tiers"] is None
                                  else round(timed_ms["tiers"], 3),
                                  "note": "hipEvents around each timed clip's first scoring pass (main stream) and its "
                                          "re-scoring tiers + spot (tier stream, beside the next clip's scoring); the "
                                          "two overlap, so they do not add up to ms_per_step"},
            "spotted_last_clip": n_spotted, "spotted_digest": spot_digest,
            "x3_overlap": overlap,
            "scoring_priority": args.scoring_priority,
            "exact_band": args.exact_band if exact else 0.0, "band_scale": band if band_scaled else None,
            "x3_band": x3_band, "bias_calibration_pairs": args.bias_calibrate,
            "operating_point": op_point, "fp8_first": fp8_cal,
            "bf16_pairs_per_step": round(n_bf16[0] / args.steps, 1),
            "rescored_pairs_per_step": round(rescored[0] / args.steps, 1),
            "fp32_rescored_pairs_per_step": round(rescored[1] / args.steps, 1),
            "decisions": ("bf16 scores; pairs within exact_band of the threshold re-scored inside the timed step "
                          "(compensated-bf16 tier, then those within x3_band in fp32-input MFMA), so spotted indices "
                          "follow the reference's fp32 evaluation"
                          if exact else "bf16 scores only (decisions within ~0.03 of the threshold may differ "
                                        "from fp32)"),
        }
        if audit is not None:
            rec.update(audit)
        if per_rank is not None:
            rec["per_rank"] = per_rank
        if not args.no_profile and conv_n.value > 0:
            # algorithmic work: each pair once through the 52 convs = the bf16 scoring tier's FLOPs
            # (9.8075 GFLOP per pair); the compensated tier's FLOPs are exactness overhead ("tiers"), not work.
            # Divided by the union of the launch intervals of BOTH tiers (they overlap with --x3-overlap).
            alg_flop = alg_flop_raw if alg_flop_raw else conv_flop.value
            achieved = alg_flop / (conv_ms.value * 1e-3) / 1e12
            traffic, traffic_step = _pmc_traffic()
            rec["roofline"] = {"bound": "mfma", "achieved": round(achieved, 2), "peak": 2500.0, "unit": "TFLOP/s",
                               "frac": round(achieved / 2500.0, 4), "traffic": traffic, "traffic_bytes_per_step": traffic_step,
                               "kernel": "ResNet-50 conv family: conv_igemm* + conv_ring + conv_stream + bottleneck_kernel (bf16 MFMA 16x16x32); "
                                         "achieved = algorithmic FLOPs (9.8075 GFLOP per pair, each pair once) / union of the launch "
                                         "intervals of the bf16 scoring pass and the compensated re-scoring tier; the compensated tier's "
                                         "own FLOPs are overhead spent on exactness (tiers.compensated_rescoring, "
                                         "overhead_tflop_per_step), not counted",
                               "tiers": tiers,
                               "overhead_tflop_per_step": round((conv_flop.value - alg_flop) / args.steps / 1e12, 3),
                               "traffic_unit": "bytes per launch, timed steps only (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                               "profiles/pmc_conv_latest.json)",
                               "recompute": f"tools/roofline_from_trace.py profiles/{TRACE_TAG}_kernel_trace.csv.gz --dump "
                                            f"profiles/{TRACE_TAG}_conv_launches.json (algorithmic_over_both_tiers_frac, "
                                            f"per_kernel; profiles/{TRACE_TAG}_roofline.json); "
                                            "traffic: profiles/pmc_conv_latest.json 'recompute'",
                               # in-bench per-kernel table (hipEvents per launch, kernel names from the runtime):
                               # the dominant kernel is the bf16 pass's largest total time
                               "dominant_kernel": next((r for r in per_kernel if r["tier"] == "bf16_scoring"), None),
                               "per_kernel": per_kernel[:16],
                               "launches": conv_n.value, "kernel_ms_per_step": round(conv_ms.value / args.steps, 3),
                               "algorithmic_tflop_per_step": round(alg_flop / args.steps / 1e12, 3)}
            iso = _isolated_per_kernel(rec["roofline"]["dominant_kernel"])
            if iso:
                rec["roofline"].update(iso)
        log(f"[bench] timed: {rec['value']} {rec['unit']}, {rec['ms_per_step']} ms per step")
        if world == 1 and not args.no_cpu_baseline:
            log("[bench] cpu baseline (bounded sample on the host cores)")
            try:
                rec["cpu_baseline"] = cpu_baseline(enc_sd, kws_sd, kws_hp, synth.synth_clip(0), K, enc_cfg)
            except Exception as e:  # the GPU result stands on its own
                rec["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
        if world == 1 and args.companions and args.mode == "clip" and not args.fp8_first \
                and args.operating_point == "synthetic":
            rec["fp8_first_mode"] = companion_runs(args)
            rec["configs_companion"] = config_runs()
            rec["end_to_end_companion"] = end_to_end_runs()
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
