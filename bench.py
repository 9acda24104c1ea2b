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

# shared setup, the non-headline modes and the companion runs live in benchlib/ (re-exported here: tests and tools
# call bench.build_keyword_db, bench.calibrate_kws, ...)
from benchlib.common import (OP_POSITIVE_FRAC, VARIANTS, _calibration_pairs, _init_dist, _probs,  # noqa: E402,F401
                             _rank_device, build_keyword_db, calibrate_fp8_tier, calibrate_kws, keyword_hs,
                             kws_hparams, log, rank_times, realistic_bias_shift)
from benchlib.companions import companion_runs, config_runs, end_to_end_runs  # noqa: E402
from benchlib.modes import run_api, run_longform, run_plumbing  # noqa: E402

METRIC = "utterances/sec (30 s clips) + keywords/sec matched, Whisper-large-v3 LEF 10k kw"

# ResNet-50 GFLOP per pair (BASELINE.md / SURVEY §6, FlopCounterMode): LEF maps [3, 75, 750], L / LE [3, 150, 1500]
RESNET50_GFLOP = {"L": 38.25, "LE": 38.25, "LEF": 10.08}


def workload_metric(model: str, variant: str, K: int) -> str:
    """BASELINE.json's metric for the headline config; the same metric named for the other configs"""
    if (model, variant, K) == ("large-v3", "LEF", 10000):
        return METRIC
    return f"utterances/sec (30 s clips) + keywords/sec matched, Whisper-{model} {variant} {K} kw"


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
