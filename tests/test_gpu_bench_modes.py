"""bench.py's scheduling modes compute the same decisions: the re-scoring tiers overlapped with the next
clip's bf16 scoring (--x3-overlap, default), run in place (--no-x3-overlap), and without the clip pipeline
(--no-pipeline) give the same spotted index list for the last clip (sha1 digest) and the same band counts;
and the calibrated bf16 network (bias correction + logit offset) with its 0.015 band (default) and with the
per-pair band spots the same keywords as the folded biases with the 0.03 band (all reproduce the fp32 decisions,
which bench.py's audit of the last timed clip confirms per run)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*flags, ranks=1):
    args = [os.path.join(REPO, "bench.py"), "--model", "small", "--keywords", "720", "--steps", "3",
            "--warmup", "1", "--no-cpu-baseline", "--no-profile", "--no-companions", *flags]
    env = dict(os.environ, PYTHONFAULTHANDLER="1")   # an abort in the subprocess prints every thread's Python stack
    if ranks > 1:   # the N-rank code path on the one GPU (gloo; RCCL refuses two ranks on one device)
        args = ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}", "--master-addr",
                "127.0.0.1", "--master-port", "29533", *args, "--gpus", str(ranks)]
        env.update(CBW_BENCH_DEVICE="0", CBW_BENCH_DIST="gloo", OMP_NUM_THREADS="4")
    out = subprocess.run([sys.executable, *args], cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    if out.returncode != 0:   # keep the whole log (a torchrun failure buries the rank's traceback mid-stream)
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", "bench_mode_failure.err"), "w") as f:
            # both streams: whether an abort came after the JSON line (teardown) or mid-run shows in stdout
            f.write(f"rc {out.returncode}\n--- stdout ---\n{out.stdout}\n--- stderr ---\n{out.stderr}")
        tb = [ln for ln in out.stderr.splitlines() if "Error" in ln or 'File "' in ln]
        raise AssertionError("\n".join(tb[-30:]) + "\n" + out.stderr[-1500:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_bench_scheduling_modes_agree():
    a = run_bench("--x3-overlap")
    b = run_bench("--no-x3-overlap")
    c = run_bench("--no-pipeline")
    d = run_bench("--bias-calibrate", "0")
    e = run_bench("--band-scale", "3e-3")
    assert a["bias_calibration_pairs"] > 0 and a["exact_band"] == 0.015 and d["bias_calibration_pairs"] == 0
    assert d["exact_band"] == 0.03 and d["band_scale"] is None and e["band_scale"] == 3e-3
    assert e["spotted_digest"] == a["spotted_digest"]
    assert d["spotted_digest"] == a["spotted_digest"]
    assert d["rescored_pairs_per_step"] > a["rescored_pairs_per_step"]
    assert a["x3_overlap"] and not b["x3_overlap"]
    assert a["rescored_pairs_per_step"] > 0
    for r in (b, c):
        assert r["spotted_last_clip"] == a["spotted_last_clip"]
        assert r["spotted_digest"] == a["spotted_digest"]
        assert r["rescored_pairs_per_step"] == a["rescored_pairs_per_step"]
    for r in (a, b, c, d, e):   # bench.py's own audit of its last timed clip: every decision equals fp32's
        assert r["audit_flips"] == 0 and r["audit_index_lists_equal"], r
        assert r["audit_clip"] == 3 and r["audit_pairs"] == 720 and r["audit_band_margin"] > 1.0


def test_api_mode_and_keyword_sharded_spot_like_the_engine_path():
    """--mode api (KWSModel.test_step with the cached keyword database, groups of 50) and --mode kwshard over two
    ranks (broadcast utterance, pipelined front end and tiers, all-gathered logits) spot the same keywords of the
    last clip as the clip-mode engine path, and the sharded run's audit finds no flip on any rank."""
    a = run_bench()
    api = run_bench("--mode", "api")
    assert api["spotted_digest"] == a["spotted_digest"], (api, a)
    assert api["band_calibration"]["held_out_pairs"] > 0 and api["exact_band"] <= 0.5
    ks = run_bench("--mode", "kwshard", ranks=2)
    assert ks["n_gpus"] == 2 and ks["scaling"] == "strong"
    assert ks["spotted_digest"] == a["spotted_digest"]
    assert ks["audit_flips"] == 0 and ks["audit_index_lists_equal"] and ks["audit_pairs"] == 720
    assert [r["keywords"] for r in ks["per_rank"]] == [360, 360]
    # one rank's workload of a keyword-sharded run on one process (rank 1 of 2: front ends of the odd clips only)
    sim = run_bench("--mode", "kwshard", "--shard-sim", "1/2", "--keywords", "360")
    assert sim["n_gpus"] == 1 and "rank 1 of a keyword-sharded x2" in sim["config"]["parallelism"]
    assert sim["audit_flips"] == 0 and sim["audit_index_lists_equal"] and sim["audit_pairs"] == 360
    assert sim["per_rank"][0]["keywords"] == 360


def test_longform_lanes_transcribe_like_one_lane():
    """--mode longform with two audios in flight per GPU (a PBAWhisper + spotter engine set, HIP stream and host
    thread each, sharing the card) transcribes every audio exactly as one lane does: the same token ids (digest) per
    audio index.  The decoder and spotter kernels are deterministic, so interleaving the lanes changes no result."""
    common = ["--mode", "longform", "--model", "micro", "--keywords", "64", "--audio-seconds", "40", "--beams", "2",
              "--warmup", "1"]
    one = run_bench(*common, "--steps", "3")
    two = run_bench(*common, "--steps", "1", "--audios-in-flight", "2")
    assert sorted(one["transcript_digests"]) == ["1", "2", "3"] and sorted(two["transcript_digests"]) == ["2", "3"]
    assert two["config"]["audios_in_flight"] == 2 and two["windows"] >= 4
    for i in ("2", "3"):
        assert two["transcript_digests"][i] == one["transcript_digests"][i]


def test_longform_generate_batch_runs_the_batched_path():
    """--generate-batch 3: each generate call transcribes three audios of different lengths (padded features +
    attention_mask: the reference's batched long-form, one spotting call and one decoder state for all the
    iteration's windows); the JSON records every audio's transcript digest."""
    common = ["--mode", "longform", "--model", "micro", "--keywords", "64", "--audio-seconds", "60", "--beams", "2",
              "--warmup", "1", "--steps", "1"]
    bat = run_bench(*common, "--generate-batch", "3")
    assert bat["config"]["generate_batch"] == 3 and sorted(bat["transcript_digests"]) == ["3", "4", "5"]
    assert bat["windows"] >= 3 and bat["value"] > 0


def test_longform_fp8_first_transcribes_like_bf16_first():
    """C5's fp8 first tier in the long-form loop: at the realistic operating point, the spotter's cascade
    fp8 -> bf16 -> compensated -> fp32 makes the decisions the bf16-first cascade makes (both equal the fp32 ones),
    so every window gets the same keyword prompt and every audio the same transcript (token-id digests)."""
    common = ["--mode", "longform", "--model", "micro", "--keywords", "600", "--audio-seconds", "40", "--beams", "2",
              "--warmup", "1", "--steps", "1", "--operating-point", "realistic"]
    b16 = run_bench(*common)
    f8 = run_bench(*common, "--fp8-first")
    assert f8["dtype"] == "e4m3+bf16" and f8["config"]["spotting_first_tier"].startswith("fp8")
    assert f8["config"]["fp8_first"]["fp8_band"] > 0 and b16["config"]["operating_point"]["name"] == "realistic"
    assert f8["transcript_digests"] == b16["transcript_digests"]
    assert f8["spotted_keywords_per_window"] == b16["spotted_keywords_per_window"]
