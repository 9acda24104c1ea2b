"""Companion runs beside bench.py's headline line: this bench as child processes (each its own GPU setup) at the
fp8-first / realistic operating points, at BASELINE.json's other configs (C2, C1) and end to end / C5 long-form.
Their values are reported in the line, never the headline ``value``."""
from __future__ import annotations

import json
import os
import sys
import time

from benchlib.common import log

BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _child_bench(extra: list, timeout: int = 420, steps: int = 5, warmup: int = 1):
    """This bench as a child process (its own GPU setup, 5 timed steps) -> (its JSON line or None, error text)."""
    import subprocess
    import threading
    cmd = [sys.executable, BENCH, "--steps", str(steps), "--warmup", str(warmup),
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
