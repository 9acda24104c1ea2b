"""bench.py's scheduling modes compute the same decisions: the re-scoring tiers overlapped with the next
clip's bf16 scoring (--x3-overlap, default), run in place (--no-x3-overlap), and without the clip pipeline
(--no-pipeline) give the same spotted index list for the last clip (sha1 digest) and the same band counts;
and the calibrated bf16 network (bias correction + logit offset) with its 0.015 band (default) and with the
per-pair band spots the same keywords as the folded biases with the 0.03 band (all reproduce the fp32 decisions)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*flags):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--model", "small", "--keywords", "720", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--no-profile", *flags]
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
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
