"""Offline error model of the bf16 decision variable from band_stats.py BS_DUMP files: does |d_bf16 - d_fp32|
(d = l1 - l0) scale with a quantity the bf16 pass already has (the logits), so that a pair-adaptive band
|d_bf16 - d_thr| <= c f(logits) holds fewer pairs than the uniform band at the same safety margin?
usage: python tools/band_model.py gpurun_out/pairs_clips_cal_0.npz [...]"""
import sys

import numpy as np

sel, bf, f32 = [], [], []
for f in sys.argv[1:]:
    z = np.load(f)
    bf.append(z["bf16"]); f32.append(z["fp32"])
bf = np.concatenate(bf).astype(np.float64)
f32 = np.concatenate(f32).astype(np.float64)
d_bf, d32 = bf[:, 1] - bf[:, 0], f32[:, 1] - f32[:, 0]
err = np.abs(d_bf - d32)
print(f"pairs {len(err)}: err max {err.max():.3e} rms {np.sqrt((err ** 2).mean()):.3e}; d range [{d32.min():.2f}, {d32.max():.2f}]")
proxies = {
    "const": np.ones_like(err),
    "|l0|+|l1|": np.abs(bf).sum(1),
    "max|l|": np.abs(bf).max(1),
    "|d|": np.abs(d_bf),
    "sqrt(l0^2+l1^2)": np.sqrt((bf ** 2).sum(1)),
}
near = np.abs(d_bf) <= 0.2   # the pairs a band around p = 0.5 (d = 0) could hold
for name, f in proxies.items():
    f = np.maximum(f, 1e-6)
    r = err / f
    c = 1.3 * r.max()
    inband = np.abs(d_bf) <= c * f
    corr = np.corrcoef(err, f)[0, 1] if name != "const" else float("nan")
    print(f"{name:16s} corr {corr:+.3f}  c {c:.3e}  pairs in band {inband.sum():5d} ({100 * inband.mean():.2f} %)")
