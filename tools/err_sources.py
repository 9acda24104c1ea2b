"""Where does the bf16 scoring error come from?  (CPU, float64 truth)

The LEF/ResNet-50 scorer at the bench widths (D = 1280, 3 layers, [3, 75, 750] maps) with seeded weights
and random per-frame unit hs; the logit difference l1 - l0 (the decision variable) in float64 vs variants
that round to bf16 at one place of the GPU path at a time:
  proj   the projected keyword / utterance rows (the bf16 database and utterance projection)
  maps   the similarity maps (stored bf16 before the stem)
  w      the BN-folded conv weights (bias kept fp32)
  act    every conv output as stored (after bias / residual / ReLU)
  all    everything above
and the fp8 alternatives (C5 g1) on the same points, OCP e4m3 with MX block scaling (a power-of-two scale
per 32 consecutive input channels, the block-scaled MFMA's format; the 3-channel stem stays bf16):
  w8     the folded conv weights in MX-e4m3, activations bf16
  a8     the conv inputs in MX-e4m3 (weights bf16)
  fp8    weights and conv inputs in MX-e4m3, outputs stored bf16 (+ bf16 maps / projections)
Keyword lengths are ragged (U{8..150} frames, masked maps as bench.py's database), so the pairs differ.
Prints max and rms |delta(l1 - l0)| per variant; at p = 0.5 a decision-variable error d moves the
probability by about d / 4, which is the band half-width the exact tiers would need.
usage: python tools/err_sources.py [pairs]
"""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd")]
from cbw import synth  # noqa: E402
from oracle import torch_ref as tr  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
D = 1280
hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True, proj_mlp_units=64,
          resnet_version="resnet-50", threshold=0.5)
sd = {k: torch.from_numpy(v).double() for k, v in synth.synth_kws_state_dict(seed=0, **hp).items()}
spec = synth.resnet_spec(3, "resnet-50")
g = torch.Generator().manual_seed(0)
utt = torch.randn((1, 3, 1500, D), generator=g, dtype=torch.float64)
utt = utt / utt.norm(dim=-1, keepdim=True)
kwd = torch.randn((P, 3, 150, D), generator=g, dtype=torch.float64)
kwd = kwd / kwd.norm(dim=-1, keepdim=True)
lens = torch.randint(8, 151, (P,), generator=g)
kmask = (torch.arange(150)[None, :] < lens[:, None]).double()            # [P, 150]
kwd = kwd * kmask[:, None, :, None]
kmask_p = F.max_pool1d(kmask[:, None], 3, 2, 1)[:, 0]                    # frames_conv pooling: [P, 75]


def bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def mx8(t, dim=1):
    """MX-e4m3 (OCP MX v1.0): blocks of 32 along ``dim`` share the scale 2^(floor(log2 amax) - 8),
    elements saturate at +-448."""
    x = t.movedim(dim, -1)
    n = x.shape[-1]
    pad = (-n) % 32
    xp = F.pad(x, (0, pad)).reshape(*x.shape[:-1], -1, 32)
    amax = xp.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    sc = torch.exp2(torch.floor(torch.log2(amax)) - 8)
    q = (xp / sc).clamp(-448, 448).float().to(torch.float8_e4m3fn).to(t.dtype) * sc
    return q.reshape(*x.shape[:-1], -1)[..., :n].movedim(-1, dim)


def folded(c):
    p = f"{c.prefix}.normalization"
    s = sd[f"{p}.weight"] / torch.sqrt(sd[f"{p}.running_var"] + 1e-5)
    w = sd[f"{c.prefix}.convolution.weight"] * s[:, None, None, None]
    b = sd[f"{p}.bias"] - sd[f"{p}.running_mean"] * s
    return w, b


def forward(q):
    def project(x):
        return tr.project(x, sd, 3, True)
    with torch.no_grad():
        pu, pk = project(utt), project(kwd)
        if "proj" in q:
            pu, pk = bf(pu), bf(pk)
        sims = []
        for l in range(3):
            a = pu[:, l] / pu[:, l].norm(dim=-1, keepdim=True)
            b = pk[:, l] / pk[:, l].norm(dim=-1, keepdim=True)
            sims.append(torch.einsum("kfd,ud->kfu", b, a[0]))
        x = torch.stack(sims, 1) * kmask_p[:, None, :, None]
        if "maps" in q:
            x = bf(x)

        def conv(h, c):
            w, b = folded(c)
            if "w" in q:
                w = bf(w)
            if c is not spec.stem and "w8" in q:
                w = mx8(w)
            if c is not spec.stem and "a8" in q:
                h = mx8(h)
            return F.conv2d(h, w, b, stride=c.stride, padding=c.k // 2)

        def st(h):
            return bf(h) if "act" in q else h
        h = F.max_pool2d(st(F.relu(conv(x, spec.stem))), 3, 2, 1)
        for blk in spec.blocks:
            r = h
            for c in blk.convs:
                h = conv(h, c)
                h = st(F.relu(h) if c.relu else h) if c is not blk.convs[-1] else h
            if blk.shortcut is not None:
                r = st(conv(r, blk.shortcut))
            h = st(F.relu(h + r))
        lg = F.linear(h.mean(dim=(2, 3)), sd["model.classifier.1.weight"], sd["model.classifier.1.bias"])
    return lg[:, 1] - lg[:, 0]


torch.set_num_threads(os.cpu_count())
ref = forward(set())
print(f"pairs {P}; decision variable l1-l0: rms {ref.pow(2).mean().sqrt():.3f}, range [{ref.min():.3f}, {ref.max():.3f}]")
for name, q in [("proj", {"proj"}), ("maps", {"maps"}), ("w", {"w"}), ("act", {"act"}),
                ("all", {"proj", "maps", "w", "act"}), ("w8", {"w8", "act"}), ("a8", {"a8", "w", "act"}),
                ("fp8", {"proj", "maps", "w8", "a8", "act"})]:
    d = (forward(q) - ref).abs()
    print(f"{name:5s} max {d.max():.2e}  rms {d.pow(2).mean().sqrt():.2e}", flush=True)
