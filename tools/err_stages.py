"""Which stored activations carry the bf16 decision error?  (CPU, float64 truth)  Same setup as err_sources.py (bench
widths, seeded weights, ragged keywords); every conv output rounded to bf16 where it is stored (the GPU path's
rounding points), except in the listed places, which stay exact:
  none      everything stored bf16 (err_sources.py "act")
  -stem     the stem / max-pool output exact
  -sN       stage N's tensors (block outputs and the reduce / 3x3 intermediates) exact
  -resid    every block output (the residual stream) exact, intermediates bf16
  -inner    every reduce / 3x3 intermediate exact, block outputs bf16
Prints max / rms |delta(l1 - l0)|: what a wider storage format for that part alone would buy the exactness band.
usage: python tools/err_stages.py [pairs]"""
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
kmask = (torch.arange(150)[None, :] < lens[:, None]).double()
kwd = kwd * kmask[:, None, :, None]
kmask_p = F.max_pool1d(kmask[:, None], 3, 2, 1)[:, 0]


def bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def folded(c):
    p = f"{c.prefix}.normalization"
    s = sd[f"{p}.weight"] / torch.sqrt(sd[f"{p}.running_var"] + 1e-5)
    return sd[f"{c.prefix}.convolution.weight"] * s[:, None, None, None], sd[f"{p}.bias"] - sd[f"{p}.running_mean"] * s


with torch.no_grad():
    pu, pk = tr.project(utt, sd, 3, True), tr.project(kwd, sd, 3, True)
    sims = []
    for l in range(3):
        a = pu[:, l] / pu[:, l].norm(dim=-1, keepdim=True)
        b = pk[:, l] / pk[:, l].norm(dim=-1, keepdim=True)
        sims.append(torch.einsum("kfd,ud->kfu", b, a[0]))
    MAPS = torch.stack(sims, 1) * kmask_p[:, None, :, None]
stage_of = []
depths = [3, 4, 6, 3]
for si, d_ in enumerate(depths):
    stage_of += [si + 1] * d_


def forward(exact):
    def st(h, where, kind):
        keep = where in exact or kind in exact
        return h if keep else bf(h)
    with torch.no_grad():
        def conv(h, c):
            w, b = folded(c)
            return F.conv2d(h, w, b, stride=c.stride, padding=c.k // 2)
        h = F.max_pool2d(st(F.relu(conv(MAPS, spec.stem)), "stem", "stem"), 3, 2, 1)
        for bi, blk in enumerate(spec.blocks):
            where = f"s{stage_of[bi]}"
            r = h
            for c in blk.convs:
                h = conv(h, c)
                if c is not blk.convs[-1]:
                    h = st(F.relu(h) if c.relu else h, where, "inner")
            if blk.shortcut is not None:
                r = st(conv(r, blk.shortcut), where, "inner")
            h = st(F.relu(h + r), where, "resid")
        lg = F.linear(h.mean(dim=(2, 3)), sd["model.classifier.1.weight"], sd["model.classifier.1.bias"])
    return lg[:, 1] - lg[:, 0]


torch.set_num_threads(os.cpu_count())
ref = forward({"stem", "s1", "s2", "s3", "s4"})
print(f"pairs {P}; decision variable l1-l0: rms {ref.pow(2).mean().sqrt():.3f}")
for name, ex in [("none", set()), ("-stem", {"stem"}), ("-s1", {"s1"}), ("-s2", {"s2"}), ("-s3", {"s3"}),
                 ("-s4", {"s4"}), ("-resid", {"resid"}), ("-inner", {"inner"})]:
    d = (forward(ex) - ref).abs()
    print(f"{name:7s} max {d.max():.2e}  rms {d.pow(2).mean().sqrt():.2e}", flush=True)
