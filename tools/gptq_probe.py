"""Can error-aware rounding of the bf16 conv weights shrink the exact-decision band?  (CPU, float64 truth)

Same scorer, widths and seeded weights as tools/err_sources.py.  For every conv (stem included) the input
second-moment matrix H = E[u u^T] over im2col patches u of the float64 forward is accumulated on calibration
pairs (other keywords, another utterance), and each weight matrix is rounded to bf16 column by column with the
rounding error of column i pushed onto the not-yet-rounded columns through the Cholesky factor of H^-1
(the OBQ / GPTQ update), instead of round-to-nearest.  Reported on held-out pairs: max / rms |delta(l1 - l0)|
of the decision variable for
  w_rtn      round-to-nearest weights (+ the mean-shift bias correction the GPU path applies)
  w_gptq     error-aware rounding (+ the same bias correction on what is left)
  all_rtn    + bf16 projections, maps and stored activations (the bf16 GPU path, bias-corrected)
  all_gptq   the same with error-aware weights
usage: python tools/gptq_probe.py [eval_pairs] [cal_pairs]
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
PC = int(sys.argv[2]) if len(sys.argv) > 2 else 16
D = 1280
hp = dict(n_layers=3, embedding_dim=D, learn_features=True, proj_mlp=True, frames_conv=True, proj_mlp_units=64,
          resnet_version="resnet-50", threshold=0.5)
sd = {k: torch.from_numpy(v).double() for k, v in synth.synth_kws_state_dict(seed=0, **hp).items()}
spec = synth.resnet_spec(3, "resnet-50")
convs = [spec.stem] + [c for b in spec.blocks for c in ([b.shortcut] if b.shortcut is not None else []) + b.convs]


def batch(seed, n):
    g = torch.Generator().manual_seed(seed)
    utt = torch.randn((1, 3, 1500, D), generator=g, dtype=torch.float64)
    utt = utt / utt.norm(dim=-1, keepdim=True)
    kwd = torch.randn((n, 3, 150, D), generator=g, dtype=torch.float64)
    kwd = kwd / kwd.norm(dim=-1, keepdim=True)
    lens = torch.randint(8, 151, (n,), generator=g)
    km = (torch.arange(150)[None, :] < lens[:, None]).double()
    return utt, kwd * km[:, None, :, None], F.max_pool1d(km[:, None], 3, 2, 1)[:, 0]


def bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def folded(c):
    p = f"{c.prefix}.normalization"
    s = sd[f"{p}.weight"] / torch.sqrt(sd[f"{p}.running_var"] + 1e-5)
    return sd[f"{c.prefix}.convolution.weight"] * s[:, None, None, None], sd[f"{p}.bias"] - sd[f"{p}.running_mean"] * s


FOLD = {c.prefix: folded(c) for c in convs}


def forward(data, q, W=None, hook=None):
    """q: subset of {proj, maps, act}; W: prefix -> (weight, bias) used instead of the float64 folded ones."""
    utt, kwd, kmp = data
    with torch.no_grad():
        pu, pk = tr.project(utt, sd, 3, True), tr.project(kwd, sd, 3, True)
        if "proj" in q:
            pu, pk = bf(pu), bf(pk)
        sims = []
        for l in range(3):
            a = pu[:, l] / pu[:, l].norm(dim=-1, keepdim=True)
            b = pk[:, l] / pk[:, l].norm(dim=-1, keepdim=True)
            sims.append(torch.einsum("kfd,ud->kfu", b, a[0]))
        x = torch.stack(sims, 1) * kmp[:, None, :, None]
        if "maps" in q:
            x = bf(x)

        def conv(h, c):
            w, b = (W or FOLD)[c.prefix]
            if hook is not None:
                hook(c, h)
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
cal = batch(101, PC)
H, MU, CNT = {}, {}, {}


def acc(c, h):
    u = F.unfold(h, c.k, padding=c.k // 2, stride=c.stride)          # [n, K, L], K ordered (cin, kh, kw)
    u = u.transpose(1, 2).reshape(-1, u.shape[1])
    H[c.prefix] = H.get(c.prefix, 0) + u.T @ u
    MU[c.prefix] = MU.get(c.prefix, 0) + u.sum(0)
    CNT[c.prefix] = CNT.get(c.prefix, 0) + u.shape[0]


for i in range(0, PC, 4):   # calibration statistics of the float64 network, 4 pairs at a time
    forward((cal[0], cal[1][i:i + 4], cal[2][i:i + 4]), set(), hook=acc)
print(f"calibration: {PC} pairs, {len(H)} convs", flush=True)


def gptq(w, Hm, damp=1e-2):
    """OBQ / GPTQ column sweep with the bf16 grid: w [Cout, K] float64, Hm [K, K]."""
    w = w.clone()
    K = w.shape[1]
    Hd = Hm.clone()
    dead = torch.diag(Hd) == 0
    Hd[dead, dead] = 1
    w[:, dead] = 0
    Hd += damp * torch.diag(Hd).mean() * torch.eye(K, dtype=Hd.dtype)
    Hinv = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hd)), upper=True)
    q = torch.empty_like(w)
    for i in range(K):
        qi = bf(w[:, i])
        q[:, i] = qi
        e = (w[:, i] - qi) / Hinv[i, i]
        w[:, i + 1:] -= e[:, None] * Hinv[i, i + 1:][None, :]
    return q


def bias_corrected(c, wq):
    w, b = FOLD[c.prefix]
    mu = MU[c.prefix] / CNT[c.prefix]
    return wq, b + (w - wq).reshape(w.shape[0], -1) @ mu


W_RTN, W_GPTQ = {}, {}
for c in convs:
    w, _ = FOLD[c.prefix]
    W_RTN[c.prefix] = bias_corrected(c, bf(w))
    Hm = H[c.prefix] / CNT[c.prefix]
    wq = gptq(w.reshape(w.shape[0], -1), Hm).reshape(w.shape)
    W_GPTQ[c.prefix] = bias_corrected(c, wq)
    # per-layer output error proxy tr(dW H dW^T) for both roundings
    d1 = (w - bf(w)).reshape(w.shape[0], -1)
    d2 = (w - wq).reshape(w.shape[0], -1)
    e1 = torch.einsum("ok,kl,ol->", d1, Hm, d1).item()
    e2 = torch.einsum("ok,kl,ol->", d2, Hm, d2).item()
    if os.environ.get("GP_VERBOSE"):
        print(f"  {c.prefix:55s} K {d1.shape[1]:5d}  E|dy|^2 rtn {e1:.3e}  gptq {e2:.3e}  ({e2 / max(e1, 1e-300):.2f}x)",
          flush=True)

ev = batch(7, P)
ref = forward(ev, set())
print(f"eval pairs {P}; decision variable l1-l0 rms {ref.pow(2).mean().sqrt():.3f}")
for name, q, W in [("w_rtn", set(), W_RTN), ("w_gptq", set(), W_GPTQ),
                   ("all_rtn", {"proj", "maps", "act"}, W_RTN), ("all_gptq", {"proj", "maps", "act"}, W_GPTQ)]:
    d = forward(ev, q, W) - ref
    dc = d - d.mean()   # what the logit-offset calibration leaves (it removes the mean error)
    print(f"{name:9s} max |d| {d.abs().max():.3e}  rms {d.pow(2).mean().sqrt():.3e}  mean {d.mean():+.3e}  "
          f"centred: max {dc.abs().max():.3e} std {dc.pow(2).mean().sqrt():.3e}", flush=True)
