"""First-contact GPU probe: numerics of every libcbw entry point vs oracle/goldens,
plus a rough throughput number.  Prints a report; exits non-zero on NaN/crash only."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "enhance-cb-whisper_amd"), os.path.join(REPO, "tests")]

from cbw import synth, _lib  # noqa: E402
from cbw.kws import KwsEngine, spot  # noqa: E402
import oracle.kws as okws  # noqa: E402
from golden_cases import KWS_CASES  # noqa: E402

G = os.path.join(REPO, "tests", "golden")
dev = torch.device("cuda:0")


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-12, np.abs(b).max()))


def conv_ref(x, w, b, stride, pad):
    xt = torch.from_numpy(x).double().permute(0, 3, 1, 2)
    wt = torch.from_numpy(w).double().permute(0, 3, 1, 2)
    y = torch.nn.functional.conv2d(xt, wt, torch.from_numpy(b).double(), stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1).numpy()


def probe_conv():
    lib = _lib.load()
    rng = np.random.default_rng(0)
    for (N, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw) in [
        (2, 19, 37, 64, 64, 1, 1, 1, 1, 0, 0), (2, 19, 37, 64, 256, 1, 1, 1, 1, 0, 0),
        (2, 19, 37, 128, 128, 3, 3, 1, 1, 1, 1), (3, 10, 23, 64, 64, 3, 3, 2, 2, 1, 1),
        (2, 10, 23, 256, 512, 1, 1, 2, 2, 0, 0), (1, 1, 300, 128, 128, 1, 3, 1, 2, 0, 1),
        (1, 1, 777, 192, 320, 1, 1, 1, 1, 0, 0)]:
        x = rng.standard_normal((N, H, W, Cin)).astype(np.float32)
        w = (rng.standard_normal((Cout, KH, KW, Cin)) / np.sqrt(Cin * KH * KW)).astype(np.float32)
        b = rng.standard_normal(Cout).astype(np.float32)
        xb = torch.from_numpy(x).to(torch.bfloat16)
        wb = torch.from_numpy(w).to(torch.bfloat16)
        Ho = (H + 2 * ph - KH) // sh + 1
        Wo = (W + 2 * pw - KW) // sw + 1
        res = rng.standard_normal((N, Ho, Wo, Cout)).astype(np.float32)
        resb = torch.from_numpy(res).to(torch.bfloat16)
        y = torch.empty((N, Ho, Wo, Cout), dtype=torch.bfloat16, device=dev)
        xd, wd, bd, rd = xb.to(dev), wb.to(dev), torch.from_numpy(b).to(dev), resb.to(dev)
        rc = lib.cbw_conv2d(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), rd.data_ptr(), y.data_ptr(), N, H, W, Cin,
                            Cout, KH, KW, sh, sw, ph, pw, 1, _lib.stream_handle())
        _lib.check(rc, "conv2d")
        torch.cuda.synchronize()
        ref = conv_ref(xb.float().numpy(), wb.float().numpy(), b, (sh, sw), (ph, pw)) + resb.float().numpy()
        ref = np.maximum(ref, 0)
        print(f"conv N{N} {H}x{W} {Cin}->{Cout} k{KH}x{KW} s{sh},{sw}: rel err {rel(y.float().cpu().numpy(), ref):.3e}")


def probe_kws():
    for name, (hp, bk) in KWS_CASES.items():
        g = np.load(os.path.join(G, f"kws_{name}.npz"))
        sd = synth.synth_kws_state_dict(seed=0, **hp)
        b = synth.synth_kws_batch(n_layers=hp["n_layers"], D=hp["embedding_dim"], **bk)
        eng = KwsEngine(hp, sd)
        pk, pkm = eng.project(torch.from_numpy(b["kwd"]).to(dev), torch.from_numpy(b["kwd_mask"]).to(dev))
        pu, pum = eng.project(torch.from_numpy(b["utt"]).to(dev), torch.from_numpy(b["utt_mask"]).to(dev))
        logits, feats = eng.score(pu[0], pum[0], pk, pkm, features=True)
        prob, idx = spot(logits, torch.from_numpy(b["ghost_mask"]).to(dev), 0.5)
        torch.cuda.synchronize()
        lg = logits.cpu().numpy()
        f = feats.cpu().numpy()
        print(f"kws {name}: logits rel {rel(lg, g['logits']):.3e}  feat_sub maxabs "
              f"{np.abs(f[:, :, ::7, ::11] - g['feat_sub']).max():.3e}  probs maxabs "
              f"{np.abs(prob.cpu().numpy() - g['probs']).max():.3e}  idx {idx.tolist()} vs {g['idx_0.5'].tolist()}")
        print("   gpu", np.round(lg, 3).tolist())
        print("   ref", np.round(g["logits"], 3).tolist())


def probe_mel():
    from cbw.whisper import log_mel
    for n_mel in (80, 128):
        g = np.load(os.path.join(G, f"mel_{n_mel}.npz"))
        m, pk = log_mel(torch.from_numpy(synth.synth_clip(0)).to(dev), n_mel, packed=True)
        torch.cuda.synchronize()
        print(f"mel {n_mel}: maxabs {np.abs(m.cpu().numpy() - g['noise_sines']).max():.3e}")


def probe_encoder():
    from cbw.whisper import EncoderEngine
    g = np.load(os.path.join(G, "encoder_micro.npz"))
    cfg = synth.WHISPER_CONFIGS["micro"]
    sd = synth.synth_whisper_encoder_state_dict("micro", seed=0)
    eng = EncoderEngine(cfg, sd)
    mel = torch.from_numpy(g["mel"]).to(dev)
    pk = torch.zeros((3000, eng.cpad), dtype=torch.bfloat16, device=dev)
    pk[:, : cfg[0]] = mel.t().to(torch.bfloat16)
    ids = list(range(cfg[2] + 1))
    hs = eng.hidden_states(pk, ids, normalize=False)
    torch.cuda.synchronize()
    h = hs[0].cpu().numpy()
    for i in ids:
        print(f"encoder hs[{i}] rel {rel(h[i], g['hidden_states'][i]):.3e}")


def probe_speed():
    hp = dict(n_layers=3, embedding_dim=1280, learn_features=True, proj_mlp=True, frames_conv=True, proj_mlp_units=64)
    sd = synth.synth_kws_state_dict(seed=0, **hp)
    eng = KwsEngine(hp, sd)
    K = 1024
    pk = (torch.randn(K, 3, 75, 64, device=dev)).to(torch.bfloat16)
    pkm = torch.ones(K, 3, 75, device=dev)
    pu = torch.randn(3, 750, 64, device=dev).to(torch.bfloat16)
    pum = torch.ones(3, 750, device=dev)
    for chunk in (128, 256, 512):
        eng.score(pu, pum, pk, pkm, chunk=chunk)
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(3):
            eng.score(pu, pum, pk, pkm, chunk=chunk)
        torch.cuda.synchronize()
        dt = (time.time() - t) / 3
        print(f"score K={K} chunk={chunk}: {dt*1e3:.1f} ms  -> {K*10.08e9/dt/1e12:.1f} TFLOP/s (resnet algorithmic)"
              f"  pairs/s {K/dt:.0f}")


if __name__ == "__main__":
    torch.cuda.set_device(0)
    for fn in (probe_conv, probe_kws, probe_mel, probe_encoder, probe_speed):
        try:
            fn()
        except Exception as e:  # keep probing the rest
            print(f"{fn.__name__} FAILED: {type(e).__name__}: {e}")
        sys.stdout.flush()
