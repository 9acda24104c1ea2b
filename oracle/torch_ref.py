"""ORACLE (test infrastructure only) — torch-fp32 CPU restatement of the reference path, with the same
torch ops the reference calls, for bench.py's ``cpu_baseline`` leg (the reference itself cannot travel to
the GPU box).  Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` may import it; the product never does.

* log-mel: HF ``WhisperFeatureExtractor._torch_extract_fbank_features`` (installed
  ``feature_extraction_whisper.py:135-170``; call site src/utils.py:186-187): ``torch.stft`` (periodic
  Hann 400, hop 160, center/reflect), |X|^2 without the last frame, slaney mel filters, log10 clamp,
  max - 8 floor, (x + 4) / 4;
* encoder: HF ``WhisperEncoder.forward(output_hidden_states=True)`` (src/model/cb_whisper.py:100-104) in
  eager attention (``F.conv1d``, ``F.gelu``, ``F.layer_norm``, ``torch.matmul``/``softmax``), then
  ``hidden_states[ids]`` / L2 norm (:104-106);
* efficient_kws: ``KWSModel.forward`` (src/efficient_kws/model.py:129-208): projector ``F.linear``/ReLU,
  time projector ``F.conv1d`` + ``F.batch_norm`` (eval) + ``F.max_pool1d``, ``sim_matrix`` (:210-218,
  ``F.normalize``-style clamp + ``torch.bmm``), masks (LEF masks max-pooled, DESIGN.md §4 deviation 1),
  HF ``ResNetModel`` (``F.conv2d`` + ``F.batch_norm`` eval + ReLU + ``F.max_pool2d``, stride in the 3x3)
  + ``Linear(2048, 2)`` (src/efficient_kws/resnet.py:51-58).

Pinned to the numpy oracle (itself pinned to the reference fixtures) by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _t(a):
    return a if torch.is_tensor(a) else torch.from_numpy(np.asarray(a, dtype=np.float32))


def log_mel(pcm, n_mel: int) -> torch.Tensor:
    from oracle.mel import N_FFT, HOP, pad_or_trim, mel_filters
    x = torch.from_numpy(pad_or_trim(np.asarray(pcm, np.float32)))
    win = torch.hann_window(N_FFT)
    st = torch.stft(x, N_FFT, HOP, window=win, return_complex=True)
    power = st[..., :-1].abs() ** 2
    fb = torch.from_numpy(mel_filters(n_mel).astype(np.float32))        # [201, n_mel]
    mel = fb.T @ power
    log_spec = torch.clamp(mel, min=1e-10).log10()
    log_spec = torch.maximum(log_spec, log_spec.max() - 8.0)
    return (log_spec + 4.0) / 4.0


def encoder_hidden_states(sd: dict, mel: torch.Tensor, n_heads: int, n_layers: int | None = None) -> list:
    """mel [n_mel, 3000] -> N+1 hidden states [1500, D] (fp32); the last is post-LN."""
    g = lambda k: _t(sd[k])   # noqa: E731
    x = F.gelu(F.conv1d(mel[None], g("conv1.weight"), g("conv1.bias"), padding=1))
    x = F.gelu(F.conv1d(x, g("conv2.weight"), g("conv2.bias"), stride=2, padding=1))
    h = x[0].T + g("embed_positions.weight")[: x.shape[2]]
    T, D = h.shape
    hd = D // n_heads
    N = len({k.split(".")[1] for k in sd if k.startswith("layers.")}) if n_layers is None else n_layers
    states = [h]
    for i in range(N):
        p = f"layers.{i}"
        a = F.layer_norm(h, (D,), g(f"{p}.self_attn_layer_norm.weight"), g(f"{p}.self_attn_layer_norm.bias"))
        q = F.linear(a, g(f"{p}.self_attn.q_proj.weight"), g(f"{p}.self_attn.q_proj.bias")) * hd ** -0.5
        k = F.linear(a, g(f"{p}.self_attn.k_proj.weight"))
        v = F.linear(a, g(f"{p}.self_attn.v_proj.weight"), g(f"{p}.self_attn.v_proj.bias"))
        q, k, v = (t.view(T, n_heads, hd).transpose(0, 1) for t in (q, k, v))
        att = torch.softmax(torch.matmul(q, k.transpose(1, 2)), dim=-1)
        o = torch.matmul(att, v).transpose(0, 1).reshape(T, D)
        h = h + F.linear(o, g(f"{p}.self_attn.out_proj.weight"), g(f"{p}.self_attn.out_proj.bias"))
        a = F.layer_norm(h, (D,), g(f"{p}.final_layer_norm.weight"), g(f"{p}.final_layer_norm.bias"))
        a = F.gelu(F.linear(a, g(f"{p}.fc1.weight"), g(f"{p}.fc1.bias")))
        h = h + F.linear(a, g(f"{p}.fc2.weight"), g(f"{p}.fc2.bias"))
        states.append(h)
    if n_layers is None:
        states[-1] = F.layer_norm(h, (D,), g("layer_norm.weight"), g("layer_norm.bias"))
    return states


def _bn(x, sd, p):
    return F.batch_norm(x, _t(sd[f"{p}.running_mean"]), _t(sd[f"{p}.running_var"]), _t(sd[f"{p}.weight"]),
                        _t(sd[f"{p}.bias"]), training=False, eps=1e-5)


def project(x: torch.Tensor, sd: dict, n_layers: int, frames_conv: bool) -> torch.Tensor:
    """model.py:143-166: x [B, L, T, D] -> [B, L, T', U]."""
    outs = []
    for i in range(n_layers):
        h = F.relu(F.linear(x[:, i], _t(sd[f"projector.{i}.0.weight"]), _t(sd[f"projector.{i}.0.bias"])))
        h = F.linear(h, _t(sd[f"projector.{i}.2.weight"]), _t(sd[f"projector.{i}.2.bias"]))
        if frames_conv:
            p = f"time_projector.{i}"
            t = F.conv1d(h.transpose(1, 2), _t(sd[f"{p}.0.weight"]), _t(sd[f"{p}.0.bias"]), padding=1)
            t = F.max_pool1d(_bn(t, sd, f"{p}.1"), 3, 2, 1)
            h = t.transpose(1, 2)
        outs.append(h)
    return torch.stack(outs, 1)


def resnet_forward(sd: dict, x: torch.Tensor, version: str = "resnet-50") -> torch.Tensor:
    from cbw.synth import resnet_spec   # topology table only (names/shapes)
    spec = resnet_spec(x.shape[1], version)

    def conv_bn(h, c):
        h = F.conv2d(h, _t(sd[f"{c.prefix}.convolution.weight"]), stride=c.stride, padding=c.k // 2)
        h = _bn(h, sd, f"{c.prefix}.normalization")
        return F.relu(h) if c.relu else h

    h = F.max_pool2d(conv_bn(x, spec.stem), 3, 2, 1)
    for b in spec.blocks:
        r = h
        for c in b.convs:
            h = conv_bn(h, c)
        if b.shortcut is not None:
            r = conv_bn(r, b.shortcut)
        h = F.relu(h + r)
    return F.linear(h.mean(dim=(2, 3)), _t(sd["model.classifier.1.weight"]), _t(sd["model.classifier.1.bias"]))


def kws_forward(sd: dict, hp: dict, kwd, utt, kwd_mask, utt_mask, group: int = 50) -> torch.Tensor:
    """KWSModel.forward per group of ``group`` keywords (eval-*.yaml hotwords_per_group 50) -> logits [K, 2]."""
    L = hp["n_layers"]
    learned = hp.get("learn_features", False) and hp.get("proj_mlp", False)
    frames_conv = learned and hp.get("frames_conv", False)
    kwd, utt, kwd_mask, utt_mask = (_t(a) for a in (kwd, utt, kwd_mask, utt_mask))
    with torch.inference_mode():
        pu = project(utt, sd, L, frames_conv) if learned else utt
        um = F.max_pool1d(utt_mask, 3, 2, 1) if frames_conv else utt_mask
        out = []
        for k0 in range(0, kwd.shape[0], group):
            kd, km = kwd[k0:k0 + group], kwd_mask[k0:k0 + group]
            pk = project(kd, sd, L, frames_conv) if learned else kd
            if frames_conv:
                km = F.max_pool1d(km, 3, 2, 1)
            K = pk.shape[0]
            sims = []
            for l in range(L):
                a = pu[:, l].expand(K, -1, -1)
                a = a / a.norm(dim=-1, keepdim=True).clamp_min(1e-6)
                b = pk[:, l] / pk[:, l].norm(dim=-1, keepdim=True).clamp_min(1e-6)
                sims.append(torch.bmm(a, b.transpose(1, 2)).transpose(1, 2))   # [K, Tk, Tu]
            x = torch.stack(sims, 1) * um[:, :, None, :] * km[..., None]
            out.append(resnet_forward(sd, x, hp.get("resnet_version", "resnet-50") if learned else "resnet-50"))
        return torch.cat(out, 0)
