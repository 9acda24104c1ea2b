"""KWS classifier engine over libcbw (LE/LEF projection, similarity maps, ResNet, decision).

Host-side owner of one ``cbw_kws`` handle: loads a reference-format state dict
(``KWSModel.state_dict()`` names, see cbw.synth.kws_param_shapes), lets the
native runtime fold BatchNorm and upload bf16 weights, and runs the hot path on
torch-owned device buffers.  Reference semantics per call are cited in
include/cbw.h.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib

VARIANT_L, VARIANT_LE, VARIANT_LEF = 0, 1, 2
RESNET_DEPTH = {"resnet-50": 50, "resnet-34": 34, "resnet-18": 18}


def variant_of(hp: dict) -> int:
    """efficient_kws/model.py:71-124.  learn_features=False -> L (Resnet on raw-hs
    similarities).  learn_features & proj_mlp -> LE (+frames_conv -> LEF).
    learn_features & !proj_mlp builds no classifier in the reference
    (AttributeError); the build treats it as L."""
    if hp.get("learn_features", False) and hp.get("proj_mlp", False):
        return VARIANT_LEF if hp.get("frames_conv", False) else VARIANT_LE
    return VARIANT_L


def lef_frames(T: int) -> int:
    """MaxPool1d(3, 2, 1) output length (model.py:120-122)."""
    return (T - 1) // 2 + 1


class KwsEngine:
    def __init__(self, hp: dict, state_dict: Dict[str, object], device: Optional[torch.device] = None,
                 classifier_only: bool = False):
        """``classifier_only``: a handle for the ResNet alone (efficient_kws/resnet.py:7-58 as its own module):
        no projector parameters, ``hp['resnet_version']`` honoured; only ``classify`` is usable."""
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.hp = dict(hp)
        self.variant = VARIANT_L if classifier_only else variant_of(hp)
        self.n_layers = int(hp.get("n_layers", 12))
        self.D = int(hp.get("embedding_dim", 1024))
        self.U = int(hp.get("proj_mlp_units", 64))
        version = (hp.get("resnet_version", "resnet-50") if self.variant != VARIANT_L or classifier_only
                   else "resnet-50")
        if version not in RESNET_DEPTH:
            raise ValueError(f"unsupported resnet_version {version}")
        cfg = _lib.KwsConfig(self.n_layers, self.D, self.variant, self.U, RESNET_DEPTH[version])
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.cbw_kws_create(ctypes.byref(cfg), ctypes.byref(h)), "cbw_kws_create")
            self.h = h
            for name, v in state_dict.items():
                if name.endswith("num_batches_tracked"):
                    continue
                a = np.ascontiguousarray(v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v),
                                         dtype=np.float32)
                _lib.check(self.lib.cbw_kws_set_param(self.h, name.encode(), a.ctypes.data, a.size),
                           f"cbw_kws_set_param({name})")
            _lib.check(self.lib.cbw_kws_finalize(self.h), "cbw_kws_finalize")
        self._ws = _lib.Workspace()
        self._ws_rescore = _lib.Workspace()   # the re-scoring tiers' own scratch: they may overlap scoring
        self._pws = _lib.Workspace()

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.cbw_kws_destroy(h)
            except Exception:
                pass

    @property
    def has_fp32(self) -> bool:
        """The fp32 / compensated re-scoring networks exist (cbw_kws_finalize builds them for n_layers <= 4, the
        ResNet input channels the fp32 stem takes; every efficient_kws config uses 3)."""
        return self.n_layers <= 4

    @property
    def feat_dim(self) -> int:
        return self.D if self.variant == VARIANT_L else self.U

    def out_frames(self, T: int) -> int:
        return lef_frames(T) if self.variant == VARIANT_LEF else T

    # ------------------------------------------------------------------ projection
    def project(self, x: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """x f32 [B, L, T, D], mask f32 [B, L, T] (device) -> (bf16 [B, L, T', E], f32 [B, L, T'])."""
        x = x.to(self.device, torch.float32).contiguous()
        mask = mask.to(self.device, torch.float32).contiguous()
        B, L, T, D = x.shape
        if L != self.n_layers or D != self.D:
            raise ValueError(f"expected [B, {self.n_layers}, T, {self.D}] features, got {tuple(x.shape)}")
        if tuple(mask.shape) != (B, L, T):
            raise ValueError(f"mask shape {tuple(mask.shape)} != {(B, L, T)}")
        To = self.out_frames(T)
        out = torch.empty((B, L, To, self.feat_dim), dtype=torch.bfloat16, device=self.device)
        mout = torch.empty((B, L, To), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_kws_project_workspace_bytes(self.h, B, T)
            ws = self._pws.get(nb, self.device)
            _lib.check(self.lib.cbw_kws_project(self.h, x.data_ptr(), mask.data_ptr(), B, T, out.data_ptr(),
                                                mout.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle()),
                       "cbw_kws_project")
        return out, mout

    def project_f32(self, x: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """fp32 projection (the exact re-scoring path): x f32 [B, L, T, D] -> (f32 [B, L, T', E], f32 [B, L, T'])."""
        x = x.to(self.device, torch.float32).contiguous()
        mask = mask.to(self.device, torch.float32).contiguous()
        B, L, T, D = x.shape
        if L != self.n_layers or D != self.D or tuple(mask.shape) != (B, L, T):
            raise ValueError(f"expected [B, {self.n_layers}, T, {self.D}] features + [B, L, T] mask")
        To = self.out_frames(T)
        out = torch.empty((B, L, To, self.feat_dim), dtype=torch.float32, device=self.device)
        mout = torch.empty((B, L, To), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_kws_project_f32_workspace_bytes(self.h, B, T)
            ws = self._pws.get(nb, self.device)
            _lib.check(self.lib.cbw_kws_project_f32(self.h, x.data_ptr(), mask.data_ptr(), B, T, out.data_ptr(),
                                                    mout.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle()),
                       "cbw_kws_project_f32")
        return out, mout

    def rescore(self, utt32: torch.Tensor, utt_mask: torch.Tensor, kwd32: torch.Tensor, kwd_mask: torch.Tensor,
                logits: torch.Tensor, sel: torch.Tensor, trusted: bool = False, tier: str = "fp32") -> torch.Tensor:
        """Re-scored ResNet logits for the keywords ``sel`` (indices into kwd32), written into ``logits`` [K, 2]
        in place.  tier "fp32": fp32-input MFMA (cbw_kws_rescore); "x3": compensated bf16, the 3-term split
        on the bf16 MFMA kernels (cbw_kws_rescore_x3).  utt32 f32 [L, Tu, E], kwd32 f32 [K, L, Tk, E]
        from project_f32."""
        if utt32.dim() == 4:
            utt32, utt_mask = utt32[0], utt_mask.reshape(utt_mask.shape[-2:])
        K, L, Tk, E = kwd32.shape
        Tu = utt32.shape[1]
        if utt32.dtype != torch.float32 or kwd32.dtype != torch.float32 or tuple(utt32.shape) != (L, Tu, E):
            raise ValueError("rescore takes the fp32 projections (KwsEngine.project_f32)")
        if tier not in ("fp32", "x3"):
            raise ValueError(f"unknown re-scoring tier {tier}")
        sel = sel.to(self.device, torch.int32).contiguous()
        n = sel.numel()
        if n == 0:
            return logits
        if tuple(logits.shape) != (K, 2) or tuple(kwd_mask.shape) != (K, L, Tk):
            # sel indexes the logits rows and the keyword rows alike (``trusted`` skips only the sel range check)
            raise ValueError(f"rescore: logits {tuple(logits.shape)} / mask {tuple(kwd_mask.shape)} for {K} keywords")
        if not trusted and (int(sel.min()) < 0 or int(sel.max()) >= K):
            raise ValueError("sel out of range")
        wsq, call = ((self.lib.cbw_kws_rescore_workspace_bytes, self.lib.cbw_kws_rescore) if tier == "fp32" else
                     (self.lib.cbw_kws_rescore_x3_workspace_bytes, self.lib.cbw_kws_rescore_x3))
        with torch.cuda.device(self.device):
            nb = wsq(self.h, Tk, Tu)
            if nb < 0:
                _lib.check(-4, f"cbw_kws_rescore ({tier}) workspace")
            ws = self._ws_rescore.get(nb, self.device)
            _lib.check(call(self.h, utt32.contiguous().data_ptr(), utt_mask.to(torch.float32).contiguous().data_ptr(),
                            kwd32.contiguous().data_ptr(), kwd_mask.to(torch.float32).contiguous().data_ptr(), K, Tk,
                            Tu, sel.data_ptr(), n, logits.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle()),
                       f"cbw_kws_rescore ({tier})")
        return logits

    def calibrate_bias(self, utt32: Optional[torch.Tensor] = None, utt_mask: Optional[torch.Tensor] = None,
                       kwd32: Optional[torch.Tensor] = None, kwd_mask: Optional[torch.Tensor] = None,
                       sel: Optional[torch.Tensor] = None, utt: Optional[torch.Tensor] = None,
                       kwd: Optional[torch.Tensor] = None) -> Optional[np.ndarray]:
        """Bias correction of the bf16 scoring network (cbw_kws_calibrate_bias): the fp32 network over the
        calibration pairs ``sel`` (default: every keyword of kwd32) gives each conv's mean input per channel,
        and the bf16 convs' biases absorb the mean shift of their rounded weights.  With the bf16 projections of
        the same pairs (``utt`` [L, Tu, E], ``kwd`` [K, L, Tk, E] bf16, masks shared), the mean fp32 - bf16 logit
        difference that remains is then taken out of the bf16 pass's classifier bias (cbw_kws_set_score_offset)
        and returned.  Inputs as rescore; no arguments restores the folded biases and a zero offset.
        Setup-time (synchronises)."""
        if utt32 is None:
            with torch.cuda.device(self.device):
                _lib.check(self.lib.cbw_kws_calibrate_bias(self.h, None, None, None, None, 0, 1, 1, None, 0, None, 0,
                                                           _lib.stream_handle()), "cbw_kws_calibrate_bias")
            return
        if utt32.dim() == 4:
            utt32, utt_mask = utt32[0], utt_mask.reshape(utt_mask.shape[-2:])
        K, L, Tk, E = kwd32.shape
        Tu = utt32.shape[1]
        if utt32.dtype != torch.float32 or kwd32.dtype != torch.float32 or tuple(utt32.shape) != (L, Tu, E):
            raise ValueError("calibrate_bias takes the fp32 projections (KwsEngine.project_f32)")
        if sel is None:
            sel = torch.arange(K, dtype=torch.int32, device=self.device)
        sel = sel.to(self.device, torch.int32).contiguous()
        if sel.numel() == 0 or int(sel.min()) < 0 or int(sel.max()) >= K:
            raise ValueError("calibration pairs out of range")
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_kws_rescore_workspace_bytes(self.h, Tk, Tu)
            if nb < 0:
                _lib.check(-4, "cbw_kws_calibrate_bias workspace")
            ws = self._ws_rescore.get(nb, self.device)
            _lib.check(self.lib.cbw_kws_calibrate_bias(
                self.h, utt32.contiguous().data_ptr(), utt_mask.to(torch.float32).contiguous().data_ptr(),
                kwd32.contiguous().data_ptr(), kwd_mask.to(torch.float32).contiguous().data_ptr(), K, Tk, Tu,
                sel.data_ptr(), sel.numel(), ws.data_ptr(), ws.numel(), _lib.stream_handle()), "cbw_kws_calibrate_bias")
        if utt is None or kwd is None:
            return None
        zero = np.zeros(2, np.float32)
        _lib.check(self.lib.cbw_kws_set_score_offset(self.h, zero.ctypes.data), "cbw_kws_set_score_offset")
        if utt.dim() == 4:
            utt = utt[0]
        s_l = sel.long()
        km = kwd_mask[s_l].contiguous()
        l16 = self.score(utt, utt_mask, kwd[s_l].contiguous(), km)
        l32 = l16.clone()
        self.rescore(utt32, utt_mask, kwd32[s_l].contiguous(), km, l32,
                     torch.arange(sel.numel(), dtype=torch.int32, device=self.device), trusted=True)
        off = (l32.double() - l16.double()).mean(0).cpu().numpy().astype(np.float32)
        _lib.check(self.lib.cbw_kws_set_score_offset(self.h, np.ascontiguousarray(off).ctypes.data),
                   "cbw_kws_set_score_offset")
        return off

    # ------------------------------------------------------------------ fp8 first tier
    def calibrate_fp8(self, utt32: torch.Tensor, utt_mask: torch.Tensor, kwd32: torch.Tensor, kwd_mask: torch.Tensor,
                      sel: Optional[torch.Tensor] = None, margin: float = 1.0, utt: Optional[torch.Tensor] = None,
                      kwd: Optional[torch.Tensor] = None) -> Optional[np.ndarray]:
        """Build the fp8 tier (cbw_kws_calibrate_fp8): the fp32 network over the calibration pairs ``sel``
        (default: every keyword of kwd32) gives each stage-2..4 tensor's absolute maximum, its e4m3 scale is
        amax * margin / 448 and the weights are quantized against it.  With the bf16 projections of the same pairs
        (``utt`` [L, Tu, E], ``kwd`` [K, L, Tk, E]) the mean fp32 - fp8 logit difference is then moved into the fp8
        pass's classifier bias (cbw_kws_set_score_offset_fp8) and returned.  Setup-time (synchronises)."""
        if utt32.dim() == 4:
            utt32, utt_mask = utt32[0], utt_mask.reshape(utt_mask.shape[-2:])
        K, L, Tk, E = kwd32.shape
        Tu = utt32.shape[1]
        if sel is None:
            sel = torch.arange(K, dtype=torch.int32, device=self.device)
        sel = sel.to(self.device, torch.int32).contiguous()
        if sel.numel() == 0 or int(sel.min()) < 0 or int(sel.max()) >= K:
            raise ValueError("calibration pairs out of range")
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_kws_rescore_workspace_bytes(self.h, Tk, Tu)
            if nb < 0:
                _lib.check(-4, "cbw_kws_calibrate_fp8 workspace")
            ws = self._ws_rescore.get(nb, self.device)
            _lib.check(self.lib.cbw_kws_calibrate_fp8(
                self.h, utt32.contiguous().data_ptr(), utt_mask.to(torch.float32).contiguous().data_ptr(),
                kwd32.contiguous().data_ptr(), kwd_mask.to(torch.float32).contiguous().data_ptr(), K, Tk, Tu,
                sel.data_ptr(), sel.numel(), float(margin), ws.data_ptr(), ws.numel(), _lib.stream_handle()),
                "cbw_kws_calibrate_fp8")
        if utt is None or kwd is None:
            return None
        zero = np.zeros(2, np.float32)
        _lib.check(self.lib.cbw_kws_set_score_offset_fp8(self.h, zero.ctypes.data), "cbw_kws_set_score_offset_fp8")
        if utt.dim() == 4:
            utt = utt[0]
        s_l = sel.long()
        km = kwd_mask[s_l].contiguous()
        l8 = self.score_fp8(utt, utt_mask, kwd[s_l].contiguous(), km)
        l32 = torch.empty_like(l8)
        self.rescore(utt32, utt_mask, kwd32[s_l].contiguous(), km, l32,
                     torch.arange(sel.numel(), dtype=torch.int32, device=self.device), trusted=True)
        off = (l32.double() - l8.double()).mean(0).cpu().numpy().astype(np.float32)
        _lib.check(self.lib.cbw_kws_set_score_offset_fp8(self.h, np.ascontiguousarray(off).ctypes.data),
                   "cbw_kws_set_score_offset_fp8")
        return off

    def fp8_scales(self) -> np.ndarray:
        n = self.lib.cbw_kws_fp8_scales(self.h, None, 0)
        out = np.zeros(max(n, 1), np.float32)
        self.lib.cbw_kws_fp8_scales(self.h, out.ctypes.data, n)
        return out[:n]

    def score_fp8(self, utt: torch.Tensor, utt_mask: torch.Tensor, kwd: torch.Tensor, kwd_mask: torch.Tensor,
                  chunk: Optional[int] = None, logits_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logits of every pair from the fp8 tier (cbw_kws_score_fp8); inputs as ``score``."""
        if utt.dim() == 4:
            utt, utt_mask = utt[0], utt_mask.reshape(utt_mask.shape[-2:])
        K, L, Tk, E = kwd.shape
        Tu = utt.shape[1]
        if L != self.n_layers or E != self.feat_dim or tuple(utt.shape) != (L, Tu, E):
            raise ValueError(f"shape mismatch: kwd {tuple(kwd.shape)} utt {tuple(utt.shape)}")
        if utt.dtype != torch.bfloat16 or kwd.dtype != torch.bfloat16:
            raise ValueError("projected features must be bf16 (use KwsEngine.project)")
        if utt_mask.numel() == L * Tu:
            utt_mask = utt_mask.reshape(L, Tu)
        if tuple(kwd_mask.shape) != (K, L, Tk) or tuple(utt_mask.shape) != (L, Tu):
            raise ValueError("mask shapes")
        chunk = chunk or self.default_chunk(Tk, Tu)
        if logits_out is not None and (tuple(logits_out.shape) != (K, 2) or logits_out.dtype != torch.float32
                                       or not logits_out.is_contiguous()):
            raise ValueError(f"logits_out must be contiguous f32 [{K}, 2]")
        logits = logits_out if logits_out is not None else torch.empty((K, 2), dtype=torch.float32, device=self.device)
        utt, kwd = utt.contiguous(), kwd.contiguous()
        utt_mask = utt_mask.to(torch.float32).contiguous()
        kwd_mask = kwd_mask.to(torch.float32).contiguous()
        with torch.cuda.device(self.device):
            ws = self.workspace(Tk, Tu, chunk)
            _lib.check(self.lib.cbw_kws_score_fp8(self.h, utt.data_ptr(), utt_mask.data_ptr(), kwd.data_ptr(),
                                                  kwd_mask.data_ptr(), K, Tk, Tu, logits.data_ptr(), chunk,
                                                  ws.data_ptr(), ws.numel(), _lib.stream_handle()), "cbw_kws_score_fp8")
        return logits

    def band(self, logits: torch.Tensor, threshold: float, band: float, ghost: Optional[torch.Tensor] = None,
             idx_out: Optional[torch.Tensor] = None, n_out: Optional[torch.Tensor] = None,
             scaled: bool = False) -> Tuple[torch.Tensor, int]:
        """Sorted keyword indices whose probability lies within ``band`` of ``threshold`` (cbw_kws_band), or with
        ``scaled`` within ``band`` x max(|l0|, |l1|) of it (cbw_kws_band_scaled): (device int32 [n], n).  Reads the
        count back to the host (one stream sync)."""
        logits = logits.to(torch.float32).contiguous()
        K = logits.shape[0]
        idx = idx_out if idx_out is not None else torch.empty((max(K, 1),), dtype=torch.int32, device=logits.device)
        n = n_out if n_out is not None else torch.zeros((1,), dtype=torch.int32, device=logits.device)
        g = None if ghost is None else ghost.to(logits.device, torch.float32).contiguous()
        if g is not None and g.numel() != K:
            raise ValueError(f"ghost mask of {g.numel()} entries for {K} logits")
        if idx.numel() < max(K, 1) or n.numel() < 1:
            raise ValueError("band output buffers too small")
        with torch.cuda.device(logits.device):
            fn = self.lib.cbw_kws_band_scaled if scaled else self.lib.cbw_kws_band
            _lib.check(fn(logits.data_ptr(), _lib.ptr(g), K, float(threshold), float(band), idx.data_ptr(),
                          n.data_ptr(), _lib.stream_handle()), "cbw_kws_band")
        cnt = int(n.item())
        return idx[:cnt], cnt

    def score_exact(self, utt: torch.Tensor, utt_mask: torch.Tensor, kwd: torch.Tensor, kwd_mask: torch.Tensor,
                    utt32: torch.Tensor, kwd32: torch.Tensor, threshold: float, band: float,
                    ghost: Optional[torch.Tensor] = None, chunk: Optional[int] = None,
                    logits_out: Optional[torch.Tensor] = None, band_x3: Optional[float] = None,
                    band_scaled: bool = False, fp8_band: Optional[float] = None):
        """bf16 scoring of every pair, then the near-threshold pairs re-scored from the cached fp32
        projections ``utt32`` [L, Tu, E] / ``kwd32`` [K, L, Tk, E] (project_f32):

        * ``band_x3`` None: every pair within ``band`` of ``threshold`` in fp32 (cbw_kws_band + cbw_kws_rescore);
        * ``band_x3`` = b2 < band: the pairs within ``band`` on the compensated-bf16 tier (cbw_kws_rescore_x3),
          then those of them still within b2 of the threshold in fp32.  Pairs outside ``band`` cannot enter b2
          (their logits are untouched), so the fp32 decision is reproduced as long as the bf16 error < band
          and the compensated error < b2.

        ``band_scaled``: the first band is ``band`` x max(|l0|, |l1|) per pair (cbw_kws_band_scaled).

        ``fp8_band`` (the fp8 first tier, calibrate_fp8 first): every pair is scored by the fp8 network
        (score_fp8); only the pairs within ``fp8_band`` of the threshold are scored in bf16 (their keywords gathered
        into one batch), then the tiers above.  Pairs outside ``fp8_band`` keep their fp8 logits and cannot enter
        the later bands (fp8_band > band), so the fp32 decision is reproduced as long as the fp8 error < fp8_band.

        Returns (logits f32 [K, 2], {"band": pairs re-scored after bf16, "fp32": pairs re-scored in fp32,
        "bf16": pairs scored in bf16})."""
        stats = {"band": 0, "fp32": 0, "bf16": kwd.shape[0]}
        if fp8_band is not None and kwd.shape[0] > 0:
            if fp8_band <= band:
                raise ValueError("fp8_band must exceed the bf16 band")
            logits = self.score_fp8(utt, utt_mask, kwd, kwd_mask, chunk=chunk, logits_out=logits_out)
            sel8, n8 = self.band(logits, threshold, fp8_band, ghost)
            stats["bf16"] = n8
            if n8:
                s_l = sel8.long()
                sub = self.score(utt, utt_mask, kwd.index_select(0, s_l), kwd_mask.index_select(0, s_l), chunk=chunk)
                logits.index_copy_(0, s_l, sub)
        else:
            logits = self.score(utt, utt_mask, kwd, kwd_mask, chunk=chunk, logits_out=logits_out)
        if band <= 0 or kwd.shape[0] == 0:
            return logits, stats
        sel, n = self.band(logits, threshold, band, ghost, scaled=band_scaled)
        stats["band"] = n
        if n == 0:
            return logits, stats
        um = utt_mask.reshape(utt_mask.shape[-2:]) if utt_mask.dim() == 3 else utt_mask
        if band_x3 is None:
            self.rescore(utt32, um, kwd32, kwd_mask, logits, sel, trusted=True)
            stats["fp32"] = n
            return logits, stats
        self.rescore(utt32, um, kwd32, kwd_mask, logits, sel, trusted=True, tier="x3")
        sel2, n2 = self.band(logits, threshold, band_x3, ghost)
        if n2:
            self.rescore(utt32, um, kwd32, kwd_mask, logits, sel2, trusted=True)
        stats["fp32"] = n2
        return logits, stats

    # ------------------------------------------------------------------ scoring
    def default_chunk(self, Tk: int, Tu: int, budget_bytes: int = 2 << 30) -> int:
        per = self.lib.cbw_kws_workspace_bytes(self.h, Tk, Tu, 1)
        return int(max(1, min(1024, budget_bytes // max(per, 1))))

    def workspace(self, Tk: int, Tu: int, chunk: int) -> torch.Tensor:
        nb = self.lib.cbw_kws_workspace_bytes(self.h, Tk, Tu, chunk)
        if nb < 0:
            raise ValueError("bad workspace query")
        return self._ws.get(nb, self.device)

    def score(self, utt: torch.Tensor, utt_mask: torch.Tensor, kwd: torch.Tensor, kwd_mask: torch.Tensor,
              features: bool = False, chunk: Optional[int] = None, logits_out: Optional[torch.Tensor] = None):
        """utt bf16 [L, Tu, E] (or [1, L, Tu, E]), utt_mask f32 [L, Tu]; kwd bf16 [K, L, Tk, E],
        kwd_mask f32 [K, L, Tk]  ->  logits f32 [K, 2] (+ features f32 [K, L, Tk, Tu])."""
        if utt.dim() == 4:
            utt, utt_mask = utt[0], utt_mask.reshape(utt_mask.shape[-2:])
        K, L, Tk, E = kwd.shape
        Tu = utt.shape[1]
        if L != self.n_layers or E != self.feat_dim or tuple(utt.shape) != (L, Tu, E):
            raise ValueError(f"shape mismatch: kwd {tuple(kwd.shape)} utt {tuple(utt.shape)}")
        if utt.dtype != torch.bfloat16 or kwd.dtype != torch.bfloat16:
            raise ValueError("projected features must be bf16 (use KwsEngine.project)")
        utt, kwd = utt.contiguous(), kwd.contiguous()
        utt_mask = utt_mask.to(torch.float32).contiguous()
        kwd_mask = kwd_mask.to(torch.float32).contiguous()
        chunk = chunk or self.default_chunk(Tk, Tu)
        if logits_out is not None and (tuple(logits_out.shape) != (K, 2) or logits_out.dtype != torch.float32
                                       or not logits_out.is_contiguous()):
            raise ValueError(f"logits_out must be contiguous f32 [{K}, 2], got {tuple(logits_out.shape)}")
        logits = logits_out if logits_out is not None else torch.empty((K, 2), dtype=torch.float32, device=self.device)
        feats = torch.empty((K, L, Tk, Tu), dtype=torch.float32, device=self.device) if features else None
        with torch.cuda.device(self.device):
            ws = self.workspace(Tk, Tu, chunk)
            _lib.check(self.lib.cbw_kws_score(self.h, utt.data_ptr(), utt_mask.data_ptr(), kwd.data_ptr(),
                                              kwd_mask.data_ptr(), K, Tk, Tu, logits.data_ptr(), _lib.ptr(feats), chunk,
                                              ws.data_ptr(), ws.numel(), _lib.stream_handle()), "cbw_kws_score")
        return (logits, feats) if features else logits

    def classify(self, maps: torch.Tensor, chunk: Optional[int] = None) -> torch.Tensor:
        """Resnet.forward (resnet.py:51-58) on NCHW f32 maps [K, L, H, W] -> logits [K, 2]."""
        maps = maps.to(self.device, torch.float32).contiguous()
        K, L, Tk, Tu = maps.shape
        if L != self.n_layers:
            raise ValueError("Make sure that the channel dimension of the pixel values match with the one set in the "
                             "configuration.")
        chunk = chunk or self.default_chunk(Tk, Tu)
        logits = torch.empty((K, 2), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            ws = self.workspace(Tk, Tu, chunk)
            _lib.check(self.lib.cbw_kws_classify(self.h, maps.data_ptr(), K, Tk, Tu, logits.data_ptr(), chunk,
                                                 ws.data_ptr(), ws.numel(), _lib.stream_handle()), "cbw_kws_classify")
        return logits

    def score_resized(self, utt_hs: torch.Tensor, kwd_hs, out_size: Tuple[int, int] = (150, 750),
                      chunk: Optional[int] = None) -> torch.Tensor:
        """CB-Whisper's own spotter (model/cb_whisper.py:110-126, :189-210; model/model.py:78-93):
        utt_hs [L, Tu, D] and keyword hs (a list of [L, Tk_k, D], ragged) per-frame L2-normalised ->
        similarity matrices -> bilinear resize to ``out_size`` -> ResNet -> logits f32 [K, 2].
        ``kwd_hs`` may also be a packed ``(bf16 [L, R, D], int32 offsets [K + 1])`` pair
        (see ``pack_keywords``)."""
        if self.variant != VARIANT_L:
            raise ValueError("score_resized takes raw hs: build the engine with learn_features=False")
        rows, off = kwd_hs if isinstance(kwd_hs, tuple) else pack_keywords(kwd_hs, self.device)
        rows = rows.to(self.device, torch.bfloat16).contiguous()
        off_host = off.to("cpu", torch.int32).contiguous()
        off_dev = off_host.to(self.device)
        utt = utt_hs.to(self.device, torch.bfloat16).contiguous()
        L, Tu, D = utt.shape
        if L != self.n_layers or rows.shape[0] != L or rows.shape[2] != D:
            raise ValueError(f"shape mismatch: utt {tuple(utt.shape)} keyword rows {tuple(rows.shape)}")
        K = off_host.numel() - 1
        Ho, Wo = out_size
        chunk = chunk or self.default_chunk(Ho, Wo, budget_bytes=1 << 30)
        logits = torch.empty((K, 2), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            nb = self.lib.cbw_kws_score_resized_workspace_bytes(self.h, off_host.data_ptr(), K, Tu, D, Ho, Wo, chunk)
            if nb < 0:
                _lib.check(-1, "cbw_kws_score_resized_workspace_bytes")
            ws = self._ws.get(nb, self.device)
            _lib.check(self.lib.cbw_kws_score_resized(self.h, utt.data_ptr(), Tu, rows.data_ptr(), rows.shape[1], D,
                                                      off_dev.data_ptr(), off_host.data_ptr(), K, Ho, Wo,
                                                      logits.data_ptr(), chunk, ws.data_ptr(), ws.numel(),
                                                      _lib.stream_handle()), "cbw_kws_score_resized")
        return logits

    # ------------------------------------------------------------------ decision
    def spot(self, logits: torch.Tensor, ghost: Optional[torch.Tensor] = None, threshold: float = 0.5,
             mode: str = "threshold") -> Tuple[torch.Tensor, torch.Tensor]:
        """(prob f32 [K], sorted int64 indices) — model.py:782-813 (mode 'threshold') or
        cb_whisper.py:128 (mode 'argmax')."""
        return spot(logits, ghost, threshold, mode)


def pack_keywords(kwd_hs, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Ragged keyword hs (list of [L, Tk_k, D]) -> (bf16 [L, sum Tk, D] rows, int32 offsets [K + 1]):
    keyword k is rows off[k] .. off[k + 1] - 1 of every layer."""
    if len(kwd_hs) == 0:
        raise ValueError("no keywords")
    t = [torch.as_tensor(k) for k in kwd_hs]
    lens = torch.tensor([0] + [k.shape[1] for k in t], dtype=torch.int64)
    rows = torch.cat([k.to(device, torch.bfloat16) for k in t], dim=1)
    return rows, torch.cumsum(lens, 0).to(torch.int32)


def spot(logits: torch.Tensor, ghost: Optional[torch.Tensor] = None, threshold: float = 0.5,
         mode: str = "threshold") -> Tuple[torch.Tensor, torch.Tensor]:
    lib = _lib.load()
    logits = logits.to(torch.float32).contiguous()
    K = logits.shape[0]
    dev = logits.device
    prob = torch.empty((K,), dtype=torch.float32, device=dev)
    idx = torch.empty((max(K, 1),), dtype=torch.int32, device=dev)
    n = torch.zeros((1,), dtype=torch.int32, device=dev)
    g = None if ghost is None else ghost.to(dev, torch.float32).contiguous()
    if g is not None and g.numel() != K:
        raise ValueError(f"ghost mask of {g.numel()} entries for {K} logits")
    with torch.cuda.device(dev):
        _lib.check(lib.cbw_kws_spot(logits.data_ptr(), _lib.ptr(g), K, float(threshold), 1 if mode == "argmax" else 0,
                                    prob.data_ptr(), idx.data_ptr(), n.data_ptr(), _lib.stream_handle()),
                   "cbw_kws_spot")
    return prob, idx[: int(n.item())].to(torch.int64)
