"""ctypes binding of libcbw.so (include/cbw.h).

The library is the product: there is no CPU or PyTorch fallback.  If
``libcbw.so`` is missing or no GPU is visible, the compute entry points raise.
Device buffers are torch tensors (the caching allocator owns memory); we pass
their data pointers and torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first so libcbw binds to the same libamdhip64)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CBW_LIB", os.path.join(_HERE, "libcbw.so"))

c_int, c_int64, c_float, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_char_p


class KwsConfig(ctypes.Structure):
    _fields_ = [("n_layers", c_int), ("embedding_dim", c_int), ("variant", c_int), ("proj_units", c_int),
                ("resnet_depth", c_int)]


class EncoderConfig(ctypes.Structure):
    _fields_ = [("n_mel", c_int), ("d_model", c_int), ("n_layers", c_int), ("n_heads", c_int), ("ffn_dim", c_int)]


class DecoderConfig(ctypes.Structure):
    _fields_ = [("vocab", c_int), ("d_model", c_int), ("n_layers", c_int), ("n_heads", c_int), ("ffn_dim", c_int),
                ("max_len", c_int)]


# name: (restype, argtypes) — mirrors include/cbw.h exactly (tests check every symbol is exported)
SIGNATURES = {
    "cbw_version": (c_int, []),
    "cbw_last_error": (c_char_p, []),
    "cbw_source_id": (c_char_p, []),
    "cbw_kws_create": (c_int, [ctypes.POINTER(KwsConfig), ctypes.POINTER(c_void_p)]),
    "cbw_kws_destroy": (c_int, [c_void_p]),
    "cbw_kws_set_param": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
    "cbw_kws_finalize": (c_int, [c_void_p]),
    "cbw_kws_project_workspace_bytes": (c_int64, [c_void_p, c_int, c_int]),
    "cbw_kws_project": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64,
                                c_void_p]),
    "cbw_kws_project_f32_workspace_bytes": (c_int64, [c_void_p, c_int, c_int]),
    "cbw_kws_project_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64,
                                    c_void_p]),
    "cbw_kws_rescore_workspace_bytes": (c_int64, [c_void_p, c_int, c_int]),
    "cbw_kws_rescore": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                c_void_p, c_void_p, c_int64, c_void_p]),
    "cbw_kws_calibrate_bias": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                       c_int, c_void_p, c_int64, c_void_p]),
    "cbw_kws_rescore_x3_workspace_bytes": (c_int64, [c_void_p, c_int, c_int]),
    "cbw_kws_rescore_x3": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                   c_int, c_void_p, c_void_p, c_int64, c_void_p]),
    "cbw_kws_workspace_bytes": (c_int64, [c_void_p, c_int, c_int, c_int]),
    "cbw_kws_score": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_int, c_void_p, c_int64, c_void_p]),
    "cbw_kws_classify": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int64,
                                 c_void_p]),
    "cbw_kws_spot": (c_int, [c_void_p, c_void_p, c_int, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cbw_checksum_workspace_bytes": (ctypes.c_int64, []),
    "cbw_checksum": (c_int, [c_void_p, ctypes.c_int64, c_void_p, c_void_p, ctypes.c_int64, c_void_p]),
    "cbw_kws_band": (c_int, [c_void_p, c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "cbw_beam_select": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "cbw_kws_set_score_offset": (c_int, [c_void_p, c_void_p]),
    "cbw_kws_band_scaled": (c_int, [c_void_p, c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "cbw_kws_score_resized_workspace_bytes": (c_int64, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int]),
    "cbw_kws_score_resized": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                                      c_int, c_int, c_void_p, c_int, c_void_p, c_int64, c_void_p]),
    "cbw_mel": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "cbw_mel_long": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "cbw_encoder_create": (c_int, [ctypes.POINTER(EncoderConfig), ctypes.POINTER(c_void_p)]),
    "cbw_encoder_destroy": (c_int, [c_void_p]),
    "cbw_encoder_set_param": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
    "cbw_encoder_finalize": (c_int, [c_void_p]),
    "cbw_encoder_workspace_bytes": (c_int64, [c_void_p, c_int]),
    "cbw_encoder_hs": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64,
                               c_void_p]),
    "cbw_conv2d": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 12 + [c_void_p]),
    "cbw_conv1x1_dual": (c_int, [c_void_p] * 6 + [c_int] * 10 + [c_void_p]),
    "cbw_gemm_splitk_factor": (c_int, [c_int, c_int, c_int]),
    "cbw_gemm": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p, c_int64, c_void_p]),
    "cbw_encoder_attention": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "cbw_kws_profile": (c_int, [c_void_p, c_int]),
    "cbw_decoder_create": (c_int, [ctypes.POINTER(DecoderConfig), ctypes.POINTER(c_void_p)]),
    "cbw_decoder_destroy": (c_int, [c_void_p]),
    "cbw_decoder_set_param": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
    "cbw_decoder_finalize": (c_int, [c_void_p]),
    "cbw_decoder_vocab_padded": (c_int, [c_void_p]),
    "cbw_decoder_state_bytes": (c_int64, [c_void_p, c_int, c_int]),
    "cbw_decoder_cross_kv": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cbw_decoder_step": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "cbw_decoder_step_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "cbw_decoder_prefill": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "cbw_decoder_cross_kv_slot": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cbw_decoder_prefill_rows": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int64,
                                         c_void_p, c_void_p]),
    "cbw_decoder_step_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "cbw_decoder_reorder": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p]),
    "cbw_decoder_cross_attn_probs": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                                             c_int64, c_void_p, c_void_p]),
    "cbw_dtw": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "cbw_logprob_topk": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "cbw_timestamp_rules": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                    c_void_p, c_void_p]),
    "cbw_kws_profile_read": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int)]),
    "cbw_kws_profile_records": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "cbw_kws_profile_tiers": (c_int, [c_void_p, c_void_p, c_int]),
    "cbw_kws_profile_kernels": (c_int, [c_void_p, c_void_p, c_int]),
    "cbw_kws_calibrate_fp8": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                      c_int, c_float, c_void_p, c_int64, c_void_p]),
    "cbw_kws_score_fp8": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                  c_int, c_void_p, c_int64, c_void_p]),
    "cbw_kws_set_score_offset_fp8": (c_int, [c_void_p, c_void_p]),
    "cbw_kws_fp8_scales": (c_int, [c_void_p, c_void_p, c_int]),
    "cbw_conv2d_fp8": (c_int, [c_void_p] * 5 + [c_float, c_void_p, c_float] + [c_int] * 9 + [c_void_p]),
    "cbw_fp8_probe": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
}

ERRORS = {-1: "CBW_ERR_INVALID", -2: "CBW_ERR_HIP", -3: "CBW_ERR_OOM", -4: "CBW_ERR_STATE", -5: "CBW_ERR_NOT_FOUND"}

_lib = None


class CbwError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libcbw.so (raises if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CbwError(f"libcbw.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().cbw_last_error()
        msg = msg.decode() if msg else ""
        err = ValueError if rc == -1 else CbwError
        raise err(f"{what} failed with {ERRORS.get(rc, rc)}: {msg}")


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise CbwError("no ROCm GPU visible: the CB-Whisper hot path runs only on MI355X (gfx950); there is no CPU fallback")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class Workspace:
    """Grow-only device scratch owned by the torch caching allocator."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        nbytes = max(int(nbytes), 256)
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != torch.device(device):
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf
