"""Token-level timestamps: transformers WhisperGenerationMixin._extract_token_timestamps, which the reference reaches
with ``return_token_timestamps`` (pba_whisper.py:333-336 in short-form; :439 -> generate_with_fallback ->
_postprocess_outputs in long-form).  The cross-attention weights of the checkpoint's alignment heads along a decoded
row are normalised over the decoder positions (mean / population std per head and frame), median-filtered along the
frames (odd width, reflect padding, sort-based median), averaged over the heads; dynamic time warping of the negated
matrix gives a monotone path, and each text position's first frame on the path, times ``time_precision``, is its time.

The weights come from libcbw (cbw_decoder_cross_attn_probs: a teacher-forced decoder pass over the row, one query row
per position -- what generate's per-step cross_attentions hold for the row that was kept, the beam's history being the
row's prefix); the DTW runs on the host in libcbw (cbw_dtw, the transformers loop step for step).

``variant``:
  * "4.37" (the pinned transformers, requirements.txt:21): every decoder position is a DTW row; timestamps has the
    row's length, timestamps[0] = 0 and timestamps[1:] = the jump times.  Restated from the 4.37.2 text -- PARITY
    UNPINNED for this row handling (4.37.2 cannot run here); the shared core below is pinned.
  * "5.x" (the installed 5.15): the first ``num_input_ids`` positions are left out of the DTW and get 0, the last
    position repeats the last jump time -- pinned to transformers 5.15's function on the same weights
    (tests/test_host.py::test_token_timestamps_match_transformers)."""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


def median_filter(x: torch.Tensor, width: int) -> torch.Tensor:
    """transformers' _median_filter along the last dimension of a 3-D / 4-D tensor."""
    if width <= 0 or width % 2 != 1:
        raise ValueError("`filter_width` should be an odd number")
    pad = width // 2
    if x.shape[-1] <= pad:
        return x
    squeeze = x.dim() == 3
    y = torch.nn.functional.pad(x[None] if squeeze else x, (pad, pad, 0, 0), mode="reflect")
    y = y.unfold(-1, width, 1).sort()[0][..., pad]
    return y[0] if squeeze else y


def dtw(matrix: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """transformers' _dynamic_time_warping on a [rows, cols] cost matrix (libcbw cbw_dtw, host code) ->
    (text_indices, time_indices) along the path."""
    m = np.ascontiguousarray(matrix, dtype=np.float64)
    rows, cols = m.shape
    ti = np.empty(rows + cols, dtype=np.int32)
    tj = np.empty(rows + cols, dtype=np.int32)
    n = np.zeros(1, dtype=np.int32)
    lib = _lib.load()
    _lib.check(lib.cbw_dtw(m.ctypes.data, rows, cols, ti.ctypes.data, tj.ctypes.data, n.ctypes.data), "cbw_dtw")
    return ti[:n[0]].astype(np.int64), tj[:n[0]].astype(np.int64)


def _normalised_mean(w: torch.Tensor, median_filter_width: int) -> torch.Tensor:
    std = torch.std(w, dim=-2, keepdim=True, unbiased=False)
    mean = torch.mean(w, dim=-2, keepdim=True)
    return median_filter((w - mean) / std, median_filter_width).mean(dim=0)


def extract_token_timestamps(weights: torch.Tensor, median_filter_width: int = 7, time_precision: float = 0.02,
                             num_frames: Optional[int] = None, variant: str = "4.37",
                             num_input_ids: Optional[int] = None) -> torch.Tensor:
    """weights [heads, positions, frames]: the alignment heads' cross-attention weights of one decoded row (one query
    row per position; the row's last token has none) -> float32 [positions + 1], the row's token timestamps."""
    if variant not in ("4.37", "5.x"):
        raise ValueError(f"unknown variant {variant}")
    w = weights.float()
    T = w.shape[1]
    ts = torch.zeros(T + 1, dtype=torch.float32)
    if num_frames is not None:
        w = w[..., : int(num_frames) // 2]
    if variant == "5.x" and num_input_ids is not None:
        w = w[:, num_input_ids:]
        if w.shape[1] == 0:
            return ts
    matrix = _normalised_mean(w, median_filter_width)
    text_idx, time_idx = dtw(-matrix.cpu().double().numpy())
    jumps = np.pad(np.diff(text_idx), (1, 0), constant_values=1).astype(bool)
    jump_times = time_idx[jumps] * time_precision
    if variant == "4.37":
        ts[1:] = torch.tensor(jump_times)
        return ts
    n0 = num_input_ids or 0
    return torch.cat([torch.zeros(n0), torch.tensor(jump_times), torch.tensor([jump_times[-1]])]).float()


def alignment_pairs(alignment_heads: Sequence[Sequence[int]]) -> np.ndarray:
    """[[layer, head], ...] -> host int32 [2 n] (cbw_decoder_cross_attn_probs' heads)."""
    a = np.asarray([[int(l), int(h)] for l, h in alignment_heads], dtype=np.int32).reshape(-1)
    if a.size == 0:
        raise ValueError("alignment_heads is empty")
    return np.ascontiguousarray(a)
