"""Multi-GPU partitioning of the keyword-spotting path, one process per GPU.

* Clip-parallel (BASELINE C5; bench.py default): every rank scores its own clips
  against the full keyword database — no data-path collective.
* Keyword-sharded (BASELINE C4, 100k keywords over 8 GPUs): rank r owns keywords
  ``shard_range(K, r, world)``; the front end of clip i (mel + encoder + utterance projection)
  runs on rank ``front_owner(i, world)`` = i mod world -- round robin, so no rank carries every
  clip's encoder beside its scoring -- which RCCL-broadcasts the projected utterance (LEF: 3x750x64 bf16 = 288 KB + mask); every
  rank scores its shard; one all-gather of the [K/world, 2] logits (padded to equal
  shards) gives every rank the full logits; the decision runs once.  Payloads are far
  below a megabyte, so single-step collectives over xGMI are latency-bound (tens of
  µs); the similarity maps (33.7 GB at 100k) never leave their GPU.

``torch.distributed`` with backend "nccl" is RCCL on ROCm; tests drive the same code
with "gloo" on CPU through an injectable ``score_fn``.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(K: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced keyword shard [lo, hi) of rank (sizes differ by at most 1)."""
    base, rem = divmod(K, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def front_owner(clip: int, world: int) -> int:
    """The rank that runs clip ``clip``'s front end and broadcasts its projected utterance (round robin)."""
    return clip % world


def max_shard(K: int, world: int) -> int:
    return (K + world - 1) // world


class KeywordShardedSpotter:
    def __init__(self, K_total: int, kwd_local: torch.Tensor, kwd_mask_local: torch.Tensor,
                 score_fn: Callable[..., torch.Tensor], group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.K = K_total
        self.lo, self.hi = shard_range(K_total, self.rank, self.world)
        if kwd_local.shape[0] != self.hi - self.lo:
            raise ValueError(f"rank {self.rank} holds {kwd_local.shape[0]} keywords, shard is {self.hi - self.lo}")
        self.kwd, self.kwd_mask = kwd_local, kwd_mask_local
        self.score_fn = score_fn
        self.pad = max_shard(K_total, self.world)

    def broadcast_utterance(self, utt: Optional[torch.Tensor], utt_mask: Optional[torch.Tensor], shape, mask_shape,
                            dtype, device, src: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        """Rank ``src``'s projected utterance (+ mask) to every rank (one broadcast each; the other ranks pass
        None)."""
        if self.rank != src:
            utt = torch.empty(shape, dtype=dtype, device=device)
            utt_mask = torch.empty(mask_shape, dtype=torch.float32, device=device)
        u = utt.contiguous()
        if u.dtype == torch.bfloat16 and device.type == "cpu":   # gloo has no bf16/int16: ship the bytes
            bits = u.view(torch.uint8)
            dist.broadcast(bits, src=src, group=self.group)
            u = bits.view(torch.bfloat16)
        else:
            dist.broadcast(u, src=src, group=self.group)
        m = utt_mask.contiguous()
        dist.broadcast(m, src=src, group=self.group)
        return u, m

    def broadcast_tensor(self, t: Optional[torch.Tensor], shape, dtype, device, src: int = 0) -> torch.Tensor:
        """Rank ``src``'s tensor (e.g. the fp32 utterance projection of the exact re-scoring band) to every rank."""
        if self.rank != src:
            t = torch.empty(shape, dtype=dtype, device=device)
        t = t.contiguous()
        dist.broadcast(t, src=src, group=self.group)
        return t

    def score(self, utt: torch.Tensor, utt_mask: torch.Tensor) -> torch.Tensor:
        """Local shard logits -> all-gathered full logits [K, 2] on every rank."""
        return self.gather(self.score_fn(utt, utt_mask, self.kwd, self.kwd_mask))

    def gather(self, local: torch.Tensor) -> torch.Tensor:
        """This rank's shard logits [hi - lo, 2] -> the full logits [K, 2] on every rank (one all-gather of the
        padded shards, issued on the caller's current stream)."""
        if local.shape[0] != self.hi - self.lo:
            raise ValueError(f"rank {self.rank}: {local.shape[0]} shard logits, shard is {self.hi - self.lo}")
        buf = torch.zeros((self.pad, 2), dtype=torch.float32, device=local.device)
        buf[: local.shape[0]] = local
        out = torch.empty((self.world * self.pad, 2), dtype=torch.float32, device=local.device)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        parts = []
        for r in range(self.world):
            lo, hi = shard_range(self.K, r, self.world)
            parts.append(out[r * self.pad: r * self.pad + (hi - lo)])
        return torch.cat(parts, 0)
