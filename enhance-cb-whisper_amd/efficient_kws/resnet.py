"""Resnet — drop-in for src/efficient_kws/resnet.py:7-58.

Same constructor (num_channels, num_classes, version) and forward contract
(NCHW similarity maps [K, C, H, W] -> logits [K, num_classes]); the network
runs in libcbw (bf16 MFMA implicit-GEMM convs, BN folded), not in HF
``ResNetModel``.  Parameters use the reference state-dict names relative to the
owning module (``feature_extractor.*``, ``classifier.1.*``).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from cbw.kws import KwsEngine
from cbw.synth import RESNET_VERSIONS


class Resnet:
    def __init__(self, num_channels: int, num_classes: Optional[int] = None, version: str = "resnet-50"):
        if version not in RESNET_VERSIONS:
            raise ValueError(f"unsupported resnet version {version}")
        if num_classes not in (None, 2):
            raise ValueError("the MI355X classifier head is Linear(hidden, 2) (efficient_kws/model.py:73-85)")
        self.num_channels = num_channels
        self.num_classes = num_classes
        self.version = version
        self.hidden = RESNET_VERSIONS[version][1][-1]
        self._sd: Dict[str, torch.Tensor] = {}
        self._engine: Optional[KwsEngine] = None

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        self._sd = {k: (v if torch.is_tensor(v) else torch.as_tensor(v)) for k, v in sd.items()}
        self._engine = None

    def state_dict(self):
        return dict(self._sd)

    def _get_engine(self) -> KwsEngine:
        if self._engine is None:
            # classifier-only handle (no projector): the ResNet's own parameters under the KWSModel prefix
            hp = dict(n_layers=self.num_channels, embedding_dim=128, resnet_version=self.version)
            sd = {f"model.{k}": v for k, v in self._sd.items()}
            self._engine = KwsEngine(hp, sd, classifier_only=True)
        return self._engine

    def forward(self, input_features: torch.Tensor) -> torch.Tensor:
        return self._get_engine().classify(input_features)

    __call__ = forward
