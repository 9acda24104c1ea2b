"""model.model.KWSModel — MI355X drop-in for CB-Whisper's own keyword spotter
(src/model/model.py:18-93): a 12-channel ResNet-50 (``Resnet(num_channels=12, num_classes=2)``,
model.py:55-58) over similarity maps resized to (150, 750), decision argmax(logits) == 1
(cb_whisper.py:128).

Kept: the constructor's hyper-parameters (inert ones included), ``forward(input_features,
labels) -> KWSOutput``, ``load_state_dict`` / ``load_from_checkpoint`` with the reference
parameter names (``model.feature_extractor.*``, ``model.classifier.1.*``).  Added for the GPU
path: ``spot_keywords(utt_hs, kwd_hs)``, the whole of cb_whisper.py:110-128 for one segment
(similarity matrices + bilinear resize + CNN + argmax) in one libcbw call.

Deviations: ``KWSOutput.features`` (the pooled 2048-d ResNet features) is not materialised
(None); training (adversarial/DANNCE heads, optimizers) is out of scope.
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from cbw.kws import KwsEngine, spot
from cbw.synth import kws_param_shapes

from .utils import KWSOutput

_DEFAULTS = dict(
    large_heads=False, adversarial_training=False, dannce=False, adversarial_examples_ratio=0.5,
    adversarial_examples_lr=1.5e-6, adversarial_train_steps=5, adv_kl_weight=1.0, entropy=False,
    domain_adversary_weight=0.1, entropy_weight=0.1, supression_decay=1e-3, early_adversary_supression=True,
    num_domains=72, sampling="utterance-examples", resample_every_epoch=True, kw_type="tts", kw_p=0.5,
    batch_size=1, accumulate_grad_batches=1, learning_rate=1e-4, features_lr=1e-4, classifier_lr=1e-4,
    discriminator_lr=1e-4, lr_step=40, weight_decay=0.0, beta_1=0.9, beta_2=0.99,
)
NUM_CHANNELS = 12   # model.py:56


class KWSModel:
    def __init__(self, **kwargs):
        hp = dict(_DEFAULTS)
        hp.update(kwargs)
        self.hparams = SimpleNamespace(**hp)
        self._sd: Dict[str, torch.Tensor] = {}
        self._engine: Optional[KwsEngine] = None
        self.training = False

    def _engine_hp(self, embedding_dim: int = 1024) -> dict:
        return dict(n_layers=NUM_CHANNELS, embedding_dim=embedding_dim, learn_features=False, proj_mlp=False,
                    resnet_version="resnet-50")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return dict(self._sd)

    def load_state_dict(self, state_dict: Dict[str, object], strict: bool = True):
        expected = {n: s for n, s, _ in kws_param_shapes(NUM_CHANNELS, 1024, False, False, False)}
        sd = {k: (v.detach().cpu() if torch.is_tensor(v) else torch.as_tensor(np.asarray(v)))
              for k, v in state_dict.items() if not k.startswith(("discriminator.", "pr_curve.", "accuracy."))}
        if strict:
            missing = sorted(set(expected) - set(sd))
            unexpected = sorted(set(sd) - set(expected))
            if missing or unexpected:
                raise RuntimeError(f"Error(s) in loading state_dict for KWSModel: missing {missing[:5]}, "
                                   f"unexpected {unexpected[:5]}")
        for k, shape in expected.items():
            if k in sd and tuple(sd[k].shape) != tuple(shape):
                raise RuntimeError(f"size mismatch for {k}: checkpoint {tuple(sd[k].shape)} vs model {tuple(shape)}")
        self._sd = {k: v for k, v in sd.items() if k in expected}
        self._engine = None
        return SimpleNamespace(missing_keys=[], unexpected_keys=[])

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: str, map_location=None, **overrides) -> "KWSModel":
        """Lightning .ckpt (cb_whisper.py:60): {'state_dict', 'hyper_parameters'}, weights_only=True."""
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = dict(ckpt.get("hyper_parameters", {}))
        hp.update(overrides)
        model = cls(**hp)
        model.load_state_dict(ckpt["state_dict"], strict=True)
        return model

    def eval(self):
        self.training = False
        return self

    def to(self, *args, **kwargs):
        return self

    def engine(self, embedding_dim: int = 1024) -> KwsEngine:
        if self._engine is None or self._engine.D != embedding_dim:
            if not self._sd:
                raise RuntimeError("KWSModel has no parameters: call load_state_dict / load_from_checkpoint")
            self._engine = KwsEngine(self._engine_hp(embedding_dim), self._sd)
        return self._engine

    def forward(self, input_features: torch.Tensor, labels: torch.Tensor = None) -> KWSOutput:
        """model.py:78-93: input_features [K, 12, H, W] similarity maps -> logits [K, 2]."""
        eng = self.engine(self._engine.D if self._engine is not None else 1024)
        logits = eng.classify(input_features)
        loss = None
        if labels is not None:
            loss = torch.nn.functional.cross_entropy(logits, labels.to(logits.device).view(-1))
        return KWSOutput(loss=loss, logits=logits, features=None)

    __call__ = forward

    def score_keywords(self, utt_hs: torch.Tensor, kwd_hs, kws_features_size=(150, 750)) -> torch.Tensor:
        """cb_whisper.py:110-126 for one segment: utt_hs [12, Tu, D], kwd_hs a list of [12, Tk_k, D]
        (L2-normalised) or its packed form (cbw.kws.pack_keywords) -> logits [K, 2] (sims, resize, CNN
        fused on the GPU)."""
        kh = kwd_hs if isinstance(kwd_hs, tuple) else list(kwd_hs)
        return self.engine(int(utt_hs.shape[-1])).score_resized(utt_hs, kh, tuple(kws_features_size))

    def spot_keywords(self, utt_hs: torch.Tensor, kwd_hs, kws_features_size=(150, 750)) -> List[int]:
        """cb_whisper.py:128: indices with argmax(logits) == 1."""
        logits = self.score_keywords(utt_hs, kwd_hs, kws_features_size)
        _, idx = spot(logits, None, 0.5, mode="argmax")
        return idx.tolist()
