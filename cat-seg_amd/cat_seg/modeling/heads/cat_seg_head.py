"""CATSegHead (reference cat_seg/modeling/heads/cat_seg_head.py:1965-2010): drops the CLS
token, reshapes tokens to B C H W and calls the predictor."""
from __future__ import annotations

from torch import nn

from ...registry import SEM_SEG_HEADS_REGISTRY, configurable
from ..transformer.cat_seg_predictor import CATSegPredictor


@SEM_SEG_HEADS_REGISTRY.register()
class CATSegHead(nn.Module):
    @configurable
    def __init__(self, *, num_classes: int, ignore_value: int = -1, feature_resolution: list,
                 transformer_predictor: nn.Module):
        super().__init__()
        self.ignore_value = ignore_value
        self.predictor = transformer_predictor
        self.num_classes = num_classes
        self.feature_resolution = feature_resolution

    @classmethod
    def from_config(cls, cfg, input_shape=None):
        return {
            "ignore_value": cfg.MODEL.SEM_SEG_HEAD.IGNORE_VALUE,
            "num_classes": cfg.MODEL.SEM_SEG_HEAD.NUM_CLASSES,
            "feature_resolution": cfg.MODEL.SEM_SEG_HEAD.FEATURE_RESOLUTION,
            "transformer_predictor": CATSegPredictor(cfg),
        }

    def forward(self, features, guidance_features, prompt=None, gt_cls=None):
        """features: (B, 1+HW, C) CLIP dense tokens; guidance {res5, res4, res3} NCHW."""
        h, w = self.feature_resolution
        B, _, C = features.shape
        img = features[:, 1:, :].reshape(B, h, w, C).permute(0, 3, 1, 2)
        return self.predictor(img, guidance_features, prompt, gt_cls)
