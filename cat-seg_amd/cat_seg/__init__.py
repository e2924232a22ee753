"""cat_seg — MI355X-native CAT-Seg dense inference, a drop-in for the reference package's
eval hot path.

Mirrors the reference's `cat_seg/__init__.py:1-20` surface: importing the package registers
the evaluation datasets (`data`, reference cat_seg/data/datasets/register_*.py), `CATSeg`
(META_ARCH) and `CATSegHead` (SEM_SEG_HEADS), and exports every name `train_net.py:74-80`
imports (`DETRPanopticDatasetMapper`, `MaskFormerPanopticDatasetMapper`,
`MaskFormerSemanticDatasetMapper`, `SemanticSegmentorWithTTA`, `add_cat_seg_config`).
The 43 ImplicitFusion research variants of the fork are not part of this path.
The compute runs in libcatseg_hip.so (include/catseg_hip.h); see DESIGN.md.
"""
from . import data  # noqa: F401  (register all new datasets)
from .config import add_cat_seg_config, get_cfg, CfgNode  # noqa: F401
from .data.dataset_mappers import (  # noqa: F401
    CATSegTestDatasetMapper, DETRPanopticDatasetMapper, MaskFormerPanopticDatasetMapper,
    MaskFormerSemanticDatasetMapper)
from .registry import META_ARCH_REGISTRY, SEM_SEG_HEADS_REGISTRY, build_model  # noqa: F401
from .cat_seg_model import CATSeg  # noqa: F401
from .test_time_augmentation import SemanticSegmentorWithTTA  # noqa: F401
from .modeling.heads.cat_seg_head import CATSegHead  # noqa: F401
from .modeling.transformer.cat_seg_predictor import CATSegPredictor  # noqa: F401
from .arch import CatSegArch, VIT_B16, VIT_L14_336, TINY  # noqa: F401
from .evaluation import SemSegEvaluator, SemSegGzeroEvaluator, VOCbEvaluator  # noqa: F401
from .inference import DatasetEvaluators, inference_on_dataset  # noqa: F401
from .data.build import build_test_loader  # noqa: F401

__all__ = ["add_cat_seg_config", "get_cfg", "build_model", "CATSeg", "CATSegHead", "CATSegPredictor",
           "CatSegArch", "META_ARCH_REGISTRY", "SEM_SEG_HEADS_REGISTRY",
           "DETRPanopticDatasetMapper", "MaskFormerPanopticDatasetMapper", "MaskFormerSemanticDatasetMapper",
           "CATSegTestDatasetMapper", "SemanticSegmentorWithTTA",
           "SemSegEvaluator", "SemSegGzeroEvaluator", "VOCbEvaluator", "DatasetEvaluators",
           "inference_on_dataset", "build_test_loader"]
