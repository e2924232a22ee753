"""cat_seg — MI355X-native CAT-Seg dense inference, a drop-in for the reference package's
eval hot path (reference cat_seg/__init__.py exports add_cat_seg_config and registers
CATSeg / CATSegHead into detectron2's registries).

Importing the package registers `CATSeg` (META_ARCH) and `CATSegHead` (SEM_SEG_HEADS).
The compute runs in libcatseg_hip.so (include/catseg_hip.h); see DESIGN.md.
"""
from .config import add_cat_seg_config, get_cfg, CfgNode  # noqa: F401
from .registry import META_ARCH_REGISTRY, SEM_SEG_HEADS_REGISTRY, build_model  # noqa: F401
from .cat_seg_model import CATSeg  # noqa: F401
from .modeling.heads.cat_seg_head import CATSegHead  # noqa: F401
from .modeling.transformer.cat_seg_predictor import CATSegPredictor  # noqa: F401
from .arch import CatSegArch, VIT_B16, VIT_L14_336, TINY  # noqa: F401
from .evaluation import SemSegEvaluator, SemSegGzeroEvaluator, VOCbEvaluator  # noqa: F401

__all__ = ["add_cat_seg_config", "get_cfg", "build_model", "CATSeg", "CATSegHead", "CATSegPredictor",
           "CatSegArch", "META_ARCH_REGISTRY", "SEM_SEG_HEADS_REGISTRY",
           "SemSegEvaluator", "SemSegGzeroEvaluator", "VOCbEvaluator"]
