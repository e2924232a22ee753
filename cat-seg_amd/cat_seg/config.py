"""Config surface of the reference (`add_cat_seg_config`, cat_seg/config.py:6-93, plus the
detectron2 defaults the eval path reads).

When detectron2 is installed its `CfgNode` / `get_cfg` are used unchanged, so the
reference's `train_net.py` / `eval.sh` overrides work as-is.  Without detectron2 a
small yacs-compatible `CfgNode` (attribute access, `merge_from_file` with `_BASE_`,
`merge_from_list`, `freeze`) stands in, so configs/*.yaml load identically.
"""
from __future__ import annotations

import ast
import copy
import os

import yaml

try:  # pragma: no cover - detectron2 is not in this image
    from detectron2.config import CfgNode as _D2CfgNode, get_cfg as _d2_get_cfg
    HAVE_D2 = True
except Exception:  # noqa: BLE001
    _D2CfgNode, _d2_get_cfg = None, None
    HAVE_D2 = False


def _decode(v):
    """yacs `_decode_cfg_value`: strings that are Python literals ("(384, 384)", "[1,1]", "True")
    become those values; anything else stays as given."""
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    return v


class CfgNode(dict):
    """Minimal yacs.CfgNode: nested dict with attribute access."""

    def __init__(self, init=None):
        super().__init__()
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v
        object.__setattr__(self, "_frozen", False)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        if self._frozen:
            raise AttributeError("config is frozen")
        self[k] = v

    def freeze(self):
        object.__setattr__(self, "_frozen", True)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.freeze()

    def defrost(self):
        object.__setattr__(self, "_frozen", False)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.defrost()

    def clone(self):
        return copy.deepcopy(self)

    def _merge(self, other: dict):
        for k, v in other.items():
            if isinstance(v, dict):
                node = self.get(k)
                if not isinstance(node, CfgNode):
                    node = CfgNode()
                    self[k] = node
                node._merge(v)
            else:
                v = _decode(v)
                self[k] = tuple(v) if isinstance(self.get(k), tuple) and isinstance(v, list) else v

    def merge_from_file(self, path: str):
        with open(path) as f:
            d = yaml.safe_load(f) or {}
        base = d.pop("_BASE_", None)
        if base is not None:
            self.merge_from_file(base if os.path.isabs(base) else os.path.join(os.path.dirname(path), base))
        self._merge(d)

    def merge_from_list(self, opts):
        assert len(opts) % 2 == 0, "KEY VALUE pairs expected"
        for k, v in zip(opts[0::2], opts[1::2]):
            node = self
            parts = k.split(".")
            for p in parts[:-1]:
                node = node[p]
            node[parts[-1]] = _decode(v)


def get_cfg():
    """detectron2's get_cfg (subset read by the CAT-Seg eval path when detectron2 is absent)."""
    if HAVE_D2:  # pragma: no cover
        return _d2_get_cfg()
    return CfgNode({
        "MODEL": {"META_ARCHITECTURE": "CATSeg", "DEVICE": "cuda", "WEIGHTS": "",
                  "PIXEL_MEAN": [103.530, 116.280, 123.675], "PIXEL_STD": [1.0, 1.0, 1.0],
                  "SEM_SEG_HEAD": {"NAME": "CATSegHead", "IGNORE_VALUE": 255, "NUM_CLASSES": 54,
                                   "IN_FEATURES": ["res2", "res3", "res4", "res5"]}},
        # detectron2 v0.6 defaults (config/defaults.py) of the keys the data / eval path reads;
        # MIN/MAX_SIZE_TEST are the CAT-Seg configs' values (configs/config.yaml:52-53)
        "INPUT": {"MIN_SIZE_TRAIN": (800,), "MIN_SIZE_TRAIN_SAMPLING": "choice", "MAX_SIZE_TRAIN": 1333,
                  "MIN_SIZE_TEST": 640, "MAX_SIZE_TEST": 2560, "FORMAT": "RGB",
                  "CROP": {"ENABLED": False, "TYPE": "relative_range", "SIZE": [0.9, 0.9]}},
        "DATASETS": {"TRAIN": (), "TEST": ()},
        "SOLVER": {"IMS_PER_BATCH": 16, "BASE_LR": 0.001, "WEIGHT_DECAY": 0.0001, "WEIGHT_DECAY_NORM": 0.0,
                   "MOMENTUM": 0.9, "MAX_ITER": 40000,
                   "CLIP_GRADIENTS": {"ENABLED": False, "CLIP_TYPE": "value", "CLIP_VALUE": 1.0, "NORM_TYPE": 2.0}},
        "TEST": {"EVAL_PERIOD": 0, "EXPECTED_RESULTS": [],
                 "AUG": {"ENABLED": False, "MIN_SIZES": (400, 500, 600, 700, 800, 900, 1000, 1100, 1200),
                         "MAX_SIZE": 4000, "FLIP": True}},
        "DATALOADER": {"NUM_WORKERS": 4},
        "OUTPUT_DIR": "./output",
        "VERSION": 2,
    })


def add_cat_seg_config(cfg):
    """Same keys and defaults as the reference add_cat_seg_config (cat_seg/config.py:6-93)."""
    C = type(cfg)
    cfg.INPUT.DATASET_MAPPER_NAME = "mask_former_semantic"
    cfg.DATASETS.VAL_ALL = ("coco_2017_val_all_stuff_sem_seg",)
    cfg.INPUT.COLOR_AUG_SSD = False
    cfg.INPUT.CROP.SINGLE_CATEGORY_MAX_AREA = 1.0
    cfg.INPUT.SIZE_DIVISIBILITY = -1
    cfg.SOLVER.WEIGHT_DECAY_EMBED = 0.0
    cfg.SOLVER.OPTIMIZER = "ADAMW"
    cfg.SOLVER.BACKBONE_MULTIPLIER = 0.1
    cfg.MODEL.MASK_FORMER = C()
    cfg.MODEL.MASK_FORMER.SIZE_DIVISIBILITY = 32
    cfg.MODEL.SWIN = C()
    cfg.MODEL.SWIN.PRETRAIN_IMG_SIZE = 224
    cfg.MODEL.SWIN.PATCH_SIZE = 4
    cfg.MODEL.SWIN.EMBED_DIM = 96
    cfg.MODEL.SWIN.DEPTHS = [2, 2, 6, 2]
    cfg.MODEL.SWIN.NUM_HEADS = [3, 6, 12, 24]
    cfg.MODEL.SWIN.WINDOW_SIZE = 7
    cfg.MODEL.SWIN.MLP_RATIO = 4.0
    cfg.MODEL.SWIN.QKV_BIAS = True
    cfg.MODEL.SWIN.QK_SCALE = None
    cfg.MODEL.SWIN.DROP_RATE = 0.0
    cfg.MODEL.SWIN.ATTN_DROP_RATE = 0.0
    cfg.MODEL.SWIN.DROP_PATH_RATE = 0.3
    cfg.MODEL.SWIN.APE = False
    cfg.MODEL.SWIN.PATCH_NORM = True
    cfg.MODEL.SWIN.OUT_FEATURES = ["res2", "res3", "res4", "res5"]
    h = cfg.MODEL.SEM_SEG_HEAD
    h.TRAIN_CLASS_JSON = "datasets/ADE20K_2021_17_01/ADE20K_847.json"
    h.TEST_CLASS_JSON = "datasets/ADE20K_2021_17_01/ADE20K_847.json"
    h.TRAIN_CLASS_INDEXES = "datasets/coco/coco_stuff/split/seen_indexes.json"
    h.TEST_CLASS_INDEXES = "datasets/coco/coco_stuff/split/unseen_indexes.json"
    h.CLIP_PRETRAINED = "ViT-B/16"
    cfg.MODEL.PROMPT_ENSEMBLE = False
    cfg.MODEL.PROMPT_ENSEMBLE_TYPE = "single"
    cfg.MODEL.CLIP_PIXEL_MEAN = [122.7709383, 116.7460125, 104.09373615]
    cfg.MODEL.CLIP_PIXEL_STD = [68.5005327, 66.6321579, 70.3231630]
    h.TEXT_GUIDANCE_DIM = 512
    h.TEXT_GUIDANCE_PROJ_DIM = 128
    h.APPEARANCE_GUIDANCE_DIM = 512
    h.APPEARANCE_GUIDANCE_PROJ_DIM = 128
    h.DECODER_DIMS = [64, 32]
    h.DECODER_GUIDANCE_DIMS = [256, 128]
    h.DECODER_GUIDANCE_PROJ_DIMS = [32, 16]
    h.NUM_LAYERS = 4
    h.NUM_HEADS = 4
    h.HIDDEN_DIMS = 128
    h.POOLING_SIZES = [6, 6]
    h.FEATURE_RESOLUTION = [24, 24]
    h.WINDOW_SIZES = 12
    h.ATTENTION_TYPE = "linear"
    h.PROMPT_DEPTH = 0
    h.PROMPT_LENGTH = 0
    cfg.SOLVER.CLIP_MULTIPLIER = 0.01
    h.CLIP_FINETUNE = "attention"
    cfg.TEST.SLIDING_WINDOW = False
    # MI355X build extensions (absent from the reference; defaults keep reference behaviour)
    cfg.MODEL.CATSEG_HIP = C()
    cfg.MODEL.CATSEG_HIP.DTYPE = "bf16"          # "bf16" | "f32"
    cfg.MODEL.CATSEG_HIP.RETURN_ALL_IMAGES = True  # reference returns batched_inputs[0] only
    cfg.MODEL.CATSEG_HIP.BPE_VOCAB = ""          # path to CLIP's bpe_simple_vocab_16e6.txt.gz
    cfg.MODEL.CATSEG_HIP.SYNTHETIC_SEED = 0      # weights when MODEL.WEIGHTS is empty
    cfg.MODEL.CATSEG_HIP.VIT_FP8 = False         # config 5: e4m3 CLIP image-encoder GEMMs (bf16 engine)
    cfg.MODEL.CATSEG_HIP.GRAPH = True            # eval forward replayed from a hipGraph per input geometry
    return cfg
