"""Dataset mappers: dataset dict -> model input dict (host side, numpy / PIL).

* `CATSegTestDatasetMapper` — what detectron2's `build_detection_test_loader` applies for
  CAT-Seg evaluation (`DatasetMapper(cfg, is_train=False)`): read the RGB image, record the
  original "height"/"width" (`check_image_size`), ResizeShortestEdge(INPUT.MIN_SIZE_TEST,
  INPUT.MAX_SIZE_TEST) (640 / 2560, vizDebug/log.txt:1876), "image" = CHW uint8 tensor.
  Ground truth is read by the evaluator from "file_name" (SemSegEvaluator's
  input_file_to_gt_file), not here.
* `MaskFormerSemanticDatasetMapper` — the reference's training mapper
  (cat_seg/data/dataset_mappers/mask_former_semantic_dataset_mapper.py:19-170): resize,
  category-area crop, SSD colour aug, flip, pad to INPUT.SIZE_DIVISIBILITY (image 128, label
  ignore), per-class binary masks.  Imported by train_net.py:74-80; the training step itself
  is outside this build's inference path.
* `DETRPanopticDatasetMapper`, `MaskFormerPanopticDatasetMapper` — panoptic mappers of the
  MaskFormer lineage that train_net.py:74-80 imports but CAT-Seg's configs never select
  (INPUT.DATASET_MAPPER_NAME "mask_former_semantic", config.py:12).  They need pycocotools /
  panopticapi, which are not part of this path: constructing one raises.
"""
from __future__ import annotations

import copy
import logging

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image, ImageOps

from . import transforms as T


def read_image(path: str, fmt: str = "RGB") -> np.ndarray:
    """detectron2 `read_image`: EXIF orientation applied, converted to `fmt` (None = as stored),
    HWC numpy (HW1 for "L")."""
    with Image.open(path) as im:
        im = ImageOps.exif_transpose(im)
        if fmt is not None and fmt not in ("BGR",):
            im = im.convert(fmt)
        elif fmt == "BGR":
            im = im.convert("RGB")
        arr = np.asarray(im)
    if fmt == "BGR":
        arr = arr[:, :, ::-1]
    if fmt == "L":
        arr = arr[:, :, None]
    return arr


def check_image_size(dataset_dict: dict, image: np.ndarray):
    h, w = image.shape[:2]
    if ("height" in dataset_dict and dataset_dict["height"] != h) or ("width" in dataset_dict and
                                                                       dataset_dict["width"] != w):
        raise ValueError(f"Mismatched image shape for {dataset_dict.get('file_name')}: got {(h, w)}, expect "
                         f"{(dataset_dict.get('height'), dataset_dict.get('width'))}")
    dataset_dict.setdefault("width", w)
    dataset_dict.setdefault("height", h)


def _cfg_get(node, key, default):
    try:
        return getattr(node, key)
    except (AttributeError, KeyError):
        return default


class CATSegTestDatasetMapper:
    def __init__(self, cfg=None, *, min_size: int = 640, max_size: int = 2560, image_format: str = "RGB"):
        if cfg is not None:
            min_size = int(_cfg_get(cfg.INPUT, "MIN_SIZE_TEST", min_size))
            max_size = int(_cfg_get(cfg.INPUT, "MAX_SIZE_TEST", max_size))
            image_format = _cfg_get(cfg.INPUT, "FORMAT", image_format)
        self.augs = [T.ResizeShortestEdge(min_size, max_size, "choice")] if min_size > 0 else []
        self.image_format = image_format

    def __call__(self, dataset_dict: dict) -> dict:
        d = copy.deepcopy(dataset_dict)
        image = read_image(d["file_name"], self.image_format)
        check_image_size(d, image)
        image, _, _ = T.apply_augmentations(self.augs, image)
        d["image"] = torch.as_tensor(np.ascontiguousarray(image.transpose(2, 0, 1)))
        d.pop("annotations", None)
        d.pop("sem_seg_file_name", None)
        return d


class MaskFormerSemanticDatasetMapper:
    def __init__(self, cfg=None, is_train: bool = True, *, augmentations=None, image_format: str = "RGB",
                 ignore_label: int = 255, size_divisibility: int = -1):
        if cfg is not None:
            inp = cfg.INPUT
            augmentations = [T.ResizeShortestEdge(tuple(inp.MIN_SIZE_TRAIN), _cfg_get(inp, "MAX_SIZE_TRAIN", 1333),
                                                  _cfg_get(inp, "MIN_SIZE_TRAIN_SAMPLING", "choice"))]
            if inp.CROP.ENABLED:
                augmentations.append(T.RandomCropCategoryArea(
                    inp.CROP.TYPE, inp.CROP.SIZE, inp.CROP.SINGLE_CATEGORY_MAX_AREA,
                    cfg.MODEL.SEM_SEG_HEAD.IGNORE_VALUE))
            if _cfg_get(inp, "COLOR_AUG_SSD", False):
                augmentations.append(T.ColorAugSSD())
            augmentations.append(T.RandomFlip())
            image_format = inp.FORMAT
            size_divisibility = inp.SIZE_DIVISIBILITY
            try:
                from .catalog import MetadataCatalog
                ignore_label = MetadataCatalog.get(cfg.DATASETS.TRAIN[0]).ignore_label
            except (AttributeError, IndexError, KeyError):
                ignore_label = cfg.MODEL.SEM_SEG_HEAD.IGNORE_VALUE
        self.is_train = is_train
        self.tfm_gens = list(augmentations or [])
        self.img_format = image_format
        self.ignore_label = ignore_label
        self.size_divisibility = size_divisibility
        logging.getLogger(__name__).info("[%s] Augmentations used in %s: %s", type(self).__name__,
                                         "training" if is_train else "inference", self.tfm_gens)

    def __call__(self, dataset_dict: dict) -> dict:
        assert self.is_train, "MaskFormerSemanticDatasetMapper should only be used for training!"
        d = copy.deepcopy(dataset_dict)
        image = read_image(d["file_name"], self.img_format)
        check_image_size(d, image)
        if "sem_seg_file_name" not in d:
            raise ValueError(f"Cannot find 'sem_seg_file_name' for semantic segmentation dataset {d['file_name']}.")
        sem = read_image(d.pop("sem_seg_file_name"), None).astype("double")
        if sem.ndim == 3:
            sem = sem[:, :, 0]
        image, sem, _ = T.apply_augmentations(self.tfm_gens, image, sem)
        image = torch.as_tensor(np.ascontiguousarray(image.transpose(2, 0, 1)))
        sem = torch.as_tensor(sem.astype("long"))
        if self.size_divisibility > 0:
            h, w = image.shape[-2:]
            d["ori_size"] = (h, w)
            pad = [0, self.size_divisibility - w, 0, self.size_divisibility - h]
            image = F.pad(image, pad, value=128).contiguous()
            sem = F.pad(sem, pad, value=self.ignore_label).contiguous()
        d["image"] = image
        d["sem_seg"] = sem.long()
        if "annotations" in d:
            raise ValueError("Semantic segmentation dataset should not have 'annotations'.")
        s = sem.numpy()
        classes = np.unique(s)
        classes = classes[classes != self.ignore_label]
        masks = (torch.stack([torch.from_numpy(np.ascontiguousarray(s == c)) for c in classes]) if len(classes)
                 else torch.zeros((0,) + s.shape[-2:], dtype=torch.bool))
        d["instances"] = {"image_size": tuple(image.shape[-2:]), "gt_classes": torch.tensor(classes, dtype=torch.int64),
                          "gt_masks": masks}
        return d


class _PanopticMapperUnavailable:
    _what = "panoptic"

    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            f"{type(self).__name__}: {self._what} training data (MaskFormer lineage) is not part of the CAT-Seg "
            "MI355X path; CAT-Seg's configs use INPUT.DATASET_MAPPER_NAME 'mask_former_semantic' "
            "(MaskFormerSemanticDatasetMapper)")


class DETRPanopticDatasetMapper(_PanopticMapperUnavailable):
    _what = "DETR-style COCO panoptic"


class MaskFormerPanopticDatasetMapper(_PanopticMapperUnavailable):
    _what = "MaskFormer panoptic"
