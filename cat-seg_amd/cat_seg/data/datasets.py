"""Registration of the evaluation datasets the reference's scripts name (eval.sh:28-104,
configs/config.yaml DATASETS), under the same names, paths, loaders and metadata as the
reference's registration modules:

  ade20k_150_test_sem_seg            register_ade20k_150.py:15-25
  ade20k_full_sem_seg_freq_val_all   register_ade20k_847.py:31-53  (16-bit TIFF labels)
  voc_2012_test_sem_seg              register_pascal_20.py:20-36
  voc_2012_test_background_sem_seg   register_pascal_20.py:20-36   (evaluator "sem_seg_background")
  context_59_test_sem_seg            register_pascal_context.py:44-54
  context_459_test_sem_seg           register_pascal_context.py:65-75 (TIFF labels, ignore 459)
  coco_2017_{train,test}_stuff_all_sem_seg   register_coco_stuff.py:194-213

Roots follow $DETECTRON2_DATASETS (default "datasets"), read at import time as there.
Nothing is read from disk until a dataset's loader is called.  Registration targets
detectron2's catalogs when detectron2 is importable (so train_net.py's Trainer.test finds
them), else the stand-in catalogs of cat_seg.data.catalog.  Class names come from the
package's copy of the reference class lists (data/class_names.json).
"""
from __future__ import annotations

import json
import os

from .catalog import DatasetCatalog, MetadataCatalog, load_sem_seg

_HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(_HERE, "class_names.json")) as _f:
    CLASS_NAMES = json.load(_f)

# VOC colours of register_pascal_20.py:9-13 (the background row first)
_VOC_COLORS = [[0, 0, 0], [128, 0, 0], [0, 128, 0], [128, 128, 0], [0, 0, 128], [128, 0, 128], [0, 128, 128],
               [128, 128, 128], [64, 0, 0], [192, 0, 0], [64, 128, 0], [192, 128, 0], [64, 0, 128], [192, 0, 128],
               [64, 128, 128], [192, 128, 128], [0, 64, 0], [128, 64, 0], [0, 192, 0], [128, 192, 0], [0, 64, 128]]


def _register(name, image_dir, gt_dir, gt_ext, image_ext="jpg", **meta):
    if name in DatasetCatalog.list():
        return
    DatasetCatalog.register(name, lambda x=image_dir, y=gt_dir, e=gt_ext, i=image_ext: load_sem_seg(y, x, gt_ext=e,
                                                                                                   image_ext=i))
    MetadataCatalog.get(name).set(image_root=image_dir, **meta)


def register_ade20k_150(root):
    root = os.path.join(root, "ADEChallengeData2016")
    image_dir = os.path.join(root, "images/validation")
    gt_dir = os.path.join(root, "annotations_detectron2/validation")
    # the reference spells the key "seg_seg_root" here (register_ade20k_150.py:25)
    _register("ade20k_150_test_sem_seg", image_dir, gt_dir, "png", seg_seg_root=gt_dir, evaluator_type="sem_seg",
              ignore_label=255, stuff_classes=list(CLASS_NAMES["ade150"]))


def register_ade20k_847(root):
    root = os.path.join(root, "ADE20K_2021_17_01")
    image_dir = os.path.join(root, "images_detectron2", "validation")
    gt_dir = os.path.join(root, "annotations_detectron2", "validation")
    _register("ade20k_full_sem_seg_freq_val_all", image_dir, gt_dir, "tif", sem_seg_root=gt_dir,
              evaluator_type="sem_seg", ignore_label=65535, stuff_classes=list(CLASS_NAMES["ade847"]))


def register_pascal_voc(root):
    root = os.path.join(root, "VOCdevkit/VOC2012")
    classes = list(CLASS_NAMES["voc20"])
    for name, image_dirname, gt_dirname in (("test", "JPEGImages", "annotations_detectron2"),
                                            ("test_background", "JPEGImages", "annotations_detectron2_bg")):
        image_dir = os.path.join(root, image_dirname)
        gt_dir = os.path.join(root, gt_dirname, "val")
        full = f"voc_2012_{name}_sem_seg"
        if "background" in name:
            _register(full, image_dir, gt_dir, "png", seg_seg_root=gt_dir, evaluator_type="sem_seg_background",
                      ignore_label=255, stuff_classes=classes + ["background"], stuff_colors=_VOC_COLORS)
        else:
            _register(full, image_dir, gt_dir, "png", seg_seg_root=gt_dir, evaluator_type="sem_seg",
                      ignore_label=255, stuff_classes=classes, stuff_colors=_VOC_COLORS)


def register_pascal_context(root):
    root = os.path.join(root, "VOCdevkit", "VOC2010")
    image_dir = os.path.join(root, "JPEGImages")
    for n, sub, ext, ignore in ((59, "pc59_val", "png", 255), (459, "pc459_val", "tif", 459)):
        gt_dir = os.path.join(root, "annotations_detectron2", sub)
        _register(f"context_{n}_test_sem_seg", image_dir, gt_dir, ext, seg_seg_root=gt_dir,
                  evaluator_type="sem_seg", ignore_label=ignore, stuff_classes=list(CLASS_NAMES[f"pc{n}"]))


def register_coco_stuff(root):
    root = os.path.join(root, "coco-stuff")
    for name, image_dirname, gt_dirname in (("train", "images/train2017", "annotations_detectron2/train2017"),
                                            ("test", "images/val2017", "annotations_detectron2/val2017")):
        image_dir = os.path.join(root, image_dirname)
        gt_dir = os.path.join(root, gt_dirname)
        _register(f"coco_2017_{name}_stuff_all_sem_seg", image_dir, gt_dir, "png", sem_seg_root=gt_dir,
                  evaluator_type="sem_seg", ignore_label=255, stuff_classes=list(CLASS_NAMES["coco"]))


def register_all(root=None):
    root = root if root is not None else os.getenv("DETECTRON2_DATASETS", "datasets")
    register_coco_stuff(root)
    register_ade20k_150(root)
    register_ade20k_847(root)
    register_pascal_voc(root)
    register_pascal_context(root)


register_all()
