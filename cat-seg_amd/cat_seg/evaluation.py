"""Evaluation harness: detectron2's `DatasetEvaluator` surface for semantic segmentation
(SURVEY §8f rank 3), with the per-image confusion-matrix update on the device.

Mirrors the evaluators the reference registers (train_net.py:89-149):
  * `SemSegEvaluator`       — detectron2 v0.6 `SemSegEvaluator` (the copy the reference keeps
                              as `SemSegGzeroEvaluator`, plain_train_net.py:48-200, without
                              the seen/unseen split);
  * `SemSegGzeroEvaluator`  — + seen / unseen IoU and their harmonic mean over
                              `val_extra_classes` (plain_train_net.py:170-197);
  * `VOCbEvaluator`         — VOC with background: predictions >= 20 fold to 20
                              (train_net.py:43-67).
`process()` bins every pixel with `catseg_semseg_confusion` (argmax over the class planes +
int64 bincount, exact); `evaluate()` sums the matrices over ranks (torch.distributed, as
detectron2's `all_gather`, plain_train_net.py:136-146) and forms the metrics on the host
from the small (N+1)^2 matrix.  Not reproduced: the COCO-RLE `sem_seg_predictions.json`
dump (`encode_json_sem_seg`, needs pycocotools).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import ops


def _metadata(dataset_name):
    """MetadataCatalog entry (detectron2's when importable, else cat_seg.data's stand-in, where
    the reference's dataset names are registered on import); None without a name."""
    from .data.catalog import MetadataCatalog
    return MetadataCatalog.get(dataset_name) if dataset_name else None


def _catalog_gt_loader(dataset_name):
    """detectron2 SemSegEvaluator's ground truth: the label file registered for the input's
    "file_name" (input_file_to_gt_file), read as stored (8-bit PNG or 16-bit TIFF)."""
    from PIL import Image
    from .data.catalog import DatasetCatalog
    table = {d["file_name"]: d["sem_seg_file_name"] for d in DatasetCatalog.get(dataset_name)}

    def load(inp):
        with Image.open(table[inp["file_name"]]) as im:
            return np.array(im, dtype=np.int64)
    return load


def reduce_confusion(conf: torch.Tensor) -> torch.Tensor:
    """Sum the per-rank confusion matrices (plain_train_net.py:136-146); returns a CPU int64 tensor."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = conf.clone() if dist.get_backend() == "nccl" else conf.cpu().clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        conf = t
    return conf.cpu()


def semseg_metrics(conf: np.ndarray, class_names: Sequence[str], val_extra_classes: Sequence[str] = ()) -> dict:
    """The metrics of SemSegGzeroEvaluator.evaluate (plain_train_net.py:153-197) from an
    (N+1) x (N+1) confusion matrix indexed [pred][gt] (row N / column N: ignored pixels)."""
    conf = np.asarray(conf, dtype=np.int64)
    n = len(class_names)
    if conf.shape != (n + 1, n + 1):
        raise ValueError(f"confusion matrix {conf.shape} does not match {n} classes")
    core = conf[:-1, :-1].astype(np.float64)
    tp = np.diagonal(conf)[:-1].astype(np.float64)
    pos_gt = core.sum(axis=0)
    pos_pred = core.sum(axis=1)
    gt_seen = pos_gt > 0
    acc = np.where(gt_seen, tp / np.where(gt_seen, pos_gt, 1.0), np.nan)
    union = pos_gt + pos_pred - tp
    iou = np.where(gt_seen, tp / np.where(gt_seen, union, 1.0), np.nan)
    weights = pos_gt / pos_gt.sum()
    res = {"mIoU": 100 * iou[gt_seen].sum() / ((pos_gt + pos_pred) > 0).sum(),
           "fwIoU": 100 * (iou[gt_seen] * weights[gt_seen]).sum()}
    res.update({f"IoU-{c}": 100 * iou[i] for i, c in enumerate(class_names)})
    res["mACC"] = 100 * acc[gt_seen].sum() / gt_seen.sum()
    res["pACC"] = 100 * tp.sum() / pos_gt.sum()
    res.update({f"ACC-{c}": 100 * acc[i] for i, c in enumerate(class_names)})
    if len(val_extra_classes):
        extra = np.array([c in val_extra_classes for c in class_names])
        unseen = (100 * iou[extra]).sum() / len(val_extra_classes)
        seen = (100 * iou[~extra]).sum() / (n - len(val_extra_classes))
        res["seen_IoU"], res["unseen_IoU"] = seen, unseen
        res["harmonic mean"] = 2 * seen * unseen / (seen + unseen)
    return res


class SemSegEvaluator:
    """reset() / process(inputs, outputs) / evaluate() -> {"sem_seg": metrics}.

    Ground truth per input: `input["sem_seg_gt"]` (H x W labels, tensor or array), else
    `gt_loader(input)` (e.g. reading `input["file_name"]`'s `sem_seg_file_name` as the
    reference does).  `class_names` / `ignore_label` come from detectron2's MetadataCatalog
    when it is importable, else from the arguments."""

    clamp_pred = -1

    def __init__(self, dataset_name: Optional[str] = None, distributed: bool = True, output_dir=None, *,
                 class_names: Optional[Sequence[str]] = None, ignore_label: Optional[int] = None,
                 gt_loader: Optional[Callable] = None, device=None):
        meta = _metadata(dataset_name)
        if class_names is None:
            class_names = meta.get("stuff_classes") if meta is not None else None
            if class_names is None:
                raise ValueError(f"SemSegEvaluator: no class names (dataset {dataset_name!r} has no 'stuff_classes' "
                                 "metadata and class_names= was not given)")
        self._class_names = list(class_names)
        self._num_classes = len(self._class_names)
        self._ignore_label = ignore_label if ignore_label is not None else (
            meta.get("ignore_label", 255) if meta is not None else 255)
        self._distributed = distributed
        self._output_dir = output_dir
        self._dataset_name = dataset_name
        self._gt_loader = gt_loader
        self._device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.reset()

    def reset(self):
        n1 = self._num_classes + 1
        self._conf = torch.zeros(n1 * n1, dtype=torch.int64, device=self._device)
        self._invalid = torch.zeros(1, dtype=torch.int64, device=self._device)

    def _gt(self, inp) -> torch.Tensor:
        gt = inp.get("sem_seg_gt")
        if gt is None:
            if self._gt_loader is None and self._dataset_name and "file_name" in inp:
                self._gt_loader = _catalog_gt_loader(self._dataset_name)
            if self._gt_loader is None:
                raise KeyError("input has no 'sem_seg_gt' and no gt_loader / registered dataset was given")
            gt = self._gt_loader(inp)
        gt = torch.as_tensor(np.asarray(gt) if not torch.is_tensor(gt) else gt)
        return gt.to(self._device, torch.int32).contiguous()

    def process(self, inputs, outputs):
        with torch.cuda.device(self._device):      # the kernel runs on this device's current stream
            self._process(inputs, outputs)

    def _process(self, inputs, outputs):
        for inp, out in zip(inputs, outputs):
            probs = out["sem_seg"] if isinstance(out, dict) else out
            probs = probs.to(self._device, torch.float32).contiguous()
            gt = self._gt(inp)
            if tuple(gt.shape) != tuple(probs.shape[1:]):
                raise ValueError(f"gt {tuple(gt.shape)} vs prediction {tuple(probs.shape[1:])}")
            ops.semseg_confusion(probs, gt, self._conf, self._invalid, num_classes=self._num_classes,
                                 ignore_label=self._ignore_label, clamp_pred=self.clamp_pred)

    def confusion_matrix(self) -> np.ndarray:
        n1 = self._num_classes + 1
        conf = reduce_confusion(self._conf) if self._distributed else self._conf.cpu()
        return conf.numpy().reshape(n1, n1)

    def _metrics(self, conf):
        return semseg_metrics(conf, self._class_names)

    def evaluate(self):
        invalid = int(reduce_confusion(self._invalid)[0]) if self._distributed else int(self._invalid.item())
        if invalid:
            # the reference's bincount would outgrow the matrix and its reshape would fail
            raise ValueError(f"{invalid} ground-truth labels outside [0, {self._num_classes}) and != ignore_label")
        conf = self.confusion_matrix()
        if self._distributed and dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return None
        res = self._metrics(conf)
        if self._output_dir:
            import os
            os.makedirs(self._output_dir, exist_ok=True)
            torch.save(res, os.path.join(self._output_dir, "sem_seg_evaluation.pth"))
        return OrderedDict({"sem_seg": res})


class SemSegGzeroEvaluator(SemSegEvaluator):
    """+ seen / unseen IoU and harmonic mean over `val_extra_classes` (plain_train_net.py:48-200)."""

    def __init__(self, *args, val_extra_classes: Optional[Sequence[str]] = None, **kw):
        super().__init__(*args, **kw)
        if val_extra_classes is None:
            meta = _metadata(args[0] if args else kw.get("dataset_name"))
            val_extra_classes = meta.get("val_extra_classes", ()) if meta is not None else ()
        self._val_extra_classes = list(val_extra_classes)

    def _metrics(self, conf):
        return semseg_metrics(conf, self._class_names, self._val_extra_classes)


class VOCbEvaluator(SemSegEvaluator):
    """VOC with background: predictions >= 20 fold to class 20 (train_net.py:55-58)."""

    clamp_pred = 20
