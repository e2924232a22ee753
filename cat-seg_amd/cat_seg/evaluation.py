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
from the small (N+1)^2 matrix.  With an `output_dir`, `process()` also keeps the COCO-stuff
RLE records of every prediction (`encode_json_sem_seg`, plain_train_net.py:125,207-228; the RLE
is pycocotools' `mask.encode`, restated in `coco_rle_encode` since pycocotools is absent) and
`evaluate()` gathers them over ranks and writes `sem_seg_predictions.json`
(plain_train_net.py:139-152).
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


def coco_rle_encode(mask: np.ndarray) -> dict:
    """pycocotools `mask.encode` of one H x W binary mask (the call in plain_train_net.py:223), as
    {"size": [H, W], "counts": str}: run lengths over the column-major pixels, alternating and
    starting with a run of zeros (0 when pixel (0, 0) is set) -- maskApi.c rleEncode -- written
    with maskApi.c rleToString's compression: from the third count on, each count minus the count
    two before, in 5-bit groups low first, 0x20 = more groups follow, 0x10 of the last group = the
    sign, each group + 48 as one ASCII character.  pycocotools is not installed here: the string is
    checked against hand-derived vectors of that published algorithm and an independent decoder
    (tests/test_eval_cpu.py), not against pycocotools itself."""
    mask = np.asarray(mask)
    h, w = mask.shape
    flat = np.asarray(mask, dtype=bool).ravel(order="F")
    if flat.size == 0:
        cnts = [0]
    else:
        edges = np.flatnonzero(flat[1:] != flat[:-1]) + 1
        runs = np.diff(np.concatenate(([0], edges, [flat.size])))
        cnts = ([0] if flat[0] else []) + runs.tolist()
    # rleToString, vectorised: x_i = c_i - c_{i-2} (i > 2), n_i = the fewest 5-bit groups whose
    # two's complement holds x_i (the loop "until the rest is the last group's sign extension")
    c = np.asarray(cnts, dtype=np.int64)
    x = c.copy()
    if c.size > 3:
        x[3:] -= c[1:-2]
    n = np.ones_like(x)
    for k in range(1, 7):
        lim = 1 << (5 * k - 1)
        n += (x >= lim) | (x < -lim)
    ks = np.arange(int(n.max()))
    groups = (x[:, None] >> (5 * ks)[None, :]) & 0x1F
    more = ks[None, :] < (n[:, None] - 1)
    chars = groups + 48 + np.where(more, 0x20, 0)
    out = chars[ks[None, :] < n[:, None]].astype(np.uint8).tobytes().decode("ascii")
    return {"size": [int(h), int(w)], "counts": out}


_OBJ_GROUP = []


def _object_group():
    """A gloo process group over all ranks for object collectives (created once, collectively);
    None (the default group) when the default backend is gloo already."""
    if dist.get_backend() == "gloo":
        return None
    if not _OBJ_GROUP:
        _OBJ_GROUP.append(dist.new_group(backend="gloo"))
    return _OBJ_GROUP[0]


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
        # contiguous training ids -> dataset category ids for the RLE records (plain_train_net.py:84-90)
        c2d = meta.get("stuff_dataset_id_to_contiguous_id") if meta is not None else None
        self._contiguous_id_to_dataset_id = {v: k for k, v in c2d.items()} if c2d else None
        self.reset()

    def reset(self):
        n1 = self._num_classes + 1
        self._conf = torch.zeros(n1 * n1, dtype=torch.int64, device=self._device)
        self._invalid = torch.zeros(1, dtype=torch.int64, device=self._device)
        self._predictions = []

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
            if self._output_dir:
                # the records are written only with an output_dir, so only then is the argmax map
                # brought to the host (the reference builds them for every image)
                pred = probs.argmax(dim=0)
                if self.clamp_pred >= 0:
                    pred = pred.clamp(max=self.clamp_pred)
                self._predictions.extend(self.encode_json_sem_seg(pred.cpu().numpy(), inp.get("file_name")))

    def encode_json_sem_seg(self, sem_seg: np.ndarray, input_file_name) -> list:
        """COCO-stuff records of one argmax map (plain_train_net.py:207-228): one per label present,
        {"file_name", "category_id", "segmentation": RLE}, labels mapped to dataset ids when the
        metadata has stuff_dataset_id_to_contiguous_id."""
        records = []
        for label in np.unique(sem_seg):
            if self._contiguous_id_to_dataset_id is not None:
                if int(label) not in self._contiguous_id_to_dataset_id:
                    raise AssertionError(f"Label {label} is not in the metadata info for {self._dataset_name}")
                dataset_id = self._contiguous_id_to_dataset_id[int(label)]
            else:
                dataset_id = int(label)
            records.append({"file_name": input_file_name, "category_id": dataset_id,
                            "segmentation": coco_rle_encode(sem_seg == label)})
        return records

    def predictions(self) -> list:
        """The RLE records of every processed image, gathered over ranks in rank order
        (plain_train_net.py:139-140)."""
        if self._distributed and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            parts = [None] * dist.get_world_size()
            # Python objects go through a gloo group (as detectron2's comm.all_gather does), never
            # pickled into device buffers of the RCCL group
            dist.all_gather_object(parts, self._predictions, group=_object_group())
            return [r for part in parts for r in part]
        return list(self._predictions)

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
        preds = self.predictions() if self._output_dir else None
        if self._distributed and dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return None
        if self._output_dir:
            import json
            import os
            os.makedirs(self._output_dir, exist_ok=True)
            with open(os.path.join(self._output_dir, "sem_seg_predictions.json"), "w") as f:
                f.write(json.dumps(preds))
        res = self._metrics(conf)
        if self._output_dir:
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
