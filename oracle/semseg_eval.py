"""CPU oracle for the evaluation harness — TEST INFRASTRUCTURE ONLY (the checker of
catseg_semseg_confusion and cat_seg.evaluation; never imported by the product path).

Restates, in numpy, the evaluator CAT-Seg runs (detectron2 v0.6 `SemSegEvaluator`, as
copied into the reference as `SemSegGzeroEvaluator`, plain_train_net.py:48-200, and its
VOC-b variant, train_net.py:43-67).  detectron2 is not vendored in the reference and not
importable here; the reference's own copy above is the anchor ("parity pinned" to it by the
hand-computed known-answer case in tests/test_eval_cpu.py).
"""
from __future__ import annotations

import numpy as np


def confusion_update(conf: np.ndarray, sem_seg: np.ndarray, gt: np.ndarray, num_classes: int,
                     ignore_label: int, clamp_pred: int = -1) -> np.ndarray:
    """SemSegGzeroEvaluator.process (plain_train_net.py:107-116); VOC-b pred fold
    (train_net.py:57): conf[(N+1) * pred + gt] += 1."""
    pred = np.asarray(sem_seg).argmax(axis=0).astype(np.int64)
    if clamp_pred >= 0:
        pred[pred >= clamp_pred] = clamp_pred
    gt = np.asarray(gt).astype(np.int64).copy()
    gt[gt == ignore_label] = num_classes
    conf += np.bincount((num_classes + 1) * pred.reshape(-1) + gt.reshape(-1),
                        minlength=conf.size).reshape(conf.shape)
    return conf


def metrics(conf: np.ndarray, class_names, val_extra_classes=()) -> dict:
    """SemSegGzeroEvaluator.evaluate (plain_train_net.py:153-197): mIoU / fwIoU / mACC / pACC,
    per-class IoU / ACC, seen / unseen IoU and their harmonic mean when val_extra_classes
    is given (with none, the plain SemSegEvaluator keys only)."""
    n = len(class_names)
    acc = np.full(n, np.nan, dtype=np.float64)
    iou = np.full(n, np.nan, dtype=np.float64)
    tp = conf.diagonal()[:-1].astype(np.float64)
    pos_gt = np.sum(conf[:-1, :-1], axis=0).astype(np.float64)
    class_weights = pos_gt / np.sum(pos_gt)
    pos_pred = np.sum(conf[:-1, :-1], axis=1).astype(np.float64)
    acc_valid = pos_gt > 0
    acc[acc_valid] = tp[acc_valid] / pos_gt[acc_valid]
    iou_valid = (pos_gt + pos_pred) > 0
    union = pos_gt + pos_pred - tp
    iou[acc_valid] = tp[acc_valid] / union[acc_valid]
    macc = np.sum(acc[acc_valid]) / np.sum(acc_valid)
    miou = np.sum(iou[acc_valid]) / np.sum(iou_valid)
    fiou = np.sum(iou[acc_valid] * class_weights[acc_valid])
    pacc = np.sum(tp) / np.sum(pos_gt)
    res = {"mIoU": 100 * miou, "fwIoU": 100 * fiou}
    for i, name in enumerate(class_names):
        res[f"IoU-{name}"] = 100 * iou[i]
    res["mACC"] = 100 * macc
    res["pACC"] = 100 * pacc
    for i, name in enumerate(class_names):
        res[f"ACC-{name}"] = 100 * acc[i]
    if len(val_extra_classes):
        seen = unseen = 0.0
        for i, name in enumerate(class_names):
            if name in val_extra_classes:
                unseen += 100 * iou[i]
            else:
                seen += 100 * iou[i]
        unseen /= len(val_extra_classes)
        seen /= n - len(val_extra_classes)
        res["seen_IoU"] = seen
        res["unseen_IoU"] = unseen
        res["harmonic mean"] = 2 * seen * unseen / (seen + unseen)
    return res


def rle_encode(mask: np.ndarray) -> dict:
    """pycocotools `mask.encode` of one H x W binary mask (plain_train_net.py:223; pycocotools is
    not vendored in the reference and not installed here), restated with plain loops after its
    published C source: maskApi.c rleEncode (column-major run lengths, alternating, starting with
    zeros) then rleToString (delta against the count two back from the third on, 5-bit groups with
    continuation bit 0x20 and sign bit 0x10, + 48).  Parity unpinned against pycocotools itself."""
    mask = np.asarray(mask)
    h, w = mask.shape
    cnts, prev, run = [], 0, 0
    for j in range(w):
        for i in range(h):
            v = 1 if mask[i, j] else 0
            if v != prev:
                cnts.append(run)
                run, prev = 0, v
            run += 1
    cnts.append(run)
    s = []
    for i, c in enumerate(cnts):
        x = c - cnts[i - 2] if i > 2 else c
        more = True
        while more:
            g = x & 0x1F
            x >>= 5
            more = x != -1 if g & 0x10 else x != 0
            if more:
                g |= 0x20
            s.append(chr(g + 48))
    return {"size": [h, w], "counts": "".join(s)}


def rle_decode(rle: dict) -> np.ndarray:
    """maskApi.c rleFrString + rleDecode: the inverse of rle_encode (an H x W uint8 mask)."""
    h, w = rle["size"]
    s, p, cnts = rle["counts"], 0, []
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(cnts) > 2:
            x += cnts[-2]
        cnts.append(x)
    flat = np.zeros(h * w, np.uint8)
    pos, v = 0, 0
    for c in cnts:
        flat[pos:pos + c] = v
        pos += c
        v ^= 1
    assert pos == h * w, "counts do not cover the mask"
    return flat.reshape(w, h).T


def sem_seg_records(pred: np.ndarray, file_name, contiguous_to_dataset=None) -> list:
    """encode_json_sem_seg (plain_train_net.py:207-228) of one argmax map."""
    out = []
    for label in np.unique(pred):
        cid = contiguous_to_dataset[int(label)] if contiguous_to_dataset is not None else int(label)
        out.append({"file_name": file_name, "category_id": cid, "segmentation": rle_encode(pred == label)})
    return out
