"""Test-time augmentation wrapper (reference cat_seg/test_time_augmentation.py:19-113, used by
train_net.py:260-274 when TEST.AUG.ENABLED).

For each image: the multi-scale + flip variants of detectron2's `DatasetMapperTTA`
(ResizeShortestEdge to every TEST.AUG.MIN_SIZES entry with long edge <= TEST.AUG.MAX_SIZE,
each also horizontally flipped when TEST.AUG.FLIP) run through the wrapped model in batches of
`batch_size`; flipped predictions are flipped back and all are averaged.  The model returns
probabilities at the original "height" x "width", so the variants align without resampling.
"""
from __future__ import annotations

import copy

import numpy as np
import torch
from torch import nn

from .data import transforms as T
from .data.dataset_mappers import read_image


def _aug_cfg(cfg):
    aug = cfg.TEST.AUG
    get = (lambda k, d: getattr(aug, k, d)) if not isinstance(aug, dict) else (lambda k, d: aug.get(k, d))
    return (tuple(get("MIN_SIZES", (400, 500, 600, 700, 800, 900, 1000, 1100, 1200))),
            int(get("MAX_SIZE", 4000)), bool(get("FLIP", True)))


class DatasetMapperTTA:
    """dataset dict with "image" (CHW uint8) -> list of augmented dicts, each with its "transforms"."""

    def __init__(self, cfg=None, *, min_sizes=(400, 500, 600, 700, 800, 900, 1000, 1100, 1200), max_size=4000,
                 flip=True):
        if cfg is not None:
            min_sizes, max_size, flip = _aug_cfg(cfg)
        self.min_sizes, self.max_size, self.flip = tuple(min_sizes), max_size, flip

    def __call__(self, dataset_dict):
        img = dataset_dict["image"].permute(1, 2, 0).numpy()
        ret = []
        for s in self.min_sizes:
            cands = [[T.ResizeShortestEdge(s, self.max_size, "choice")]]
            if self.flip:
                cands.append([T.ResizeShortestEdge(s, self.max_size, "choice"), T.RandomFlip(prob=1.0)])
            for augs in cands:
                new, _, tfms = T.apply_augmentations(augs, np.copy(img))
                d = copy.deepcopy({k: v for k, v in dataset_dict.items() if k != "image"})
                d["image"] = torch.from_numpy(np.ascontiguousarray(new.transpose(2, 0, 1)))
                d["transforms"] = tfms
                ret.append(d)
        return ret


class SemanticSegmentorWithTTA(nn.Module):
    def __init__(self, cfg, model, tta_mapper=None, batch_size: int = 1):
        super().__init__()
        if isinstance(model, nn.parallel.DistributedDataParallel):
            model = model.module
        self.cfg = cfg.clone() if hasattr(cfg, "clone") else cfg
        self.model = model
        self.tta_mapper = tta_mapper if tta_mapper is not None else DatasetMapperTTA(cfg)
        self.batch_size = batch_size

    def _batch_inference(self, batched_inputs):
        outputs = []
        for i in range(0, len(batched_inputs), self.batch_size):
            with torch.no_grad():
                outputs.extend(self.model(batched_inputs[i:i + self.batch_size]))
        return outputs

    def __call__(self, batched_inputs):
        def maybe_read(d):
            ret = copy.copy(d)
            if "image" not in ret:
                image = read_image(ret.pop("file_name"), getattr(self.model, "input_format", "RGB"))
                ret["image"] = torch.from_numpy(np.ascontiguousarray(image.transpose(2, 0, 1)))
            if "height" not in ret and "width" not in ret:
                ret["height"], ret["width"] = ret["image"].shape[1], ret["image"].shape[2]
            return ret

        return [self._inference_one_image(maybe_read(x)) for x in batched_inputs]

    def _inference_one_image(self, inp):
        augmented = self.tta_mapper(inp)
        tfms = [a.pop("transforms") for a in augmented]
        outputs = self._batch_inference(augmented)
        del augmented
        acc = None
        for out, tfm in zip(outputs, tfms):
            p = out.pop("sem_seg")
            if any(isinstance(t, T.HFlipTransform) for t in tfm):
                p = p.flip(dims=[2])
            acc = p if acc is None else acc + p
        return {"sem_seg": acc / len(outputs)}
