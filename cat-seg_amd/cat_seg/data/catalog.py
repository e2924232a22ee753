"""Dataset / metadata catalogs and `load_sem_seg` (detectron2 v0.6 `data/catalog.py`,
`data/datasets/load_sem_seg`, reached from the reference's registration modules,
e.g. cat_seg/data/datasets/register_ade20k_150.py:1-4,24-25).

With detectron2 importable its own `DatasetCatalog` / `MetadataCatalog` / `load_sem_seg`
are used, so `train_net.py` sees the datasets the reference registers.  Without it the
same surface is provided here: a name -> loader registry, attribute-style metadata with
`set()` / `get()`, and the file-pairing rule of `load_sem_seg`.
"""
from __future__ import annotations

import logging
import os
from typing import Callable, Dict, List

try:  # pragma: no cover - detectron2 is not in this image
    from detectron2.data import DatasetCatalog, MetadataCatalog  # noqa: F401
    from detectron2.data.datasets import load_sem_seg  # noqa: F401
    HAVE_D2 = True
except Exception:  # noqa: BLE001
    HAVE_D2 = False

    class _DatasetCatalog(dict):
        """name -> zero-argument function returning list[dict] (detectron2 DatasetCatalog)."""

        def register(self, name: str, func: Callable[[], List[dict]]):
            if not callable(func):
                raise TypeError("DatasetCatalog.register needs a callable")
            if name in self:
                raise AssertionError(f"Dataset '{name}' is already registered!")
            self[name] = func

        def get(self, name: str) -> List[dict]:
            try:
                f = self[name]
            except KeyError as e:
                raise KeyError(f"Dataset '{name}' is not registered! Available datasets are: "
                               f"{', '.join(sorted(self.keys()))}") from e
            return f()

        def list(self) -> List[str]:
            return list(self.keys())

        def remove(self, name: str):
            self.pop(name)

    class Metadata:
        """Attribute bag with write-once fields (detectron2 `Metadata`)."""

        def __init__(self, name: str):
            object.__setattr__(self, "name", name)

        def __getattr__(self, key):
            raise AttributeError(f"Attribute '{key}' does not exist in the metadata of dataset "
                                 f"'{self.name}'. Available keys are {list(self.__dict__)}.")

        def __setattr__(self, key, val):
            old = self.__dict__.get(key)
            if key in self.__dict__ and old != val:
                raise AssertionError(f"Attribute '{key}' in the metadata of '{self.name}' cannot be set "
                                     f"to a different value!\n{old} != {val}")
            object.__setattr__(self, key, val)

        def set(self, **kwargs):
            for k, v in kwargs.items():
                setattr(self, k, v)
            return self

        def get(self, key, default=None):
            return self.__dict__.get(key, default)

        def as_dict(self) -> dict:
            return dict(self.__dict__)

    class _MetadataCatalog(dict):
        def get(self, name: str) -> "Metadata":
            if name not in self:
                self[name] = Metadata(name)
            return self[name]

        def list(self) -> List[str]:
            return list(self.keys())

        def remove(self, name: str):
            self.pop(name)

    DatasetCatalog = _DatasetCatalog()
    MetadataCatalog = _MetadataCatalog()

    def load_sem_seg(gt_root: str, image_root: str, gt_ext: str = "png", image_ext: str = "jpg") -> List[Dict]:
        """detectron2 `load_sem_seg`: list the files of `image_root` / `gt_root` (one directory
        level) ending in image_ext / gt_ext, sorted by name; when the counts differ keep the
        names present in both.  Returns [{"file_name", "sem_seg_file_name"}]."""
        log = logging.getLogger(__name__)
        inputs = sorted(f for f in os.listdir(image_root) if f.endswith(image_ext))
        gts = sorted(f for f in os.listdir(gt_root) if f.endswith(gt_ext))
        if not gts:
            raise FileNotFoundError(f"No annotations found in {gt_root}.")
        if len(inputs) != len(gts):
            log.warning("Directory %s and %s has %d and %d files, respectively.", image_root, gt_root,
                        len(inputs), len(gts))
            both = sorted({f[: -len(image_ext)] for f in inputs} & {f[: -len(gt_ext)] for f in gts})
            inputs = [f + image_ext for f in both]
            gts = [f + gt_ext for f in both]
        log.info("Loaded %d images with semantic segmentation from %s", len(inputs), image_root)
        return [{"file_name": os.path.join(image_root, i), "sem_seg_file_name": os.path.join(gt_root, g)}
                for i, g in zip(inputs, gts)]
