"""Detectron2 plugin surface: META_ARCH_REGISTRY / SEM_SEG_HEADS_REGISTRY, `configurable`,
`build_model` (reference: cat_seg_model.py:18-20, cat_seg_head.py:1965-1968).

With detectron2 installed, its registries and `configurable` are used, so
`MODEL.META_ARCHITECTURE: "CATSeg"` in train_net.py / eval.sh resolves to this
package's CATSeg.  Without it, equivalent minimal versions are provided.
"""
from __future__ import annotations

import functools
import inspect

try:  # pragma: no cover - detectron2 is not in this image
    from detectron2.config import configurable  # noqa: F401
    from detectron2.modeling import META_ARCH_REGISTRY, SEM_SEG_HEADS_REGISTRY  # noqa: F401
    HAVE_D2 = True
except Exception:  # noqa: BLE001
    HAVE_D2 = False

    class Registry:
        def __init__(self, name):
            self.name = name
            self._obj = {}

        def register(self, obj=None):
            def deco(o):
                if o.__name__ in self._obj:
                    raise KeyError(f"{o.__name__} already registered in {self.name}")
                self._obj[o.__name__] = o
                return o
            return deco(obj) if obj is not None else deco

        def get(self, name):
            if name not in self._obj:
                raise KeyError(f"No object named '{name}' found in '{self.name}' registry!")
            return self._obj[name]

        def __contains__(self, name):
            return name in self._obj

    META_ARCH_REGISTRY = Registry("META_ARCH")
    SEM_SEG_HEADS_REGISTRY = Registry("SEM_SEG_HEADS")

    def _is_cfg(x):
        return hasattr(x, "MODEL") and hasattr(x, "merge_from_file")

    def configurable(init_func):
        """detectron2.config.configurable for __init__: `Cls(cfg, ...)` -> `Cls(**Cls.from_config(cfg, ...))`."""
        @functools.wraps(init_func)
        def wrapped(self, *args, **kwargs):
            if args and _is_cfg(args[0]):
                fc = type(self).from_config
                n = len(inspect.signature(fc).parameters)
                explicit = fc(*args[: n], **{k: v for k, v in kwargs.items()
                                             if k in inspect.signature(fc).parameters})
                explicit.update({k: v for k, v in kwargs.items() if k not in inspect.signature(fc).parameters})
                return init_func(self, **explicit)
            return init_func(self, *args, **kwargs)
        return wrapped


def build_model(cfg):
    """detectron2.modeling.build_model: META_ARCH_REGISTRY[cfg.MODEL.META_ARCHITECTURE](cfg), moved
    to cfg.MODEL.DEVICE.  A "cuda" device is only bound when CUDA is present (the CPU-only
    tests build models without a GPU; the HIP engine itself always needs one)."""
    import torch
    model = META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg)
    dev = torch.device(getattr(cfg.MODEL, "DEVICE", "cuda") or "cuda")
    if dev.type != "cuda" or torch.cuda.is_available():
        model.to(dev)
    return model


def build_sem_seg_head(cfg, input_shape=None):
    return SEM_SEG_HEADS_REGISTRY.get(cfg.MODEL.SEM_SEG_HEAD.NAME)(cfg, input_shape)
