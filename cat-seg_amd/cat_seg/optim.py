"""The training loop's optimizer on the device: torch.optim.AdamW inside the reference's
FullModelGradientClippingOptimizer (train_net.py:228-253), as one HIP multi-tensor pass
(catseg_adamw_step, include/catseg_hip_train.h).

`AdamW` is a `torch.optim.Optimizer` with torch.optim.AdamW's constructor, parameter groups and
state layout ('step', 'exp_avg', 'exp_avg_sq'), so `build_optimizer`-style group construction,
LR schedulers and checkpoints interchange with torch's.  `max_grad_norm > 0` adds the full-model
gradient clipping the reference wraps around it (SOLVER.CLIP_GRADIENTS.CLIP_TYPE "full_model"):
the global norm and the clip coefficient stay on the device (no host sync), the gradients are
scaled in place as clip_grad_norm_ does.  `build_optimizer(cfg, model)` restates the reference's
per-parameter rules (train_net.py:174-226) on top of it.
"""
from __future__ import annotations

import copy
import ctypes as C
from typing import Any, Dict, List, Set

import torch

from . import _lib as L
from .ops import _stream, call


class _Desc(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("numel", C.c_int64), ("lr", C.c_float), ("weight_decay", C.c_float),
                ("bias_correction1", C.c_float), ("bias_correction2", C.c_float)]


def chunk_table(numels: List[int]) -> torch.Tensor:
    """The (tensor << 40 | chunk) table of catseg_adamw_step (host, int64)."""
    arr = (C.c_int64 * len(numels))(*numels)
    n = L.load().catseg_adamw_chunks(arr, len(numels))
    table = torch.empty(n, dtype=torch.int64)
    L.call("catseg_adamw_chunk_table", arr, len(numels), table.data_ptr())
    return table


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 max_grad_norm: float = 0.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("AdamW: invalid hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = float(max_grad_norm)
        self._table_key = None
        self._table = None
        self._norm = None

    @property
    def last_grad_norm(self):
        """Device tensor [total_norm, clip_coef] of the last step (clipping on), else None."""
        return self._norm

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        entries = []
        hp = set()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            hp.add((b1, b2, group["eps"]))
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise TypeError("AdamW (HIP): dense contiguous fp32 device parameters only")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                step = float(st["step"])
                entries.append((p, st, group["lr"], group["weight_decay"], 1 - b1 ** step, 1 - b2 ** step))
        if not entries:
            return loss
        if len(hp) != 1:
            raise ValueError("AdamW (HIP): one (betas, eps) for all parameter groups (the reference's setting)")
        b1, b2, eps = hp.pop()
        dev = entries[0][0].device
        key = tuple(p.numel() for p, *_ in entries)
        if key != self._table_key:
            self._table = chunk_table(list(key)).to(dev)
            self._table_key = key
            self._ws = torch.empty(self._table.numel(), device=dev, dtype=torch.float32)
        descs = (_Desc * len(entries))()
        for i, (p, st, lr, wd, bc1, bc2) in enumerate(entries):
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            if g is not p.grad:
                p.grad = g
            descs[i] = _Desc(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             p.numel(), lr, wd, bc1, bc2)
        raw = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev, non_blocking=False)
        clip = self.max_grad_norm > 0
        if clip and self._norm is None:
            self._norm = torch.empty(2, device=dev, dtype=torch.float32)
        call("catseg_adamw_step", raw.data_ptr(), self._table.data_ptr(), self._table.numel(), b1, b2, eps,
             self.max_grad_norm, self._norm.data_ptr() if clip else None, self._ws.data_ptr() if clip else None,
             self._ws.numel() * 4 if clip else 0, _stream())
        self._keep = raw          # the descriptor array must outlive the queued kernels
        # the kernel wrote the parameters through raw pointers, which autograd's version counters do
        # not see: bump them as an in-place torch op would, so that everything keyed on `_version`
        # (CATSeg.engine's converted inference weights, saved-tensor checks) sees the update
        torch.autograd.graph.increment_version([p for p, *_ in entries])
        return loss


class FullModelClipSGD(torch.optim.SGD):
    """torch.optim.SGD inside the reference's FullModelGradientClippingOptimizer (train_net.py:228-243):
    clip_grad_norm_ over every parameter of every group, then the SGD step."""

    def __init__(self, params, lr, momentum=0.0, max_grad_norm: float = 0.0):
        super().__init__(params, lr, momentum=momentum)
        self.max_grad_norm = float(max_grad_norm)

    def step(self, closure=None):
        if self.max_grad_norm > 0:
            all_params = [p for g in self.param_groups for p in g["params"]]
            torch.nn.utils.clip_grad_norm_(all_params, self.max_grad_norm)
        return super().step(closure=closure)


_NORM_TYPES = (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d, torch.nn.BatchNorm3d, torch.nn.SyncBatchNorm,
               torch.nn.GroupNorm, torch.nn.InstanceNorm1d, torch.nn.InstanceNorm2d, torch.nn.InstanceNorm3d,
               torch.nn.LayerNorm, torch.nn.LocalResponseNorm)


def build_optimizer(cfg, model: torch.nn.Module) -> torch.optim.Optimizer:
    """Trainer.build_optimizer (train_net.py:174-258): one group per trainable parameter with the
    reference's rules (BACKBONE_MULTIPLIER on "backbone", CLIP_MULTIPLIER on "clip_model",
    WEIGHT_DECAY_NORM on norm modules, WEIGHT_DECAY_EMBED on nn.Embedding, weight decay 0 for
    relative_position_bias_table / absolute_pos_embed), SOLVER.OPTIMIZER ADAMW on the device, SGD as
    torch's; either with full-model clipping when SOLVER.CLIP_GRADIENTS asks for it."""
    S = cfg.SOLVER
    defaults = {"lr": S.BASE_LR, "weight_decay": S.WEIGHT_DECAY}
    params: List[Dict[str, Any]] = []
    memo: Set[torch.nn.Parameter] = set()
    for module_name, module in model.named_modules():
        for param_name, value in module.named_parameters(recurse=False):
            if not value.requires_grad or value in memo:
                continue
            memo.add(value)
            hyper = copy.copy(defaults)
            if "backbone" in module_name:
                hyper["lr"] = hyper["lr"] * S.BACKBONE_MULTIPLIER
            if "clip_model" in module_name:
                hyper["lr"] = hyper["lr"] * S.CLIP_MULTIPLIER
            if "relative_position_bias_table" in param_name or "absolute_pos_embed" in param_name:
                hyper["weight_decay"] = 0.0            # train_net.py:216-221 (Swin-backbone parameters)
            if isinstance(module, _NORM_TYPES):
                hyper["weight_decay"] = S.WEIGHT_DECAY_NORM
            if isinstance(module, torch.nn.Embedding):
                hyper["weight_decay"] = S.WEIGHT_DECAY_EMBED
            params.append({"params": [value], **hyper})
    cg = S.CLIP_GRADIENTS
    full_clip = cg.ENABLED and cg.CLIP_TYPE == "full_model" and cg.CLIP_VALUE > 0.0
    if cg.ENABLED and cg.CLIP_TYPE != "full_model":
        raise NotImplementedError("per-parameter gradient clipping (detectron2 maybe_add_gradient_clipping, "
                                  "CLIP_TYPE 'value' / 'norm') is not built; the CAT-Seg configs use 'full_model'")
    if S.OPTIMIZER == "ADAMW":
        return AdamW(params, S.BASE_LR, max_grad_norm=cg.CLIP_VALUE if full_clip else 0.0)
    if S.OPTIMIZER == "SGD":
        return FullModelClipSGD(params, S.BASE_LR, momentum=S.MOMENTUM, max_grad_norm=cg.CLIP_VALUE if full_clip else 0.0)
    raise NotImplementedError(f"no optimizer type {S.OPTIMIZER}")
