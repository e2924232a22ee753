"""Real `nn.Module` parameter trees under the reference's module names.

The reference's CATSeg owns its weights through an nn.Module tree (CLIP under
`sem_seg_head.predictor.clip_model`, the Aggregator under `sem_seg_head.predictor.transformer`,
the guidance upsamplers `upsample1/2`; module tree printed in reference `vizDebug/log.txt:1446-1870`).
Training code written against it — detectron2's `build_optimizer` in `train_net.py:174-258`,
which picks per-parameter hyper-parameters by module name ("clip_model") and by module type
(nn.LayerNorm / nn.GroupNorm / nn.Embedding) — needs that tree.  `attach_parameters` builds it
from a flat reference state dict: every leaf is the torch module type the reference uses
(nn.Linear, nn.Conv2d, nn.ConvTranspose2d, nn.LayerNorm, nn.GroupNorm, nn.Embedding), created on
the meta device and then given the state-dict tensors as its nn.Parameters (no copy).  Free
parameters (class_embedding, positional_embedding, proj, q/k/v_proj_weight, in_proj_bias,
padding_tokens, ...) sit on plain container modules, as in the reference.

These modules are parameter holders: their forward is never called.  The HIP engine reads the
tensors (CatSegEngine for inference, cat_seg.training for the training step).
"""
from __future__ import annotations

import re
from typing import Dict

import torch
from torch import nn

# module path patterns -> leaf module kind (first match wins)
_KINDS = [
    (re.compile(r"(^|\.)(ln_1|ln_2|ln_pre|ln_post|ln_final|norm1|norm2|guidance_norm)$"), "layernorm"),
    (re.compile(r"\.double_conv\.(1|4)$"), "groupnorm"),
    (re.compile(r"(^|\.)token_embedding$"), "embedding"),
    (re.compile(r"(^upsample[12]|\.up)$"), "convt"),
    (re.compile(r"(\.conv1|\.guidance_projection\.0|\.decoder_guidance_projection\.\d+\.0|\.double_conv\.(0|3)|\.head)$"),
     "conv"),
]


def _kind(path: str, tensors: Dict[str, torch.Tensor]) -> str:
    for pat, kind in _KINDS:
        if pat.search(path):
            return kind
    if set(tensors) <= {"weight", "bias"} and "weight" in tensors and tensors["weight"].dim() == 2:
        return "linear"
    return "container"


def _leaf(kind: str, t: Dict[str, torch.Tensor]) -> nn.Module:
    w = t.get("weight")
    meta = {"device": "meta"}
    if kind == "layernorm":
        return nn.LayerNorm(w.shape[0], **meta)
    if kind == "groupnorm":
        return nn.GroupNorm(w.shape[0] // 16, w.shape[0], **meta)      # model.py:529,532: C // 16 groups
    if kind == "embedding":
        return nn.Embedding(w.shape[0], w.shape[1], **meta)
    if kind == "convt":
        return nn.ConvTranspose2d(w.shape[0], w.shape[1], w.shape[2], stride=w.shape[2], bias="bias" in t, **meta)
    if kind == "conv":
        return nn.Conv2d(w.shape[1], w.shape[0], w.shape[2], padding=w.shape[2] // 2, bias="bias" in t, **meta)
    if kind == "linear":
        return nn.Linear(w.shape[1], w.shape[0], bias="bias" in t, **meta)
    return nn.Module()


def attach_parameters(root: nn.Module, sd: Dict[str, torch.Tensor], prefix: str = "") -> None:
    """Create the module tree for every key of `sd` starting with `prefix` (relative to `root`) and
    register the tensors as its nn.Parameters.  Existing attributes on the path are reused."""
    groups: Dict[str, Dict[str, torch.Tensor]] = {}
    for key, t in sd.items():
        if not key.startswith(prefix):
            continue
        rel = key[len(prefix):]
        mod, _, name = rel.rpartition(".")
        groups.setdefault(mod, {})[name] = t
    # parents before children, so containers exist when a leaf is placed under them
    for mod in sorted(groups, key=lambda m: (m.count("."), m)):
        tensors = groups[mod]
        parent = root
        parts = mod.split(".") if mod else []
        for i, part in enumerate(parts):
            last = i == len(parts) - 1
            child = parent._modules.get(part)
            if child is None:
                child = _leaf(_kind(".".join(parts[: i + 1]), tensors), tensors) if last else nn.Module()
                parent.add_module(part, child)
            parent = child
        for name, t in tensors.items():
            if name in parent._parameters or hasattr(parent, name) and not isinstance(getattr(parent, name),
                                                                                       nn.Parameter):
                # drop a meta placeholder created by the torch module's constructor
                parent._parameters.pop(name, None)
            parent.register_parameter(name, nn.Parameter(t, requires_grad=True))
        # torch leaves created with parameters the state dict does not carry keep meta tensors: remove
        for name in list(parent._parameters):
            p = parent._parameters[name]
            if p is not None and p.device.type == "meta":
                parent._parameters[name] = None


def apply_clip_finetune(clip_model: nn.Module, mode: str) -> None:
    """requires_grad of the CLIP parameters as CATSeg.__init__ sets it (cat_seg_model.py:57-75):
    inside `transformer`: 'prompt' -> prompt params, 'attention' -> q_proj / v_proj weights of the
    attention blocks and positional parameters, 'full' -> all; everything outside `transformer` frozen."""
    for name, p in clip_model.named_parameters():
        if "transformer" in name:
            if mode == "prompt":
                p.requires_grad = "prompt" in name
            elif mode == "attention":
                if "attn" in name:
                    p.requires_grad = "q_proj" in name or "v_proj" in name
                elif "position" in name:
                    p.requires_grad = True
                else:
                    p.requires_grad = False
            elif mode == "full":
                p.requires_grad = True
            else:
                p.requires_grad = False
        else:
            p.requires_grad = False
