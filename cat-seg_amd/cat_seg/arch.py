"""Architecture description of the CAT-Seg dense-inference path.

One frozen record (`CatSegArch`) carries every shape the HIP path and the
oracle need.  It is derived from the same config keys the reference reads:

* CLIP geometry from the pretrained name, as `clip.load` + `build_model` would
  produce it (reference `cat_seg/third_party/model_vpt.py:482-532`,
  `cat_seg/third_party/clip.py:19-31`).
* `CATSeg` constants: clip resolution, upsampler input width, hook indices
  (`cat_seg/cat_seg_model.py:78-87`).
* `Aggregator` kwargs (`cat_seg/modeling/transformer/cat_seg_predictor.py:97-113`,
  defaults `cat_seg/modeling/transformer/model.py:559-576`).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Tuple


@dataclass(frozen=True)
class CatSegArch:
    # ---- CLIP vision tower (model_vpt.py:269-314) ----
    vision_width: int
    vision_layers: int
    vision_patch: int
    vision_pretrain_res: int          # image_resolution of the checkpoint (pos-embed grid)
    embed_dim: int                    # CLIP output dim C_o (visual.proj columns)
    # ---- CLIP text tower (model_vpt.py:380-438) ----
    text_width: int
    text_layers: int
    context_length: int = 77
    vocab_size: int = 49408
    # ---- CATSeg meta-arch (cat_seg_model.py:78-87) ----
    clip_resolution: int = 384
    hook_layers: Tuple[int, int] = (3, 7)
    # ---- Aggregator (model.py:559-634) ----
    hidden_dim: int = 128
    nheads: int = 4
    num_layers: int = 2
    pooling_size: Tuple[int, int] = (1, 1)
    feature_resolution: Tuple[int, int] = (24, 24)
    window_size: int = 12
    text_guidance_proj_dim: int = 128
    appearance_guidance_proj_dim: int = 128
    decoder_dims: Tuple[int, int] = (64, 32)
    decoder_guidance_dims: Tuple[int, int] = (256, 128)
    decoder_guidance_proj_dims: Tuple[int, int] = (32, 16)
    prompt_channel: int = 1
    pad_len: int = 256
    # ClassTransformerLayer attention (model.py:324-334): "linear" (LinearAttention, every shipped
    # config) or "full" (FullAttention, softmax over the padded class axis)
    attention_type: str = "linear"
    # ---- visual prompt tuning (model_vpt.py:243-265): PROMPT_LENGTH learned tokens per layer joined
    # after CLS for the first PROMPT_DEPTH vision blocks (cat_seg_predictor.py:76, clip.load) ----
    prompt_depth: int = 0
    prompt_length: int = 0
    # ---- image preprocessing (config.py:36,67-68) ----
    size_divisibility: int = 32
    clip_pixel_mean: Tuple[float, float, float] = (122.7709383, 116.7460125, 104.09373615)
    clip_pixel_std: Tuple[float, float, float] = (68.5005327, 66.6321579, 70.3231630)
    name: str = "custom"

    # derived -------------------------------------------------------------
    @property
    def vision_heads(self) -> int:
        return self.vision_width // 64          # model_vpt.py:368

    @property
    def text_heads(self) -> int:
        return self.text_width // 64            # model_vpt.py:504

    @property
    def grid(self) -> int:
        return self.clip_resolution // self.vision_patch

    @property
    def pretrain_grid(self) -> int:
        return self.vision_pretrain_res // self.vision_patch

    @property
    def n_tokens(self) -> int:
        return self.grid * self.grid + 1

    @property
    def vpt(self) -> int:
        """Prompt rows per vision sequence (0: no visual prompt tuning)."""
        return self.prompt_length if self.prompt_length > 0 and self.prompt_depth > 0 else 0

    @property
    def text_guidance_dim(self) -> int:
        return self.embed_dim

    @property
    def appearance_guidance_dim(self) -> int:
        return self.embed_dim

    @property
    def upsample_in_dim(self) -> int:
        # cat_seg_model.py:80 hard-codes 768 (B/16) / 1024 (L/14) = vision width
        return self.vision_width

    def replace(self, **kw) -> "CatSegArch":
        return dataclasses.replace(self, **kw)


# ViT-B/16 as loaded by clip.load("ViT-B/16"): pretrain 224 -> 14x14 grid, resized to 24x24
VIT_B16 = CatSegArch(
    vision_width=768, vision_layers=12, vision_patch=16, vision_pretrain_res=224,
    embed_dim=512, text_width=512, text_layers=12,
    clip_resolution=384, hook_layers=(3, 7), name="ViT-B/16")

# ViT-L/14@336px: pretrain 336 -> 24x24 grid, no pos-embed resize
VIT_L14_336 = CatSegArch(
    vision_width=1024, vision_layers=24, vision_patch=14, vision_pretrain_res=336,
    embed_dim=768, text_width=768, text_layers=12,
    clip_resolution=336, hook_layers=(7, 15), name="ViT-L/14@336px")

# Small geometry for fast tests: same aggregator, narrow CLIP (not a reference model).
TINY = CatSegArch(
    vision_width=128, vision_layers=4, vision_patch=16, vision_pretrain_res=224,
    embed_dim=96, text_width=64, text_layers=2, context_length=16, vocab_size=512,
    clip_resolution=384, hook_layers=(1, 2), name="tiny")

PRESETS = {"ViT-B/16": VIT_B16, "ViT-L/14@336px": VIT_L14_336, "tiny": TINY}


def arch_from_cfg(cfg) -> CatSegArch:
    """Build the arch from a detectron2/yacs-style cfg (attribute access)."""
    head = cfg.MODEL.SEM_SEG_HEAD
    base = PRESETS[head.CLIP_PRETRAINED]
    return base.replace(
        hidden_dim=int(head.HIDDEN_DIMS),
        nheads=int(head.NUM_HEADS),
        num_layers=int(head.NUM_LAYERS),
        pooling_size=tuple(int(p) for p in head.POOLING_SIZES),
        feature_resolution=tuple(int(p) for p in head.FEATURE_RESOLUTION),
        window_size=int(head.WINDOW_SIZES),
        attention_type=str(getattr(head, "ATTENTION_TYPE", "linear")),
        prompt_depth=int(getattr(head, "PROMPT_DEPTH", 0)),
        prompt_length=int(getattr(head, "PROMPT_LENGTH", 0)),
        text_guidance_proj_dim=int(head.TEXT_GUIDANCE_PROJ_DIM),
        appearance_guidance_proj_dim=int(head.APPEARANCE_GUIDANCE_PROJ_DIM),
        decoder_dims=tuple(head.DECODER_DIMS),
        decoder_guidance_dims=tuple(head.DECODER_GUIDANCE_DIMS),
        decoder_guidance_proj_dims=tuple(head.DECODER_GUIDANCE_PROJ_DIMS),
        size_divisibility=int(cfg.MODEL.MASK_FORMER.SIZE_DIVISIBILITY),
        clip_pixel_mean=tuple(cfg.MODEL.CLIP_PIXEL_MEAN),
        clip_pixel_std=tuple(cfg.MODEL.CLIP_PIXEL_STD),
    )
