"""Deterministic synthetic weights under the reference's state-dict key names.

There is no network and no checkpoint here, so every parameter is synthesized
from `(seed, key)`: a per-key 63-bit seed (FNV-1a of the key mixed with the
run seed) feeds a CPU `torch.Generator`, so the same tensor comes out on every
host with this torch build.  Every tensor is non-trivial, including parameters
the reference zero-initialises (`padding_tokens`, `model.py:372-373`) or leaves
uninitialised (`positional_embedding`, `text_projection`, `model_vpt.py:393,396`),
so no branch of the path is degenerate.

Key names follow the module tree of a detectron2 `CATSeg` checkpoint
(`{"model": state_dict}`; tree printed in reference `vizDebug/log.txt:1446-1870`),
so a real checkpoint's state dict can replace the synthetic one unchanged.
"""
from __future__ import annotations

import math
from typing import Dict

import torch

from .arch import CatSegArch

CLIP = "sem_seg_head.predictor.clip_model."
AGG = "sem_seg_head.predictor.transformer."


def _key_seed(seed: int, key: str) -> int:
    h = 0xCBF29CE484222325
    for b in key.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    h ^= (seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    return h & 0x7FFFFFFFFFFFFFFF


def _uniform(seed: int, key: str, shape, lo: float, hi: float) -> torch.Tensor:
    g = torch.Generator().manual_seed(_key_seed(seed, key))
    return torch.rand(tuple(shape), generator=g, dtype=torch.float32) * (hi - lo) + lo


class _Synth:
    def __init__(self, seed: int):
        self.seed = seed
        self.sd: Dict[str, torch.Tensor] = {}

    def unit(self, key, shape, fan_in, gain=1.0):
        a = gain * math.sqrt(3.0 / fan_in)        # unit-variance-preserving uniform
        self.sd[key] = _uniform(self.seed, key, shape, -a, a)

    def const_noise(self, key, shape, center, amp):
        self.sd[key] = _uniform(self.seed, key, shape, center - amp, center + amp)

    def linear(self, prefix, n_out, n_in, bias=True, gain=1.0):
        self.unit(prefix + "weight", (n_out, n_in), n_in, gain)
        if bias:
            self.const_noise(prefix + "bias", (n_out,), 0.0, 0.1)

    def conv(self, prefix, c_out, c_in, k, bias=True, gain=1.0):
        self.unit(prefix + "weight", (c_out, c_in, k, k), c_in * k * k, gain)
        if bias:
            self.const_noise(prefix + "bias", (c_out,), 0.0, 0.1)

    def conv_t(self, prefix, c_in, c_out, k):
        # nn.ConvTranspose2d weight is (in, out, k, k); each output sees c_in inputs
        self.unit(prefix + "weight", (c_in, c_out, k, k), c_in)
        self.const_noise(prefix + "bias", (c_out,), 0.0, 0.1)

    def norm(self, prefix, c):
        self.const_noise(prefix + "weight", (c,), 1.0, 0.1)
        self.const_noise(prefix + "bias", (c,), 0.0, 0.1)


def _clip_block(s: _Synth, p: str, width: int):
    # model_vpt.py:169-200 Attention with split q/k/v weights + in_proj_bias
    for w in ("q", "k", "v"):
        s.unit(f"{p}attn.{w}_proj_weight", (width, width), width)
    s.const_noise(f"{p}attn.in_proj_bias", (3 * width,), 0.0, 0.1)
    s.linear(f"{p}attn.out_proj.", width, width, gain=0.5)
    s.norm(f"{p}ln_1.", width)
    s.linear(f"{p}mlp.c_fc.", 4 * width, width)
    s.linear(f"{p}mlp.c_proj.", width, 4 * width, gain=0.5)
    s.norm(f"{p}ln_2.", width)


def synthesize_state_dict(arch: CatSegArch, seed: int = 0) -> Dict[str, torch.Tensor]:
    s = _Synth(seed)
    a = arch
    # ---------------- CLIP visual (model_vpt.py:269-314) ----------------
    W = a.vision_width
    s.unit(CLIP + "visual.conv1.weight", (W, 3, a.vision_patch, a.vision_patch),
           3 * a.vision_patch * a.vision_patch)
    s.const_noise(CLIP + "visual.class_embedding", (W,), 0.0, 1.0)
    s.const_noise(CLIP + "visual.positional_embedding", (a.pretrain_grid ** 2 + 1, W), 0.0, 0.5)
    s.norm(CLIP + "visual.ln_pre.", W)
    for i in range(a.vision_layers):
        _clip_block(s, f"{CLIP}visual.transformer.resblocks.{i}.", W)
    if a.prompt_length > 0:          # Transformer.prompt_tokens (model_vpt.py:252), VPT only
        s.const_noise(CLIP + "visual.transformer.prompt_tokens", (a.prompt_depth, a.prompt_length, W), 0.0, 1.0)
    s.norm(CLIP + "visual.ln_post.", W)
    s.unit(CLIP + "visual.proj", (W, a.embed_dim), W)
    # ---------------- CLIP text (model_vpt.py:380-438) ----------------
    TW = a.text_width
    s.const_noise(CLIP + "token_embedding.weight", (a.vocab_size, TW), 0.0, 1.0)
    s.const_noise(CLIP + "positional_embedding", (a.context_length, TW), 0.0, 0.5)
    for i in range(a.text_layers):
        _clip_block(s, f"{CLIP}transformer.resblocks.{i}.", TW)
    s.norm(CLIP + "ln_final.", TW)
    s.unit(CLIP + "text_projection", (TW, a.embed_dim), TW)
    s.sd[CLIP + "logit_scale"] = torch.tensor(math.log(1 / 0.07))
    # ---------------- CATSeg upsamplers (cat_seg_model.py:81-82) ----------------
    s.conv_t("upsample1.", a.upsample_in_dim, a.decoder_guidance_dims[0], 2)
    s.conv_t("upsample2.", a.upsample_in_dim, a.decoder_guidance_dims[1], 4)
    # ---------------- Aggregator (model.py:602-634) ----------------
    D, G, TG = a.hidden_dim, a.appearance_guidance_proj_dim, a.text_guidance_proj_dim
    for l in range(a.num_layers):
        sw = f"{AGG}layers.{l}.swin_block."
        for blk in ("block_1", "block_2"):
            p = f"{sw}{blk}."
            s.norm(p + "norm1.", D)
            s.linear(p + "attn.q.", D, D + G)
            s.linear(p + "attn.k.", D, D + G)
            s.linear(p + "attn.v.", D, D)
            s.linear(p + "attn.proj.", D, D, gain=0.5)
            s.norm(p + "norm2.", D)
            s.linear(p + "mlp.fc1.", 4 * D, D)
            s.linear(p + "mlp.fc2.", D, 4 * D, gain=0.5)
        s.norm(sw + "guidance_norm.", G)
        ca = f"{AGG}layers.{l}.attention."
        s.linear(ca + "attention.q.", D, D + TG)
        s.linear(ca + "attention.k.", D, D + TG)
        s.linear(ca + "attention.v.", D, D)
        s.linear(ca + "MLP.0.", 4 * D, D)
        s.linear(ca + "MLP.2.", D, 4 * D, gain=0.5)
        s.norm(ca + "norm1.", D)
        s.norm(ca + "norm2.", D)
        if a.pad_len > 0:
            s.const_noise(ca + "padding_tokens", (1, 1, D), 0.0, 0.5)
            s.const_noise(ca + "padding_guidance", (1, 1, TG), 0.0, 0.5)
    s.conv(AGG + "conv1.", D, a.prompt_channel, 7)
    s.conv(AGG + "guidance_projection.0.", G, a.appearance_guidance_dim, 3)
    s.linear(AGG + "text_guidance_projection.0.", TG, a.text_guidance_dim)
    for i, (d, dp) in enumerate(zip(a.decoder_guidance_dims, a.decoder_guidance_proj_dims)):
        s.conv(f"{AGG}decoder_guidance_projection.{i}.0.", dp, d, 3)
    c_in = D
    for i, (c_out, gdim) in enumerate(zip(a.decoder_dims, a.decoder_guidance_proj_dims)):
        p = f"{AGG}decoder{i + 1}."
        s.conv_t(p + "up.", c_in, c_in - gdim, 2)
        s.conv(p + "conv.double_conv.0.", c_out, c_in, 3, bias=False)
        s.norm(p + "conv.double_conv.1.", c_out)
        s.conv(p + "conv.double_conv.3.", c_out, c_out, 3, bias=False)
        s.norm(p + "conv.double_conv.4.", c_out)
        c_in = c_out
    s.conv(AGG + "head.", 1, a.decoder_dims[1], 3)
    return s.sd
