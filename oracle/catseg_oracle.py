"""CPU oracle for the CAT-Seg dense-inference path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it.
It restates the reference algorithm in plain fp32 PyTorch on the CPU, using
the same unfused ATen ops the reference dispatches to, one function per
reference function, each citing the reference `file:line` it follows
(paths relative to the reference repo root).

Parity pin: `tests/golden/make_golden.py` imports the reference's own modules
(`cat_seg/third_party/model_vpt.py`, `cat_seg/modeling/transformer/model.py`)
in the build container, runs them on synthetic weights, and commits the
input/output vectors under `tests/golden/`; `tests/test_oracle_golden.py`
checks this restatement against them.  The detectron2 glue (`ImageList`,
`sem_seg_postprocess`) is not importable anywhere here and is restated from
`cat_seg/cat_seg_model.py:147-229`.

Weights are a flat dict under the reference checkpoint key names
(`cat_seg.weights`).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

CLIP = "sem_seg_head.predictor.clip_model."
AGG = "sem_seg_head.predictor.transformer."

Tensor = torch.Tensor


def _lin(x: Tensor, sd, p: str, bias: bool = True) -> Tensor:
    return F.linear(x, sd[p + "weight"], sd[p + "bias"] if bias else None)


def _ln(x: Tensor, sd, p: str, eps: float = 1e-5) -> Tensor:
    # model_vpt.py:156-162 (LayerNorm upcasts to fp32; a no-op in fp32)
    return F.layer_norm(x, (x.shape[-1],), sd[p + "weight"], sd[p + "bias"], eps)


# --------------------------------------------------------------------------
# CLIP (cat_seg/third_party/model_vpt.py)
# --------------------------------------------------------------------------
def mha(x: Tensor, sd, p: str, n_heads: int, attn_mask: Optional[Tensor] = None) -> Tensor:
    """nn.MultiheadAttention with split q/k/v weights (model_vpt.py:169-182,202-206).
    x: (L, N, D) sequence-first.  The `need_weights=True` head average is dead."""
    L, N, D = x.shape
    b = sd[p + "attn.in_proj_bias"]
    q = F.linear(x, sd[p + "attn.q_proj_weight"], b[:D])
    k = F.linear(x, sd[p + "attn.k_proj_weight"], b[D:2 * D])
    v = F.linear(x, sd[p + "attn.v_proj_weight"], b[2 * D:])
    hd = D // n_heads

    def heads(t):  # (L, N, D) -> (N*H, L, hd)
        return t.reshape(L, N * n_heads, hd).transpose(0, 1)

    q, k, v = heads(q) * (hd ** -0.5), heads(k), heads(v)
    s = torch.bmm(q, k.transpose(1, 2))
    if attn_mask is not None:
        s = s + attn_mask
    a = torch.softmax(s, dim=-1)
    o = torch.bmm(a, v).transpose(0, 1).reshape(L, N, D)
    return _lin(o, sd, p + "attn.out_proj.")


def quick_gelu(x: Tensor) -> Tensor:
    return x * torch.sigmoid(1.702 * x)          # model_vpt.py:165-167


def resblock(x: Tensor, sd, p: str, n_heads: int, attn_mask=None) -> Tensor:
    """ResidualAttentionBlock.forward (model_vpt.py:208-217)."""
    x = x + mha(_ln(x, sd, p + "ln_1."), sd, p, n_heads, attn_mask)
    h = quick_gelu(_lin(_ln(x, sd, p + "ln_2."), sd, p + "mlp.c_fc."))
    return x + _lin(h, sd, p + "mlp.c_proj.")


def resblock_dense(x: Tensor, sd, p: str) -> Tensor:
    """ResidualAttentionBlock.forward_dense (model_vpt.py:219-240): the v path only,
    out_proj applied to v, residual = the input CLS token broadcast over tokens."""
    D = x.shape[-1]
    y = _ln(x, sd, p + "ln_1.")
    v = F.linear(y, sd[p + "attn.v_proj_weight"], sd[p + "attn.in_proj_bias"][2 * D:])
    v = _lin(v, sd, p + "attn.out_proj.")
    v = v + x[:1]
    h = quick_gelu(_lin(_ln(v, sd, p + "ln_2."), sd, p + "mlp.c_fc."))
    return v + _lin(h, sd, p + "mlp.c_proj.")


def resized_pos_embed(pos: Tensor, in_side: int, tgt_side: int) -> Tensor:
    """VisualTransformer.resized_pos_embed (model_vpt.py:316-329), bicubic."""
    D = pos.shape[1]
    grid = pos[1:].reshape(1, in_side, in_side, D).permute(0, 3, 1, 2)
    grid = F.interpolate(grid, size=(tgt_side, tgt_side), mode="bicubic", align_corners=False)
    return torch.cat([pos[:1], grid.squeeze(0).reshape(D, -1).T], dim=0)


def encode_image_dense(arch, sd, img: Tensor) -> Tuple[Tensor, List[Tensor]]:
    """CLIP.encode_image(dense=True) -> VisualTransformer.forward (model_vpt.py:288-314,
    413-419) plus the forward hooks CATSeg registers (cat_seg_model.py:84-87).
    img: (B,3,R,R) normalized.  Returns (features (B,1+HW,C_o), [hook (L,B,W)]*2)."""
    p = CLIP + "visual."
    x = F.conv2d(img, sd[p + "conv1.weight"], stride=arch.vision_patch)
    B, W = x.shape[:2]
    x = x.reshape(B, W, -1).permute(0, 2, 1)
    cls = sd[p + "class_embedding"] + torch.zeros(B, 1, W)
    x = torch.cat([cls, x], dim=1)
    pos = sd[p + "positional_embedding"]
    if x.shape[1] != pos.shape[0]:
        pos = resized_pos_embed(pos, arch.pretrain_grid, int(math.sqrt(x.shape[1] - 1)))
    x = _ln(x + pos, sd, p + "ln_pre.")
    x = x.permute(1, 0, 2)
    hooks = []
    P = getattr(arch, "prompt_length", 0)
    for i in range(arch.vision_layers):
        bp = f"{p}transformer.resblocks.{i}."
        if P > 0 and i < arch.prompt_depth:      # Transformer.forward (model_vpt.py:258-259): after CLS
            pt = sd[p + "transformer.prompt_tokens"][i].unsqueeze(1).expand(P, x.shape[1], -1)
            x = torch.cat([x[:1], pt, x[1:]], dim=0)
        if i == arch.vision_layers - 1:
            x = resblock_dense(x, sd, bp)
        else:
            x = resblock(x, sd, bp, arch.vision_heads)
        if P > 0:                                # every block drops rows 1..P (model_vpt.py:213-214,238-239)
            x = torch.cat([x[:1], x[P + 1:]], dim=0)
        if i in arch.hook_layers:
            hooks.append(x)
    x = _ln(x.permute(1, 0, 2), sd, p + "ln_post.")
    return x @ sd[p + "proj"], hooks


def encode_text(arch, sd, tokens: Tensor) -> Tensor:
    """CLIP.encode_text (model_vpt.py:421-438) with the causal mask (:400-406)."""
    x = sd[CLIP + "token_embedding.weight"][tokens] + sd[CLIP + "positional_embedding"]
    n = x.shape[1]
    mask = torch.full((n, n), float("-inf")).triu_(1)
    x = x.permute(1, 0, 2)
    for i in range(arch.text_layers):
        x = resblock(x, sd, f"{CLIP}transformer.resblocks.{i}.", arch.text_heads, mask)
    x = _ln(x.permute(1, 0, 2), sd, CLIP + "ln_final.")
    x = x[torch.arange(x.shape[0]), tokens.argmax(dim=-1)]
    return x @ sd[CLIP + "text_projection"]


def text_embeds(arch, sd, tokens: Tensor) -> Tensor:
    """CATSegPredictor.get_text_embeds (cat_seg_predictor.py:190-224): L2-normalized,
    (T, 1, C_o) for the single-template prompt."""
    e = encode_text(arch, sd, tokens)
    e = e / e.norm(dim=-1, keepdim=True)
    return e.unsqueeze(1)


# --------------------------------------------------------------------------
# Aggregator (cat_seg/modeling/transformer/model.py)
# --------------------------------------------------------------------------
def window_partition(x: Tensor, ws: int) -> Tensor:      # model.py:18-30
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(-1, ws, ws, C)


def window_reverse(w: Tensor, ws: int, H: int, W: int) -> Tensor:   # model.py:33-47
    B = w.shape[0] // ((H // ws) * (W // ws))
    x = w.view(B, H // ws, W // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(B, H, W, -1)


def shift_mask(H: int, W: int, ws: int, shift: int) -> Tensor:
    """SW-MSA region mask, -100 across regions (model.py:161-183)."""
    img = torch.zeros(1, H, W, 1)
    cnt = 0
    bands = ((0, H - ws), (H - ws, H - shift), (H - shift, H))
    for h0, h1 in bands:
        for w0, w1 in ((0, W - ws), (W - ws, W - shift), (W - shift, W)):
            img[:, h0:h1, w0:w1, :] = cnt
            cnt += 1
    mw = window_partition(img, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return torch.where(m != 0, torch.tensor(-100.0), torch.tensor(0.0))


def window_attention(x: Tensor, sd, p: str, dim: int, nheads: int, mask) -> Tensor:
    """WindowAttention.forward (model.py:86-114); q,k from [x||guid], v from x only."""
    B_, N, _ = x.shape
    hd = dim // nheads
    q = _lin(x, sd, p + "q.").reshape(B_, N, nheads, hd).permute(0, 2, 1, 3)
    k = _lin(x, sd, p + "k.").reshape(B_, N, nheads, hd).permute(0, 2, 1, 3)
    v = _lin(x[:, :, :dim], sd, p + "v.").reshape(B_, N, nheads, hd).permute(0, 2, 1, 3)
    a = (q * hd ** -0.5) @ k.transpose(-2, -1)
    if mask is not None:
        nw = mask.shape[0]
        a = (a.view(B_ // nw, nw, nheads, N, N) + mask.unsqueeze(1).unsqueeze(0)).view(-1, nheads, N, N)
    a = torch.softmax(a, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B_, N, -1)
    return _lin(o, sd, p + "proj.")


def swin_block(x: Tensor, guid: Tensor, sd, p: str, arch, shift: int) -> Tensor:
    """SwinTransformerBlock.forward (model.py:185-225).  x: (B', HW, C)."""
    H, W = arch.feature_resolution
    ws = arch.window_size
    if min(H, W) <= ws:                    # model.py:146-149
        shift, ws = 0, min(H, W)
    B_, L, C = x.shape
    short = x
    x = _ln(x, sd, p + "norm1.").view(B_, H, W, C)
    x = torch.cat([x, guid.view(B_, H, W, -1)], dim=-1)
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    xw = window_partition(x, ws).view(-1, ws * ws, x.shape[-1])
    mask = shift_mask(H, W, ws, shift) if shift > 0 else None
    aw = window_attention(xw, sd, p + "attn.", C, arch.nheads, mask)
    x = window_reverse(aw.view(-1, ws, ws, C), ws, H, W)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    x = short + x.reshape(B_, H * W, C)
    h = F.gelu(_lin(_ln(x, sd, p + "norm2."), sd, p + "mlp.fc1."))     # timm Mlp, exact GELU
    return x + _lin(h, sd, p + "mlp.fc2.")


def swin_wrapper(x: Tensor, guid: Tensor, sd, p: str, arch) -> Tensor:
    """SwinTransformerBlockWrapper.forward (model.py:239-253).  x: (B,C,T,H,W),
    guid: (B,C,H,W)."""
    B, C, T, H, W = x.shape
    x = x.permute(0, 2, 3, 4, 1).reshape(B * T, H * W, C)
    g = guid.permute(0, 2, 3, 1).reshape(B, 1, H * W, -1).expand(B, T, H * W, -1)
    g = _ln(g.reshape(B * T, H * W, -1), sd, p + "guidance_norm.")
    x = swin_block(x, g, sd, p + "block_1.", arch, 0)
    x = swin_block(x, g, sd, p + "block_2.", arch, arch.window_size // 2)
    return x.reshape(B, T, H, W, C).permute(0, 4, 1, 2, 3)


def elu1(x: Tensor) -> Tensor:
    return F.elu(x) + 1                              # model.py:256-257


def linear_attention(q: Tensor, k: Tensor, v: Tensor, eps: float = 1e-6) -> Tensor:
    """LinearAttention.forward (model.py:266-286).  q,k,v: (N, L, H, D)."""
    Q, K = elu1(q), elu1(k)
    S = v.size(1)
    v = v / S
    KV = torch.einsum("nshd,nshv->nhdv", K, v)
    Z = 1 / (torch.einsum("nlhd,nhd->nlh", Q, K.sum(dim=1)) + eps)
    return torch.einsum("nlhd,nhdv,nlh->nlhv", Q, KV, Z) * S


def full_attention(q: Tensor, k: Tensor, v: Tensor) -> Tensor:
    """FullAttention.forward (model.py:300-320), no masks, no dropout at eval.  q,k,v: (N, L, H, D)."""
    QK = torch.einsum("nlhd,nshd->nlsh", q, k)
    A = torch.softmax(QK / q.size(3) ** .5, dim=2)
    return torch.einsum("nlsh,nshd->nlhd", A, v)


def class_layer(x: Tensor, tguid: Tensor, sd, p: str, arch) -> Tensor:
    """ClassTransformerLayer.forward (model.py:387-424).  x: (B,C,T,H,W), tguid (B,T,C')."""
    B, C, T, H, W = x.shape
    ph, pw = arch.pooling_size
    xp = F.avg_pool2d(x.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W), (ph, pw))
    Hp, Wp = xp.shape[-2:]
    xp = xp.reshape(B, T, C, Hp, Wp).permute(0, 2, 1, 3, 4)
    pad = arch.pad_len > 0 and T < arch.pad_len
    if pad:
        npad = arch.pad_len - T
        pt = sd[p + "padding_tokens"].reshape(1, C, 1, 1, 1).expand(B, C, npad, Hp, Wp)
        xp = torch.cat([xp, pt], dim=2)
        pg = sd[p + "padding_guidance"].reshape(1, 1, -1).expand(B, npad, -1)
        tguid = torch.cat([tguid, pg], dim=1)
    L = xp.shape[2]
    xp = xp.permute(0, 3, 4, 2, 1).reshape(B * Hp * Wp, L, C)
    g = tguid.unsqueeze(1).expand(B, Hp * Wp, L, -1).reshape(B * Hp * Wp, L, -1)
    nh = arch.nheads
    xn = _ln(xp, sd, p + "norm1.")
    ap = p + "attention."
    q = _lin(torch.cat([xn, g], -1), sd, ap + "q.").reshape(-1, L, nh, C // nh)
    k = _lin(torch.cat([xn, g], -1), sd, ap + "k.").reshape(-1, L, nh, C // nh)
    v = _lin(xn, sd, ap + "v.").reshape(-1, L, nh, C // nh)
    attn = full_attention if getattr(arch, "attention_type", "linear") == "full" else linear_attention
    xp = xp + attn(q, k, v).reshape(-1, L, C)           # AttentionLayer (model.py:331-334,352)
    h = F.relu(_lin(_ln(xp, sd, p + "norm2."), sd, p + "MLP.0."))
    xp = xp + _lin(h, sd, p + "MLP.2.")
    xp = xp.reshape(B, Hp, Wp, L, C).permute(0, 3, 4, 1, 2).reshape(B * L, C, Hp, Wp)
    xp = F.interpolate(xp, size=(H, W), mode="bilinear", align_corners=True)
    xp = xp.reshape(B, L, C, H, W).permute(0, 2, 1, 3, 4)
    if pad:
        xp = xp[:, :, :T]
    return x + xp


def _conv(x, sd, p, bias=True, pad=1):
    return F.conv2d(x, sd[p + "weight"], sd[p + "bias"] if bias else None, padding=pad)


def up_block(x: Tensor, guid: Optional[Tensor], sd, p: str) -> Tensor:
    """Up + DoubleConv (model.py:520-555)."""
    x = F.conv_transpose2d(x, sd[p + "up.weight"], sd[p + "up.bias"], stride=2)
    if guid is not None:
        T = x.shape[0] // guid.shape[0]
        x = torch.cat([x, guid.repeat_interleave(T, dim=0)], dim=1)
    dc = p + "conv.double_conv."
    for a, n in (("0.", "1."), ("3.", "4.")):
        x = _conv(x, sd, dc + a, bias=False)
        c = x.shape[1]
        x = F.relu(F.group_norm(x, c // 16, sd[dc + n + "weight"], sd[dc + n + "bias"], 1e-5))
    return x


def aggregator(arch, sd, img_feats: Tensor, text_feats: Tensor, guidance: Sequence[Tensor],
               classes: Optional[Tensor] = None) -> Tensor:
    """Aggregator.forward (model.py:683-725).  img_feats (B,C,H,W), text (B,T,P,C),
    guidance [res3, res4, res5].  `classes` (B, pad_len) int64, test use only: replaces the
    top-k selection of model.py:694-697 by a caller-supplied one (the classes the HIP path
    selected), so everything downstream of the selection is checked at full tolerance when
    bf16 rounding reorders near-tied classes; None = the reference's own top-k."""
    p = AGG
    imgn = F.normalize(img_feats, dim=1)
    txtn = F.normalize(text_feats, dim=-1)
    corr = torch.einsum("bchw,btpc->bpthw", imgn, txtn)            # model.py:648-652
    T0 = text_feats.shape[1]
    if arch.pad_len > 0 and T0 > arch.pad_len:                       # model.py:694-702
        if classes is None:
            m = corr.permute(0, 2, 1, 3, 4).flatten(-3).max(dim=-1)[0]
            classes = m.topk(arch.pad_len, dim=-1, sorted=False)[1]
        classes = classes.long()
        idx = classes[..., None, None].expand(-1, -1, txtn.shape[-2], txtn.shape[-1])
        txtn = torch.gather(txtn, 1, idx)
        text_feats = txtn
        corr = torch.einsum("bchw,btpc->bpthw", imgn, txtn)
    B, P, T, H, W = corr.shape
    x = _conv(corr.permute(0, 2, 1, 3, 4).reshape(B * T, P, H, W), sd, p + "conv1.", pad=3)
    x = x.reshape(B, T, -1, H, W).permute(0, 2, 1, 3, 4)            # model.py:654-659
    g3 = F.relu(_conv(guidance[0], sd, p + "guidance_projection.0."))
    gd = [F.relu(_conv(g, sd, f"{p}decoder_guidance_projection.{i}.0."))
          for i, g in enumerate(guidance[1:])]
    t = text_feats.mean(dim=-2)
    t = t / t.norm(dim=-1, keepdim=True)
    tg = F.relu(_lin(t, sd, p + "text_guidance_projection.0."))      # model.py:706-715
    for l in range(arch.num_layers):
        lp = f"{p}layers.{l}."
        x = swin_wrapper(x, g3, sd, lp + "swin_block.", arch)
        x = class_layer(x, tg, sd, lp + "attention.", arch)
    y = x.permute(0, 2, 1, 3, 4).reshape(B * T, -1, H, W)           # model.py:674-681
    y = up_block(y, gd[0], sd, p + "decoder1.")
    y = up_block(y, gd[1], sd, p + "decoder2.")
    y = _conv(y, sd, p + "head.")
    logit = y.reshape(B, T, y.shape[-2], y.shape[-1])
    if classes is not None:                                          # model.py:721-724
        out = torch.full((B, T0, logit.shape[-2], logit.shape[-1]), -100.0)
        out.scatter_(1, classes[..., None, None].expand(-1, -1, logit.shape[-2], logit.shape[-1]), logit)
        logit = out
    return logit


# --------------------------------------------------------------------------
# CATSeg meta-arch glue (cat_seg/cat_seg_model.py) + detectron2 restatements
# --------------------------------------------------------------------------
def image_list_pad(imgs: List[Tensor], div: int) -> Tuple[Tensor, List[Tuple[int, int]]]:
    """detectron2 ImageList.from_tensors: zero-pad bottom/right to the batch max,
    rounded up to `div` (call sites cat_seg_model.py:140,152)."""
    sizes = [(int(i.shape[-2]), int(i.shape[-1])) for i in imgs]
    H = max(s[0] for s in sizes)
    W = max(s[1] for s in sizes)
    if div > 1:
        H = (H + div - 1) // div * div
        W = (W + div - 1) // div * div
    out = imgs[0].new_zeros(len(imgs), imgs[0].shape[0], H, W)
    for i, im in enumerate(imgs):
        out[i, :, : im.shape[-2], : im.shape[-1]] = im
    return out, sizes


def sem_seg_postprocess(result: Tensor, img_size, out_h: int, out_w: int) -> Tensor:
    """detectron2 sem_seg_postprocess (call sites cat_seg_model.py:217,227)."""
    result = result[:, : img_size[0], : img_size[1]].expand(1, -1, -1, -1)
    return F.interpolate(result, size=(out_h, out_w), mode="bilinear", align_corners=False)[0]


def head_logits(arch, sd, clip_images: Tensor, text: Tensor, classes: Optional[Tensor] = None) -> Tensor:
    """cat_seg_model.py:155-188 + CATSegHead/Predictor (cat_seg_head.py:2009-2010,
    cat_seg_predictor.py:151-162).  clip_images (B,3,R,R) normalized+resized,
    text (T,1,C_o) cached embeddings.  Returns logits (B,T,96,96).  `classes`: see aggregator."""
    feats, hooks = encode_image_dense(arch, sd, clip_images)
    B = clip_images.shape[0]
    g = arch.grid
    res3 = feats[:, 1:, :].reshape(B, g, g, -1).permute(0, 3, 1, 2)
    res4 = hooks[0][1:].permute(1, 2, 0).reshape(B, -1, g, g)
    res5 = hooks[1][1:].permute(1, 2, 0).reshape(B, -1, g, g)
    res4 = F.conv_transpose2d(res4, sd["upsample1.weight"], sd["upsample1.bias"], stride=2)
    res5 = F.conv_transpose2d(res5, sd["upsample2.weight"], sd["upsample2.bias"], stride=4)
    text_b = text.unsqueeze(0).expand(B, -1, -1, -1)
    return aggregator(arch, sd, res3, text_b, [res3, res4, res5], classes=classes)


def class_corr_max(arch, sd, clip_images: Tensor, text: Tensor) -> Tensor:
    """Per-image, per-class max of the fp32 cost volume over (P, H, W): the top-k key of
    model.py:694-697 (correlation model.py:648-652).  Returns (B, T)."""
    with torch.no_grad():
        feats, _ = encode_image_dense(arch, sd, clip_images)
        B, g = clip_images.shape[0], arch.grid
        img = F.normalize(feats[:, 1:, :].reshape(B, g, g, -1).permute(0, 3, 1, 2), dim=1)
        txt = F.normalize(text.unsqueeze(0).expand(B, -1, -1, -1), dim=-1)
        corr = torch.einsum("bchw,btpc->bpthw", img, txt)
        return corr.permute(0, 2, 1, 3, 4).flatten(2).max(dim=-1)[0]


def preprocess(arch, images: List[Tensor]) -> Tuple[Tensor, List[Tuple[int, int]]]:
    """cat_seg_model.py:149-154: normalize, ImageList pad /32, bilinear resize."""
    mean = torch.tensor(arch.clip_pixel_mean).view(-1, 1, 1)
    std = torch.tensor(arch.clip_pixel_std).view(-1, 1, 1)
    norm = [(x.float() - mean) / std for x in images]
    padded, sizes = image_list_pad(norm, arch.size_divisibility)
    R = arch.clip_resolution
    return F.interpolate(padded, size=(R, R), mode="bilinear", align_corners=False), sizes


def catseg_forward(arch, sd, batched_inputs: List[dict], text: Tensor, all_images: bool = False):
    """CATSeg.forward, eval, non-sliding (cat_seg_model.py:147-155,178-188,220-229).
    The reference returns image 0 only; `all_images=True` returns every image
    (the batched boundary's behaviour)."""
    with torch.no_grad():
        clip_images, sizes = preprocess(arch, [x["image"] for x in batched_inputs])
        logits = head_logits(arch, sd, clip_images, text).sigmoid()
        n = len(batched_inputs) if all_images else 1
        out = []
        for i in range(n):
            h = batched_inputs[i].get("height", sizes[i][0])
            w = batched_inputs[i].get("width", sizes[i][1])
            out.append({"sem_seg": sem_seg_postprocess(logits[i], sizes[i], h, w)})
        return out


def sliding_clip_images(arch, image: Tensor) -> Tensor:
    """The 5 crops of the sliding-window branch, normalized and resized (cat_seg_model.py:158-176)."""
    kernel, overlap, out_res = 384, 0.333, [640, 640]
    stride = int(kernel * (1 - overlap))
    img = image.float()
    unfold = torch.nn.Unfold(kernel_size=kernel, stride=stride)
    x = F.interpolate(img.unsqueeze(0), size=out_res, mode="bilinear", align_corners=False).squeeze()
    x = unfold(x).reshape(3, kernel, kernel, -1).permute(3, 0, 1, 2)
    glob = F.interpolate(img.unsqueeze(0), size=(kernel, kernel), mode="bilinear", align_corners=False)
    x = torch.cat([x, glob], dim=0)
    mean = torch.tensor(arch.clip_pixel_mean).view(-1, 1, 1)
    std = torch.tensor(arch.clip_pixel_std).view(-1, 1, 1)
    R = arch.clip_resolution
    return F.interpolate((x - mean) / std, size=(R, R), mode="bilinear", align_corners=False)


def catseg_forward_sliding(arch, sd, batched_inputs: List[dict], text: Tensor, classes: Optional[Tensor] = None):
    """CATSeg.forward sliding-window branch (cat_seg_model.py:156-176,204-218).
    `classes` (5, pad_len): per-crop top-k override, see aggregator."""
    kernel, overlap, out_res = 384, 0.333, [640, 640]
    stride = int(kernel * (1 - overlap))
    with torch.no_grad():
        img = batched_inputs[0]["image"].float()
        unfold = torch.nn.Unfold(kernel_size=kernel, stride=stride)
        fold = torch.nn.Fold(out_res, kernel_size=kernel, stride=stride)
        image = F.interpolate(img.unsqueeze(0), size=out_res, mode="bilinear", align_corners=False).squeeze()
        image = unfold(image).reshape(3, kernel, kernel, -1).permute(3, 0, 1, 2)
        glob = F.interpolate(img.unsqueeze(0), size=(kernel, kernel), mode="bilinear", align_corners=False)
        image = torch.cat([image, glob], dim=0)
        mean = torch.tensor(arch.clip_pixel_mean).view(-1, 1, 1)
        std = torch.tensor(arch.clip_pixel_std).view(-1, 1, 1)
        R = arch.clip_resolution
        clip_images = F.interpolate((image - mean) / std, size=(R, R), mode="bilinear", align_corners=False)
        outputs = head_logits(arch, sd, clip_images, text, classes=classes)
        outputs = F.interpolate(outputs, size=kernel, mode="bilinear", align_corners=False).sigmoid()
        glob_out = F.interpolate(outputs[-1:], size=out_res, mode="bilinear", align_corners=False)
        outputs = outputs[:-1]
        outputs = fold(outputs.flatten(1).T) / fold(unfold(torch.ones([1] + out_res)))
        outputs = (outputs + glob_out) / 2.0
        h = batched_inputs[0].get("height", out_res[0])
        w = batched_inputs[0].get("width", out_res[1])
        return [{"sem_seg": sem_seg_postprocess(outputs[0], out_res, h, w)}]
