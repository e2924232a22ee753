"""The training step's aggregation head with a HIP backward.

`head_train_forward` runs the reference's training-mode head (cat_seg_model.py:178-188 ->
CATSegHead -> Aggregator.forward, model.py:683-725) on fp32 device tensors and returns logits
carrying an autograd graph whose every node is a `torch.autograd.Function` backed by the HIP
kernels of libcatseg_hip.so (forward: catseg_hip.h, backward: catseg_hip_train.h):

  ConvTUpsample   CATSeg.upsample1/2 ConvTranspose2d (cat_seg_model.py:81-82,184-185)
  CostVolume      Aggregator.correlation (model.py:648-652)
  CorrEmbed       conv1 7x7 (model.py:613,654-659)
  Conv3x3         guidance projections + ReLU (model.py:615-630,706-711)
  L2Norm / Linear text guidance (model.py:712-715)
  LayerNormRows   guidance_norm (model.py:233,249)
  SwinBlock       SwinTransformerBlock (model.py:117-225) with WindowAttention (model.py:51-114)
  ClassLayer      ClassTransformerLayer (model.py:357-424) with LinearAttention (model.py:256-286)
  UpBlock         Up + DoubleConv (model.py:520-555)
  HeadConv        head conv3x3 (model.py:634,679)

Forward saves what the backward reads (the intermediate activations of each block, fp32); the
window / linear attention backward kernels recompute their probabilities from q / k / v.
Parameters are the reference-shaped nn.Parameters of cat_seg.params (nn.Linear weight
[out][in], Conv2d (co, ci, k, k), ConvTranspose2d (ci, co, k, k)); each Function derives the kernel
layouts from them per call (small weight reshapes) and returns gradients in the reference shapes,
so torch autograd accumulates them into `.grad` and any torch optimizer sees them.

Everything is fp32 — the reference trains in fp32 — and deterministic (no atomics anywhere).
Layouts: rows X[(b*T + t)*HW + p][128] as in the engine; NHWC maps; logits [B][T][h][w].
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _lib as L
from . import ops, train_ops as TO
from ._lib import rowmap
from .arch import CatSegArch
from .weights import AGG

_f32 = torch.float32


def _empty(*shape, like):
    return torch.empty(*shape, device=like.device, dtype=_f32)


def _c(t):
    return t.contiguous() if t is not None else None


def _mm_t(dy, x, out=None, beta=0):
    """dW = dy^T . x over rows: dy [R][N], x [R][K] -> [N][K] (catseg_gemm_ex, K = R split)."""
    R, N = dy.shape
    K = x.shape[1]
    if out is None:
        out = _empty(N, K, like=dy)
    return TO.gemm_ex(dy, 1, dy.stride(0), x, x.stride(0), 1, out, M=N, N=K, K=R, beta=beta)


def _colsum(x, out=None, beta=0):
    if out is None:
        out = _empty(x.shape[1], like=x)
    return TO.colsum(x, out, beta=beta)


def _conv_w(w):        # Conv2d (co, ci, k, k) -> [(tap, ci)][co]
    co, ci, k, _ = w.shape
    return w.detach().permute(2, 3, 1, 0).reshape(k * k * ci, co).contiguous()


def _conv_w_flip(w):   # the data-gradient weight: [(tap, co)][ci] of the flipped kernel
    co, ci, k, _ = w.shape
    return w.detach().flip(2, 3).permute(2, 3, 0, 1).reshape(k * k * co, ci).contiguous()


def _conv_dw(dw, w):   # [(tap, ci)][co] -> (co, ci, k, k)
    co, ci, k, _ = w.shape
    return dw.reshape(k, k, ci, co).permute(3, 2, 0, 1).contiguous()


def _convt_w(w):       # ConvTranspose2d (ci, co, k, k) -> [(ky, kx, co)][ci]
    ci, co, k, _ = w.shape
    return w.detach().permute(2, 3, 1, 0).reshape(k * k * co, ci).contiguous()


def _convt_dw(dwg, w):
    ci, co, k, _ = w.shape
    return dwg.reshape(k, k, co, ci).permute(3, 2, 0, 1).contiguous()


def _qkv_split(qw, qb, kw, kb, vw, vb, D):
    """[q | k | v] x-half weights [3D][D] + bias [3D], and the guidance halves of q, k [2D][Dg]
    (q, k = Linear(D + Dg -> D) on [x | guidance], v = Linear(D -> D) on x; model.py:94-96, 344-346)."""
    wx = torch.cat([qw.detach()[:, :D], kw.detach()[:, :D], vw.detach()], 0).contiguous()
    bx = torch.cat([qb.detach(), kb.detach(), vb.detach()]).contiguous()
    wg = torch.cat([qw.detach()[:, D:], kw.detach()[:, D:]], 0).contiguous()
    return wx, bx, wg


def _qkv_grads(dwx, dbx, dwg, D):
    dqw = torch.cat([dwx[:D], dwg[:D]], 1)
    dkw = torch.cat([dwx[D:2 * D], dwg[D:]], 1)
    return dqw, dbx[:D], dkw, dbx[D:2 * D], dwx[2 * D:].contiguous(), dbx[2 * D:]


def _add_cls_rows(d, B, HW):
    """[B*HW][C] token-row gradients -> [B*(1+HW)][C] with zero CLS rows (the backward of dropping CLS)."""
    out = torch.zeros(B * (HW + 1), d.shape[1], device=d.device, dtype=_f32)
    for b in range(B):
        ops.convert(d[b * HW:(b + 1) * HW], out[b * (HW + 1) + 1:(b + 1) * (HW + 1)])
    return out


# ------------------------------------------------------------------------------------- small blocks
class DropClsFn(torch.autograd.Function):
    """image_features = clip_features[:, 1:, :] (cat_seg_model.py:178): [B*(1+HW)][C] -> [B*HW][C]."""

    @staticmethod
    def forward(ctx, feats, HW):
        feats = feats.contiguous()
        B = feats.shape[0] // (HW + 1)
        out = _empty(B * HW, feats.shape[1], like=feats)
        ops.convert(feats, out, inmap=rowmap(d1=HW, s1=HW + 1, d2=1, m2=HW, s2=1, off=1))
        ctx.geo = (B, HW)
        return out

    @staticmethod
    def backward(ctx, d):
        B, HW = ctx.geo
        return _add_cls_rows(d.contiguous(), B, HW), None



class LinearFn(torch.autograd.Function):
    """y = act(x . W^T + b) (nn.Linear [+ ReLU]): catseg_gemm forward, catseg_gemm_ex / colsum backward."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x = x.contiguous()
        y = _empty(x.shape[0], w.shape[0], like=x)
        ops.gemm(x, w.detach().contiguous(), y, bias=b.detach().contiguous(), act=act)
        ctx.act = act
        ctx.save_for_backward(x, w, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == L.ACT_RELU:
            dy = TO.act_backward(y, dy, L.ACT_RELU)
        dx = TO.mm(dy, w.detach().contiguous()) if ctx.needs_input_grad[0] else None
        return dx, _mm_t(dy, x), _colsum(dy), None


class L2NormFn(torch.autograd.Function):
    """F.normalize over the last dim (model.py:649-650,714)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        ops.l2normalize(x, y)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        TO.l2normalize_backward(x, dy.contiguous(), dx, rows=x.shape[0], cols=x.shape[1])
        return dx


class LayerNormRowsFn(torch.autograd.Function):
    """nn.LayerNorm over rows (guidance_norm, model.py:233,249; applied once per image — the
    reference's repeat over classes is summed back by the consumers' backward)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x = x.contiguous()
        y = torch.empty_like(x)
        ops.layernorm(x, w.detach(), b.detach(), y)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = torch.empty_like(x)
        dw = _empty(x.shape[1], like=x)
        db = torch.empty_like(dw)
        TO.layernorm_backward(x, w.detach(), dy.contiguous(), dx, dgamma=dw, dbeta=db)
        return dx, dw, db


class ConvTUpsampleFn(torch.autograd.Function):
    """CATSeg.upsample1/2: ConvTranspose2d(k, stride k) on the hook tokens without CLS
    (cat_seg_model.py:81-82,182-185).  hook [B*(1+G^2)][Wv] -> NHWC [B*(kG)^2][co]."""

    @staticmethod
    def forward(ctx, hook, w, b, G):
        hook = hook.contiguous()
        ci, co, k, _ = w.shape
        HW = G * G
        B = hook.shape[0] // (HW + 1)
        drop_cls = rowmap(d1=HW, s1=HW + 1, d2=1, m2=HW, s2=1, off=1)
        xh = _empty(B * HW, ci, like=hook)
        ops.convert(hook, xh, inmap=drop_cls)
        wg = _convt_w(w)
        out = _empty(B * HW * k * k, co, like=hook)
        ops.gemm(xh, wg, out, bias=b.detach().repeat(k * k).contiguous(), store=(k, G, G, co))
        ctx.save_for_backward(xh, w)
        ctx.geo = (B, G)
        return out

    @staticmethod
    def backward(ctx, dout):
        xh, w = ctx.saved_tensors
        B, G = ctx.geo
        ci, co, k, _ = w.shape
        HW = G * G
        g = _empty(B * HW, k * k * co, like=xh)
        TO.convt_gather(dout.contiguous(), g, S=B, hin=G, win=G, k=k, cout=co)
        dw = _convt_dw(_mm_t(g, xh), w)
        db = _empty(co, like=xh)
        TO.colsum(g, db, rows=B * HW * k * k, cols=co, ld=co)
        dhook = _add_cls_rows(TO.mm(g, _convt_w(w)), B, HW) if ctx.needs_input_grad[0] else None
        return dhook, dw, db, None


class CostVolumeFn(torch.autograd.Function):
    """Aggregator.correlation (model.py:648-652): corr[b][t][p] = <normalize(img[b, :, p]),
    normalize(text[t])>, img = the dense CLIP tokens without CLS.  feats [B*(1+HW)][Co],
    text [T][Co] -> corr [B][T][HW]."""

    @staticmethod
    def forward(ctx, feats, text, HW):
        feats, text = feats.contiguous(), text.contiguous()
        B = feats.shape[0] // (HW + 1)
        T, Co = text.shape
        drop_cls = rowmap(d1=HW, s1=HW + 1, d2=1, m2=HW, s2=1, off=1)
        fn = _empty(B * HW, Co, like=feats)
        ops.l2normalize(feats, fn, inmap=drop_cls)
        txn = torch.empty_like(text)
        ops.l2normalize(text, txn)
        corr = _empty(B, T, HW, like=feats)
        for b in range(B):
            ops.gemm(txn, fn[b * HW:(b + 1) * HW], corr[b])
        ctx.save_for_backward(feats, text, fn, txn)
        ctx.HW = HW
        return corr

    @staticmethod
    def backward(ctx, dcorr):
        feats, text, fn, txn = ctx.saved_tensors
        HW = ctx.HW
        B = feats.shape[0] // (HW + 1)
        T, Co = text.shape
        dcorr = dcorr.contiguous()
        dfeats = dtext = None
        if ctx.needs_input_grad[0]:
            dfn = _empty(B * HW, Co, like=feats)
            for b in range(B):      # d fn[b] = dcorr[b]^T . txn
                TO.gemm_ex(dcorr[b], 1, HW, txn, Co, 1, dfn[b * HW:(b + 1) * HW], M=HW, N=Co, K=T)
            dfeats = torch.zeros_like(feats)
            m = rowmap(d1=HW, s1=HW + 1, d2=1, m2=HW, s2=1, off=1)
            TO.l2normalize_backward(feats, dfn, dfeats, rows=B * HW, cols=Co, inmap=m, outmap=m)
        if ctx.needs_input_grad[1]:
            dtxn = _empty(T, Co, like=text)
            for b in range(B):      # d txn = sum_b dcorr[b] . fn[b]
                TO.gemm_ex(dcorr[b], HW, 1, fn[b * HW:(b + 1) * HW], Co, 1, dtxn, M=T, N=Co, K=HW, beta=int(b > 0))
            dtext = torch.empty_like(text)
            TO.l2normalize_backward(text, dtxn, dtext, rows=T, cols=Co)
        return dfeats, dtext, None


class CorrEmbedFn(torch.autograd.Function):
    """Aggregator.corr_embed: Conv2d(1, D, 7, pad 3) per (image, class) cost slice (model.py:654-659).
    corr [B][T][G*G] -> X rows [B*T*G*G][D]."""

    @staticmethod
    def forward(ctx, corr, w, b, G):
        corr = corr.contiguous()
        B, T, HW = corr.shape
        D = w.shape[0]
        X = _empty(B * T * HW, D, like=corr)
        ops.corr_embed(corr, t_stride=HW, b_stride=T * HW, B=B, T=T, H=G, W=G,
                       weight=w.detach().reshape(D, -1).contiguous(), bias=b.detach().contiguous(), out=X)
        ctx.save_for_backward(corr, w)
        ctx.G = G
        return X

    @staticmethod
    def backward(ctx, dX):
        corr, w = ctx.saved_tensors
        G = ctx.G
        B, T, HW = corr.shape
        D, _, k, _ = w.shape
        dX = dX.contiguous()
        dw = _empty(k * k, D, like=corr)
        TO.conv2d_wgrad(corr.reshape(-1, 1), dX, dw, S=B * T, H=G, W=G, cin=1, cout=D, ksize=k, ld_x=1)
        dcorr = None
        if ctx.needs_input_grad[0]:
            dcorr = torch.empty_like(corr)
            TO.corr_embed_backward_input(dX, w.detach().contiguous(), dcorr, S=B * T, H=G, W=G)
        return dcorr, _conv_dw(dw, w), _colsum(dX), None


class Conv3x3Fn(torch.autograd.Function):
    """relu(Conv2d(x) + b) over NHWC rows [S*H*W][ci] (guidance projections, model.py:615-630)."""

    @staticmethod
    def forward(ctx, x, w, b, S, H, W):
        x = x.contiguous()
        co, ci, k, _ = w.shape
        y = _empty(S * H * W, co, like=x)
        TO.conv2d(x, _conv_w(w), y, S=S, H=H, W=W, cin=ci, cout=co, ksize=k, bias=b.detach().contiguous(),
                  act=L.ACT_RELU)
        ctx.save_for_backward(x, w, y)
        ctx.geo = (S, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        S, H, W = ctx.geo
        co, ci, k, _ = w.shape
        d = TO.act_backward(y, dy.contiguous(), L.ACT_RELU)
        dw = _empty(k * k * ci, co, like=x)
        TO.conv2d_wgrad(x, d, dw, S=S, H=H, W=W, cin=ci, cout=co, ksize=k)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            TO.conv2d(d, _conv_w_flip(w), dx, S=S, H=H, W=W, cin=co, cout=ci, ksize=k)
        return dx, _conv_dw(dw, w), _colsum(d), None, None, None


# ------------------------------------------------------------------------------------- Swin block
@dataclass
class Geo:
    B: int
    T: int
    H: int
    W: int
    nh: int


class SwinBlockFn(torch.autograd.Function):
    """SwinTransformerBlock.forward (model.py:185-225): x' = x + proj(W-MSA(LN1(x) | guidance));
    out = x' + fc2(GELU(fc1(LN2(x')))).  X rows [B*T*HW][D]; gn = guidance_norm(guidance) per image
    [B*HW][Dg] (the reference repeats it over T, model.py:249: its gradient is summed over T)."""

    @staticmethod
    def forward(ctx, X, gn, geo, ws, shift, n1w, n1b, qw, qb, kw, kb, vw, vb, pw, pb, n2w, n2b, w1, b1, w2, b2):
        X, gn = X.contiguous(), gn.contiguous()
        R, D = X.shape
        HW = geo.H * geo.W
        wx, bx, wg = _qkv_split(qw, qb, kw, kb, vw, vb, D)
        h = torch.empty_like(X)
        ops.layernorm(X, n1w.detach(), n1b.detach(), h)
        gqk = _empty(gn.shape[0], 2 * D, like=X)
        ops.gemm(gn, wg, gqk)
        qkv = _empty(R, 3 * D, like=X)
        ops.gemm(h, wx, qkv, bias=bx, add=gqk, addmap=rowmap(d1=geo.T * HW, s1=HW, d2=1, m2=HW, s2=1), add_ncols=2 * D)
        o = torch.empty_like(X)
        nwin = (geo.H // ws) * (geo.W // ws)
        hd = D // geo.nh
        ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, n_seq=(R // HW) * nwin, seq_len=ws * ws,
                      n_heads=geo.nh, head_dim=hd, scale=hd ** -0.5, mode=1, img_hw=(geo.H, geo.W), window=ws,
                      shift=shift)
        x1 = torch.empty_like(X)
        ops.gemm(o, pw.detach().contiguous(), x1, bias=pb.detach().contiguous(), res=X)
        h2 = torch.empty_like(X)
        ops.layernorm(x1, n2w.detach(), n2b.detach(), h2)
        u = _empty(R, w1.shape[0], like=X)
        ops.gemm(h2, w1.detach().contiguous(), u, bias=b1.detach().contiguous())
        a = TO.act_forward(u, L.ACT_GELU)
        out = torch.empty_like(X)
        ops.gemm(a, w2.detach().contiguous(), out, bias=b2.detach().contiguous(), res=x1)
        ctx.save_for_backward(X, gn, h, qkv, o, x1, h2, u, a, n1w, n2w, qw, kw, vw, pw, w1, w2, qb, kb, vb)
        ctx.cfg = (geo, ws, shift)
        return out

    @staticmethod
    def backward(ctx, dout):
        (X, gn, h, qkv, o, x1, h2, u, a, n1w, n2w, qw, kw, vw, pw, w1, w2, qb, kb, vb) = ctx.saved_tensors
        geo, ws, shift = ctx.cfg
        R, D = X.shape
        HW = geo.H * geo.W
        dout = dout.contiguous()
        # MLP: out = x1 + fc2(GELU(fc1(LN2(x1))))
        dw2, db2 = _mm_t(dout, a), _colsum(dout)
        du = TO.mm(dout, w2.detach(), act_u=u, act=L.ACT_GELU)      # GELU backward in the epilogue
        dw1, db1 = _mm_t(du, h2), _colsum(du)
        dh2 = TO.mm(du, w1.detach())
        del du
        dx1 = dout.clone()
        dn2w, dn2b = _empty(D, like=X), _empty(D, like=X)
        TO.layernorm_backward(x1, n2w.detach(), dh2, dx1, acc_dx=True, dgamma=dn2w, dbeta=dn2b)
        # x1 = X + proj(o)
        dpw, dpb = _mm_t(dx1, o), _colsum(dx1)
        do = TO.mm(dx1, pw.detach())
        hd = D // geo.nh
        dqkv = _empty(R, 3 * D, like=X)
        TO.window_attention_backward(qkv, o, do, dqkv, S=R // HW, img_hw=(geo.H, geo.W), window=ws, shift=shift,
                                     n_heads=geo.nh, head_dim=hd, scale=hd ** -0.5)
        del do
        wx, _, wg = _qkv_split(qw, qb, kw, kb, vw, vb, D)
        dwx, dbx = _mm_t(dqkv, h), _colsum(dqkv)
        dh = TO.mm(dqkv, wx)
        dX = dx1
        dn1w, dn1b = _empty(D, like=X), _empty(D, like=X)
        TO.layernorm_backward(X, n1w.detach(), dh, dX, acc_dx=True, dgamma=dn1w, dbeta=dn1b)
        # guidance halves of q, k: sum over the classes the guidance was repeated over
        dqk = _empty(gn.shape[0], 2 * D, like=X)
        TO.sum_classes(dqkv, dqk, B=geo.B, T=geo.T, HW=HW, C_=2 * D)
        dwg = _mm_t(dqk, gn)
        dgn = TO.mm(dqk, wg) if ctx.needs_input_grad[1] else None
        dqw, dqb, dkw, dkb, dvw, dvb = _qkv_grads(dwx, dbx, dwg, D)
        return (dX, dgn, None, None, None, dn1w, dn1b, dqw, dqb, dkw, dkb, dvw, dvb, dpw, dpb, dn2w, dn2b,
                dw1, db1, dw2, db2)


# ------------------------------------------------------------------------------------- class layer
class ClassLayerFn(torch.autograd.Function):
    """ClassTransformerLayer.forward (model.py:387-424): x_pool = AvgPool(x), padded with the learned
    padding token / guidance to pad_len classes (model.py:397-410); x_pool += LinearAttn(LN1(x_pool),
    text guidance); x_pool += MLP(LN2(x_pool)); x + bilinear_align_corners(x_pool) cropped to T.
    X rows [B*T*HW][D], tg [T][Dt] (text_guidance_projection output, shared by the images)."""

    @staticmethod
    def forward(ctx, X, tg, geo, pool, pad_len, n1w, n1b, qw, qb, kw, kb, vw, vb, n2w, n2b, w0, b0, w2, b2,
                pad_tok, pad_guid):
        X, tg = X.contiguous(), tg.contiguous()
        R, D = X.shape
        ph, pw_ = pool
        pooled = (ph, pw_) != (1, 1)
        Hp, Wp = geo.H // ph, geo.W // pw_
        HWc = Hp * Wp
        S = geo.B * geo.T
        Rp = S * HWc
        if pooled:
            Xp = _empty(Rp, D, like=X)
            ops.avgpool_rows(X, Xp, S=S, H=geo.H, W=geo.W, C=D, pool=pool)
        else:
            Xp = X
        wx, bx, wt = _qkv_split(qw, qb, kw, kb, vw, vb, D)
        h = torch.empty_like(Xp)
        ops.layernorm(Xp, n1w.detach(), n1b.detach(), h)
        tgqk = _empty(geo.T, 2 * D, like=X)
        ops.gemm(tg, wt, tgqk)
        qkv = _empty(Rp, 3 * D, like=X)
        ops.gemm(h, wx, qkv, bias=bx, add=tgqk, addmap=rowmap(d1=HWc, m1=geo.T), add_ncols=2 * D)
        n_pad = pad_len - geo.T if pad_len > 0 and geo.T < pad_len else 0
        hp = kvp = None
        if n_pad:
            pt = pad_tok.detach().reshape(1, D).contiguous()
            hp = _empty(1, D, like=X)
            ops.layernorm(pt, n1w.detach(), n1b.detach(), hp)
            pg = _empty(1, 2 * D, like=X)
            ops.gemm(pad_guid.detach().reshape(1, -1).contiguous(), wt, pg)
            kvp = _empty(1, 3 * D, like=X)
            ops.gemm(hp, wx, kvp, bias=bx, add=pg, add_ncols=2 * D)
        y = torch.empty_like(Xp)
        kp = kvp[0, D:2 * D].contiguous() if n_pad else None
        vp = kvp[0, 2 * D:].contiguous() if n_pad else None
        ops.linear_attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], Xp, y, B=geo.B, T=geo.T, HW=HWc,
                             n_heads=geo.nh, head_dim=D // geo.nh, n_pad=n_pad, k_pad=kp, v_pad=vp)
        h2 = torch.empty_like(y)
        ops.layernorm(y, n2w.detach(), n2b.detach(), h2)
        u = _empty(Rp, w0.shape[0], like=X)
        ops.gemm(h2, w0.detach().contiguous(), u, bias=b0.detach().contiguous())
        a = TO.act_forward(u, L.ACT_RELU)
        if pooled:
            yo = torch.empty_like(y)
            ops.gemm(a, w2.detach().contiguous(), yo, bias=b2.detach().contiguous(), res=y)
            out = X.clone()
            ops.upsample_add_rows(yo, out, S=S, Hp=Hp, Wp=Wp, C=D, H=geo.H, W=geo.W)
        else:
            out = torch.empty_like(X)
            ops.gemm(a, w2.detach().contiguous(), out, bias=b2.detach().contiguous(), res=y, res2=X)
        ctx.save_for_backward(Xp, tg, h, qkv, y, h2, u, a, hp, kp, vp, n1w, n2w, qw, kw, vw, qb, kb, vb, w0, w2,
                              pad_tok, pad_guid)
        ctx.cfg = (geo, pool, n_pad, pooled)
        return out

    @staticmethod
    def backward(ctx, dout):
        (Xp, tg, h, qkv, y, h2, u, a, hp, kp, vp, n1w, n2w, qw, kw, vw, qb, kb, vb, w0, w2, pad_tok,
         pad_guid) = ctx.saved_tensors
        geo, pool, n_pad, pooled = ctx.cfg
        Rp, D = Xp.shape
        ph, pw_ = pool
        Hp, Wp = geo.H // ph, geo.W // pw_
        HWc = Hp * Wp
        S = geo.B * geo.T
        dout = dout.contiguous()
        if pooled:
            dyo = _empty(Rp, D, like=dout)
            TO.upsample_ac_backward_rows(dout, dyo, S=S, H=geo.H, W=geo.W, C_=D, Hp=Hp, Wp=Wp)
        else:
            dyo = dout
        # MLP: yo = y + MLP.2(ReLU(MLP.0(LN2(y))))
        dw2, db2 = _mm_t(dyo, a), _colsum(dyo)
        du = TO.mm(dyo, w2.detach(), act_u=u, act=L.ACT_RELU)
        dw0, db0 = _mm_t(du, h2), _colsum(du)
        dh2 = TO.mm(du, w0.detach())
        del du
        dy = dyo.clone()
        dn2w, dn2b = _empty(D, like=Xp), _empty(D, like=Xp)
        TO.layernorm_backward(y, n2w.detach(), dh2, dy, acc_dx=True, dgamma=dn2w, dbeta=dn2b)
        # y = Xp + LinearAttention(q, k, v)
        dqkv = _empty(Rp, 3 * D, like=Xp)
        dkp = dvp = None
        if n_pad:
            dkp, dvp = _empty(D, like=Xp), _empty(D, like=Xp)
        TO.linear_attention_backward(qkv, dy, dqkv, B=geo.B, T=geo.T, HW=HWc, n_heads=geo.nh, head_dim=D // geo.nh,
                                     n_pad=n_pad, k_pad=kp, v_pad=vp, dk_pad=dkp, dv_pad=dvp)
        wx, _, wt = _qkv_split(qw, qb, kw, kb, vw, vb, D)
        dwx, dbx = _mm_t(dqkv, h), _colsum(dqkv)
        dh = TO.mm(dqkv, wx)
        dXp = dy
        dn1w, dn1b = _empty(D, like=Xp), _empty(D, like=Xp)
        TO.layernorm_backward(Xp, n1w.detach(), dh, dXp, acc_dx=True, dgamma=dn1w, dbeta=dn1b)
        # text-guidance halves of q, k: broadcast over images and pixels
        dtqk = _empty(geo.T, 2 * D, like=Xp)
        TO.sum_pixels(dqkv, dtqk, B=geo.B, T=geo.T, HW=HWc, C_=2 * D)
        dwt = _mm_t(dtqk, tg)
        dtg = TO.mm(dtqk, wt) if ctx.needs_input_grad[1] else None
        dpad_tok = dpad_guid = None
        if n_pad:
            # the padding tokens' k, v: kvp = LN1(pad_tok) . wx^T + bx (+ pad_guid . wt^T on k)
            dkvp = torch.zeros(1, 3 * D, device=Xp.device, dtype=_f32)
            dkvp[0, D:2 * D] = dkp
            dkvp[0, 2 * D:] = dvp
            _mm_t(dkvp, hp, out=dwx, beta=1)
            TO.colsum(dkvp, dbx, beta=1)
            pg = pad_guid.detach().reshape(1, -1).contiguous()
            _mm_t(dkvp[:, :2 * D], pg, out=dwt, beta=1)
            dpad_guid = TO.mm(dkvp[:, :2 * D], wt).reshape(pad_guid.shape)
            dhp = TO.mm(dkvp, wx)
            dpt = _empty(1, D, like=Xp)
            TO.layernorm_backward(pad_tok.detach().reshape(1, D).contiguous(), n1w.detach(), dhp, dpt,
                                  dgamma=dn1w, dbeta=dn1b, acc_param=True)
            dpad_tok = dpt.reshape(pad_tok.shape)
        # out = X + U(yo) (pooled: U = align-corners upsample of the pooled grid; else out = X + yo)
        if pooled:
            dX = dout.clone()
            TO.avgpool_backward_rows(dXp, dX, S=S, H=geo.H, W=geo.W, C_=D, pool=pool, beta=1)
        else:
            dX = TO.axpby(dXp, dout, dXp)
        dqw, dqb, dkw, dkb, dvw, dvb = _qkv_grads(dwx, dbx, dwt, D)
        return (dX, dtg, None, None, None, dn1w, dn1b, dqw, dqb, dkw, dkb, dvw, dvb, dn2w, dn2b, dw0, db0, dw2, db2,
                dpad_tok, dpad_guid)


# ------------------------------------------------------------------------------------- decoder
class UpBlockFn(torch.autograd.Function):
    """Up.forward + DoubleConv (model.py:520-555): u = ConvT(x) (k=2, s=2); [u | guidance repeated
    over T] -> conv3x3 -> GN -> ReLU -> conv3x3 -> GN -> ReLU.  x NHWC [S*h*h][ci], gd [B*(2h)^2][cg]
    -> [S*(2h)^2][cout]."""

    @staticmethod
    def forward(ctx, x, gd, geo, h, up_w, up_b, c0w, g1w, g1b, c3w, g4w, g4b):
        x, gd = x.contiguous(), gd.contiguous()
        ci, cu, k, _ = up_w.shape
        cg = gd.shape[1]
        cout = c0w.shape[0]
        S = geo.B * geo.T
        H2 = 2 * h
        P2 = H2 * H2
        u = _empty(S * P2, cu, like=x)
        ops.gemm(x, _convt_w(up_w), u, bias=up_b.detach().repeat(4).contiguous(), store=(2, h, h, cu))
        cat = _empty(S * P2, cu + cg, like=x)
        ops.convert(u, cat[:, :cu])
        ops.convert(gd, cat[:, cu:], inmap=rowmap(d1=geo.T * P2, s1=P2, d2=1, m2=P2, s2=1))
        del u
        c1 = _empty(S * P2, cout, like=x)
        TO.conv2d(cat, _conv_w(c0w), c1, S=S, H=H2, W=H2, cin=cu + cg, cout=cout)
        G = cout // 16
        m1, r1 = _empty(S * G, like=x), _empty(S * G, like=x)
        TO.groupnorm_stats_rows(c1, S, P2, cout, 16, m1, r1)
        n1 = torch.empty_like(c1)
        ops.groupnorm_relu(c1, n1, S=S, HW=P2, C=cout, cpg=16, mean=m1, rstd=r1, gamma=g1w.detach(), beta=g1b.detach())
        c2 = torch.empty_like(c1)
        TO.conv2d(n1, _conv_w(c3w), c2, S=S, H=H2, W=H2, cin=cout, cout=cout)
        m2, r2 = _empty(S * G, like=x), _empty(S * G, like=x)
        TO.groupnorm_stats_rows(c2, S, P2, cout, 16, m2, r2)
        n2 = torch.empty_like(c2)
        ops.groupnorm_relu(c2, n2, S=S, HW=P2, C=cout, cpg=16, mean=m2, rstd=r2, gamma=g4w.detach(), beta=g4b.detach())
        ctx.save_for_backward(x, cat, c1, n1, c2, m1, r1, m2, r2, up_w, c0w, g1w, g1b, c3w, g4w, g4b)
        ctx.cfg = (geo, h)
        return n2

    @staticmethod
    def backward(ctx, dn2):
        x, cat, c1, n1, c2, m1, r1, m2, r2, up_w, c0w, g1w, g1b, c3w, g4w, g4b = ctx.saved_tensors
        geo, h = ctx.cfg
        ci, cu, k, _ = up_w.shape
        cout = c0w.shape[0]
        ccat = cat.shape[1]
        cg = ccat - cu
        S = geo.B * geo.T
        H2 = 2 * h
        P2 = H2 * H2
        dn2 = dn2.contiguous()
        # second conv + GN + ReLU
        dc2 = torch.empty_like(c2)
        dg4w, dg4b = _empty(cout, like=x), _empty(cout, like=x)
        TO.groupnorm_relu_backward(c2, dn2, dc2, S=S, HW=P2, C_=cout, cpg=16, mean=m2, rstd=r2, gamma=g4w.detach(),
                                   beta=g4b.detach(), dgamma=dg4w, dbeta=dg4b)
        dw3 = _empty(9 * cout, cout, like=x)
        TO.conv2d_wgrad(n1, dc2, dw3, S=S, H=H2, W=H2, cin=cout, cout=cout)
        dn1 = torch.empty_like(c1)
        TO.conv2d(dc2, _conv_w_flip(c3w), dn1, S=S, H=H2, W=H2, cin=cout, cout=cout)
        del dc2
        # first conv + GN + ReLU (over the concat [u | guidance])
        dc1 = dn1
        dg1w, dg1b = _empty(cout, like=x), _empty(cout, like=x)
        TO.groupnorm_relu_backward(c1, dn1, dc1, S=S, HW=P2, C_=cout, cpg=16, mean=m1, rstd=r1, gamma=g1w.detach(),
                                   beta=g1b.detach(), dgamma=dg1w, dbeta=dg1b)
        dw0 = _empty(9 * ccat, cout, like=x)
        TO.conv2d_wgrad(cat, dc1, dw0, S=S, H=H2, W=H2, cin=ccat, cout=cout)
        dcat = torch.empty_like(cat)
        TO.conv2d(dc1, _conv_w_flip(c0w), dcat, S=S, H=H2, W=H2, cin=cout, cout=ccat)
        del dc1
        dgd = None
        if ctx.needs_input_grad[1]:
            dgd = _empty(geo.B * P2, cg, like=x)
            TO.sum_classes(dcat[:, cu:], dgd, B=geo.B, T=geo.T, HW=P2, C_=cg)
        # ConvTranspose (k = s = 2)
        g = _empty(S * h * h, 4 * cu, like=x)
        TO.convt_gather(dcat, g, S=S, hin=h, win=h, k=2, cout=cu, ld=ccat)
        del dcat
        dup_w = _convt_dw(_mm_t(g, x), up_w)
        dup_b = _empty(cu, like=x)
        TO.colsum(g, dup_b, rows=S * h * h * 4, cols=cu, ld=cu)
        dx = TO.mm(g, _convt_w(up_w)) if ctx.needs_input_grad[0] else None
        return (dx, dgd, None, None, dup_w, dup_b, _conv_dw(dw0, c0w), dg1w, dg1b, _conv_dw(dw3, c3w), dg4w, dg4b)


class HeadConvFn(torch.autograd.Function):
    """head: Conv2d(C, 1, 3, pad 1) + bias (model.py:634,679).  x NHWC [B*T*h*w][C] -> logits [B][T][h][w]."""

    @staticmethod
    def forward(ctx, x, w, b, geo, hw):
        x = x.contiguous()
        C = w.shape[1]
        logits = _empty(geo.B, geo.T, hw, hw, like=x)
        wt = w.detach()[0].permute(1, 2, 0).reshape(9 * C).contiguous()       # [ky][kx][c]
        ops.conv3x3_head(x, B=geo.B, T=geo.T, H=hw, W=hw, C=C, weight=wt, bias=0.0, out=logits, T_out=geo.T)
        TO.add_dev_scalar(logits, b.detach().reshape(1).contiguous())
        ctx.save_for_backward(x, wt, w)
        ctx.cfg = (geo, hw)
        return logits

    @staticmethod
    def backward(ctx, dl):
        x, wt, w = ctx.saved_tensors
        geo, hw = ctx.cfg
        C = w.shape[1]
        S = geo.B * geo.T
        dl = dl.contiguous()
        dx = torch.empty_like(x)
        dwt = _empty(9, C, like=x)
        TO.head_conv_backward(x, dl, wt.reshape(9, C), dx, dwt, S=S, H=hw, W=hw, C_=C)
        db = _empty(1, like=x)
        TO.colsum(dl.reshape(-1, 1), db, rows=dl.numel(), cols=1, ld=1)
        return dx, dwt.reshape(3, 3, C).permute(2, 0, 1).reshape(w.shape).contiguous(), db.reshape(1), None, None


# ------------------------------------------------------------------------------------- CLIP encoders
def _ln_bwd(x, w, dh, dx, need_param, acc_dx=True):
    """LayerNorm backward into dx (accumulated); the parameter gradients only when asked for."""
    if need_param:
        dw, db = _empty(x.shape[1], like=x), _empty(x.shape[1], like=x)
        TO.layernorm_backward(x, w.detach(), dh, dx, acc_dx=acc_dx, dgamma=dw, dbeta=db)
        return dw, db
    TO.layernorm_backward(x, w.detach(), dh, dx, acc_dx=acc_dx)
    return None, None


class ClipBlockFn(torch.autograd.Function):
    """ResidualAttentionBlock.forward (model_vpt.py:208-217): x1 = x + out_proj(MHA(ln_1(x))) with split
    q/k/v weights + in_proj_bias (model_vpt.py:169-182), x2 = x1 + c_proj(QuickGELU(c_fc(ln_2(x1)))).
    Rows [n_seq*L][W] token-major per sequence; causal = the text encoder's mask (model_vpt.py:400-406).
    Every parameter's gradient is computed only when autograd asks for it (CLIP_FINETUNE 'attention'
    trains the q / v projections only, cat_seg_model.py:57-75)."""

    @staticmethod
    def forward(ctx, x, cfg, ln1w, ln1b, qw, kw, vw, ipb, ow, ob, ln2w, ln2b, fcw, fcb, pw, pb):
        n_seq, L_, nh, causal = cfg
        x = x.contiguous()
        R, W = x.shape
        h = torch.empty_like(x)
        ops.layernorm(x, ln1w.detach(), ln1b.detach(), h)
        wqkv = torch.cat([qw.detach(), kw.detach(), vw.detach()], 0).contiguous()
        qkv = _empty(R, 3 * W, like=x)
        ops.gemm(h, wqkv, qkv, bias=ipb.detach().contiguous())
        o = torch.empty_like(x)
        hd = W // nh
        ops.attention(qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:], o, n_seq=n_seq, seq_len=L_, n_heads=nh,
                      head_dim=hd, scale=hd ** -0.5, causal=causal)
        x1 = torch.empty_like(x)
        ops.gemm(o, ow.detach().contiguous(), x1, bias=ob.detach().contiguous(), res=x)
        h2 = torch.empty_like(x)
        ops.layernorm(x1, ln2w.detach(), ln2b.detach(), h2)
        u = _empty(R, fcw.shape[0], like=x)
        ops.gemm(h2, fcw.detach().contiguous(), u, bias=fcb.detach().contiguous())
        a = TO.act_forward(u, L.ACT_QUICKGELU)
        out = torch.empty_like(x)
        ops.gemm(a, pw.detach().contiguous(), out, bias=pb.detach().contiguous(), res=x1)
        ctx.save_for_backward(x, h, qkv, o, x1, h2, u, a, ln1w, qw, kw, vw, ow, ln2w, fcw, pw)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, dout):
        x, h, qkv, o, x1, h2, u, a, ln1w, qw, kw, vw, ow, ln2w, fcw, pw = ctx.saved_tensors
        n_seq, L_, nh, causal = ctx.cfg
        ni = ctx.needs_input_grad
        R, W = x.shape
        dout = dout.contiguous()
        g = [None] * 16
        if ni[14]:
            g[14] = _mm_t(dout, a)
        if ni[15]:
            g[15] = _colsum(dout)
        du = TO.mm(dout, pw.detach(), act_u=u, act=L.ACT_QUICKGELU)
        if ni[12]:
            g[12] = _mm_t(du, h2)
        if ni[13]:
            g[13] = _colsum(du)
        dh2 = TO.mm(du, fcw.detach())
        del du
        dx1 = dout.clone()
        g[10], g[11] = _ln_bwd(x1, ln2w, dh2, dx1, ni[10] or ni[11])
        if ni[8]:
            g[8] = _mm_t(dx1, o)
        if ni[9]:
            g[9] = _colsum(dx1)
        do = TO.mm(dx1, ow.detach())
        hd = W // nh
        dqkv = _empty(R, 3 * W, like=x)
        TO.attention_backward(qkv, o, do, dqkv, n_seq=n_seq, seq_len=L_, n_heads=nh, head_dim=hd, scale=hd ** -0.5,
                              causal=causal)
        del do
        for i, j in ((4, 0), (5, 1), (6, 2)):
            if ni[i]:
                g[i] = _mm_t(dqkv[:, j * W:(j + 1) * W], h)
        if ni[7]:
            g[7] = _colsum(dqkv)
        if ni[0] or ni[2] or ni[3]:    # not for the first block of a frozen embedding: nothing reads dx there
            dh = TO.mm(dqkv, torch.cat([qw.detach(), kw.detach(), vw.detach()], 0).contiguous())
            dx = dx1
            g[2], g[3] = _ln_bwd(x, ln1w, dh, dx, ni[2] or ni[3])
            g[0] = dx if ni[0] else None
        return tuple(g)


class ClipDenseBlockFn(torch.autograd.Function):
    """ResidualAttentionBlock.forward_dense (model_vpt.py:219-240), the image encoder's last block:
    v = ln_1(x) . v_proj^T + b_v; vo = out_proj(v) + x[CLS] (the input CLS token of each image, broadcast
    over its tokens); out = vo + c_proj(QuickGELU(c_fc(ln_2(vo)))).  The q / k projections feed dead
    outputs in the reference (their out_proj results are discarded): their gradients are zero."""

    @staticmethod
    def forward(ctx, x, cfg, ln1w, ln1b, qw, kw, vw, ipb, ow, ob, ln2w, ln2b, fcw, fcb, pw, pb):
        n_img, L_ = cfg
        x = x.contiguous()
        R, W = x.shape
        y = torch.empty_like(x)
        ops.layernorm(x, ln1w.detach(), ln1b.detach(), y)
        v = torch.empty_like(x)
        ops.gemm(y, vw.detach().contiguous(), v, bias=ipb.detach()[2 * W:].contiguous())
        vo = torch.empty_like(x)
        ops.gemm(v, ow.detach().contiguous(), vo, bias=ob.detach().contiguous(), add=x, addmap=rowmap(d1=L_, s1=L_))
        h2 = torch.empty_like(x)
        ops.layernorm(vo, ln2w.detach(), ln2b.detach(), h2)
        u = _empty(R, fcw.shape[0], like=x)
        ops.gemm(h2, fcw.detach().contiguous(), u, bias=fcb.detach().contiguous())
        a = TO.act_forward(u, L.ACT_QUICKGELU)
        out = torch.empty_like(x)
        ops.gemm(a, pw.detach().contiguous(), out, bias=pb.detach().contiguous(), res=vo)
        ctx.save_for_backward(x, y, v, vo, h2, u, a, ln1w, vw, ow, ln2w, fcw, pw, qw, kw)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y, v, vo, h2, u, a, ln1w, vw, ow, ln2w, fcw, pw, qw, kw = ctx.saved_tensors
        n_img, L_ = ctx.cfg
        ni = ctx.needs_input_grad
        R, W = x.shape
        dout = dout.contiguous()
        g = [None] * 16
        if ni[14]:
            g[14] = _mm_t(dout, a)
        if ni[15]:
            g[15] = _colsum(dout)
        du = TO.mm(dout, pw.detach(), act_u=u, act=L.ACT_QUICKGELU)
        if ni[12]:
            g[12] = _mm_t(du, h2)
        if ni[13]:
            g[13] = _colsum(du)
        dh2 = TO.mm(du, fcw.detach())
        del du
        dvo = dout.clone()
        g[10], g[11] = _ln_bwd(vo, ln2w, dh2, dvo, ni[10] or ni[11])
        if ni[8]:
            g[8] = _mm_t(dvo, v)
        if ni[9]:
            g[9] = _colsum(dvo)
        dv = TO.mm(dvo, ow.detach())
        if ni[6]:
            g[6] = _mm_t(dv, y)
        if ni[4]:
            g[4] = torch.zeros_like(qw)
        if ni[5]:
            g[5] = torch.zeros_like(kw)
        if ni[7]:
            g[7] = torch.zeros(3 * W, device=x.device, dtype=_f32)
            _colsum(dv, out=g[7][2 * W:])
        dy = TO.mm(dv, vw.detach())
        dx = torch.empty_like(x)
        g[2], g[3] = _ln_bwd(x, ln1w, dy, dx, ni[2] or ni[3], acc_dx=False)
        # + x[:1]: the CLS row of each image receives the sum over the image's tokens (catseg_sum_classes
        # over the L token rows of each image, written to row b at stride L*W = the CLS rows)
        TO.sum_classes(dvo, dx.view(n_img, L_ * W), B=n_img, T=L_, HW=1, C_=W, beta=1)
        g[0] = dx
        return tuple(g)


class LnProjFn(torch.autograd.Function):
    """y = LayerNorm(x) @ proj: ln_post + visual.proj (model_vpt.py:306-313) and ln_final +
    text_projection (model_vpt.py:434-437).  proj [W][C_o]."""

    @staticmethod
    def forward(ctx, x, lnw, lnb, proj):
        x = x.contiguous()
        h = torch.empty_like(x)
        ops.layernorm(x, lnw.detach(), lnb.detach(), h)
        y = _empty(x.shape[0], proj.shape[1], like=x)
        ops.gemm(h, proj.detach().t().contiguous(), y)
        ctx.save_for_backward(x, h, lnw, proj)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, h, lnw, proj = ctx.saved_tensors
        ni = ctx.needs_input_grad
        dy = dy.contiguous()
        W, Co = proj.shape
        pr = proj.detach()
        dh = _empty(x.shape[0], W, like=x)
        TO.gemm_ex(dy, Co, 1, pr, 1, Co, dh, M=x.shape[0], N=W, K=Co)        # dh = dy . proj^T
        dproj = _mm_t(h, dy) if ni[3] else None
        dx = torch.empty_like(x)
        dlw, dlb = _ln_bwd(x, lnw, dh, dx, ni[1] or ni[2], acc_dx=False)
        return dx, dlw, dlb, dproj


class EotGatherFn(torch.autograd.Function):
    """x[arange(n), tokens.argmax(-1)] (model_vpt.py:436): rows [n*ctx][W] -> [n][W]."""

    @staticmethod
    def forward(ctx, x, tokens, eot_rows):
        x = x.contiguous()
        n, cl = tokens.shape
        out = _empty(n, x.shape[1], like=x)
        ops.eot_gather(x, tokens, out)
        ctx.save_for_backward(eot_rows)
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, dy):
        (eot_rows,) = ctx.saved_tensors
        dx = torch.zeros(ctx.shape, device=dy.device, dtype=_f32)
        TO.scatter_rows(dy.contiguous(), eot_rows, dx)
        return dx, None, None


def _clip_block_params(P, p):
    return [P[p + k] for k in ("ln_1.weight", "ln_1.bias", "attn.q_proj_weight", "attn.k_proj_weight",
                               "attn.v_proj_weight", "attn.in_proj_bias", "attn.out_proj.weight",
                               "attn.out_proj.bias", "ln_2.weight", "ln_2.bias", "mlp.c_fc.weight", "mlp.c_fc.bias",
                               "mlp.c_proj.weight", "mlp.c_proj.bias")]


def clip_image_train_forward(arch: CatSegArch, P: Dict[str, torch.Tensor], eng, raw: torch.Tensor,
                             sizes: torch.Tensor):
    """CLIP.encode_image(dense=True) with the forward hooks (cat_seg_model.py:84-87,144-146,
    model_vpt.py:288-314), the transformer blocks as autograd Functions.  The embedding (patch conv,
    class / positional embedding, ln_pre) is outside `transformer` and frozen under every CLIP_FINETUNE
    mode (cat_seg_model.py:58-75): the engine computes it without a graph.
    Returns feats [B*(1+G^2)][C_o] and the two hook outputs [B*(1+G^2)][W]."""
    from .weights import CLIP
    if arch.vpt:
        raise NotImplementedError("training step: visual prompt tuning (CLIP_FINETUNE 'prompt') is not built")
    B = raw.shape[0]
    L_ = arch.grid * arch.grid + 1
    x = eng.embed_image(raw, sizes)
    p = CLIP + "visual."
    hooks: List[torch.Tensor] = []
    for i in range(arch.vision_layers - 1):
        x = ClipBlockFn.apply(x, (B, L_, arch.vision_heads, False),
                              *_clip_block_params(P, f"{p}transformer.resblocks.{i}."))
        if i in arch.hook_layers:
            hooks.append(x)
    x = ClipDenseBlockFn.apply(x, (B, L_), *_clip_block_params(P, f"{p}transformer.resblocks.{arch.vision_layers - 1}."))
    feats = LnProjFn.apply(x, P[p + "ln_post.weight"], P[p + "ln_post.bias"], P[p + "proj"])
    return feats, hooks


def clip_text_train_forward(arch: CatSegArch, P: Dict[str, torch.Tensor], eng, tokens: torch.Tensor) -> torch.Tensor:
    """CLIP.encode_text + L2 norm (model_vpt.py:421-438, cat_seg_predictor.py:214-216) with the causal
    blocks as autograd Functions, on the first max(EOT)+1 positions (causal: later positions never reach
    the EOT rows, forward or backward).  tokens (T, ctx) int.  Returns [T][C_o]."""
    from .weights import CLIP
    toks = torch.as_tensor(tokens)
    last = int(toks.argmax(dim=1).max()) + 1
    toks = toks[:, :last]
    n, cl = toks.shape
    eot_rows = (torch.arange(n) * cl + toks.argmax(dim=1)).to(torch.int32)
    tdev = toks.to(eng.device, torch.int32).contiguous()
    x = eng.embed_text(tdev)
    for i in range(arch.text_layers):
        x = ClipBlockFn.apply(x, (n, cl, arch.text_heads, True), *_clip_block_params(P, f"{CLIP}transformer.resblocks.{i}."))
    e = EotGatherFn.apply(x, tdev, eot_rows.to(eng.device))
    t = LnProjFn.apply(e, P[CLIP + "ln_final.weight"], P[CLIP + "ln_final.bias"], P[CLIP + "text_projection"])
    return L2NormFn.apply(t)


# ------------------------------------------------------------------------------------- the head
def head_train_forward(arch: CatSegArch, P: Dict[str, torch.Tensor], feats: torch.Tensor, hooks: List[torch.Tensor],
                       text: torch.Tensor) -> torch.Tensor:
    """Training-mode head (cat_seg_model.py:178-188 -> CATSegHead.forward -> Aggregator.forward,
    model.py:683-725), fp32, with the HIP backward.  P: parameters by reference key (nn.Parameters
    of the model); feats [B*(1+G^2)][C_o] dense CLIP tokens, hooks 2 x [B*(1+G^2)][W_v] (the forward
    hooks of cat_seg_model.py:84-87), text [T][C_o] class embeddings.  Returns logits [B][T][4G][4G]."""
    a = arch
    if a.vpt:
        raise NotImplementedError("training step: visual prompt tuning is not built (frozen-CLIP features "
                                  "carry the prompt rows)")
    if a.attention_type != "linear":
        raise NotImplementedError("training step: ATTENTION_TYPE 'linear' only (the full-attention backward is not built)")
    G = a.grid
    HW = G * G
    B = feats.shape[0] // (HW + 1)
    T = text.shape[0]
    if a.pad_len > 0 and T > a.pad_len:
        raise NotImplementedError("training with more classes than pad_len (top-k selection) is not built")
    if a.hidden_dim != 128 or a.nheads != 4:
        raise NotImplementedError("HIP training path: hidden_dim 128 / 4 heads only")
    geo = Geo(B=B, T=T, H=G, W=G, nh=a.nheads)
    p = AGG
    # guidance maps (cat_seg_model.py:178-186): res3 = dense tokens, res4/res5 = ConvTranspose of the hooks
    res3 = DropClsFn.apply(feats, HW)
    res4 = ConvTUpsampleFn.apply(hooks[0], P["upsample1.weight"], P["upsample1.bias"], G)
    res5 = ConvTUpsampleFn.apply(hooks[1], P["upsample2.weight"], P["upsample2.bias"], G)
    # cost volume + embedding (model.py:648-659,689-699)
    corr = CostVolumeFn.apply(feats, text, HW)
    X = CorrEmbedFn.apply(corr, P[p + "conv1.weight"], P[p + "conv1.bias"], G)
    # guidance projections (model.py:706-715)
    g3 = Conv3x3Fn.apply(res3, P[p + "guidance_projection.0.weight"], P[p + "guidance_projection.0.bias"], B, G, G)
    gd = [Conv3x3Fn.apply(r, P[f"{p}decoder_guidance_projection.{i}.0.weight"],
                          P[f"{p}decoder_guidance_projection.{i}.0.bias"], B, G * 2 ** (i + 1), G * 2 ** (i + 1))
          for i, r in enumerate((res4, res5))]
    tn = L2NormFn.apply(text)          # text_feats.mean over prompts (one) then normalized again (model.py:712-714)
    tg = LinearFn.apply(tn, P[p + "text_guidance_projection.0.weight"], P[p + "text_guidance_projection.0.bias"],
                        L.ACT_RELU)
    ws = a.window_size
    shift2 = ws // 2
    if min(G, G) <= ws:
        ws, shift2 = min(G, G), 0
    for l in range(a.num_layers):
        sw = f"{p}layers.{l}.swin_block."
        gn = LayerNormRowsFn.apply(g3, P[sw + "guidance_norm.weight"], P[sw + "guidance_norm.bias"])
        for name, shift in (("block_1", 0), ("block_2", shift2)):
            q = f"{sw}{name}."
            X = SwinBlockFn.apply(X, gn, geo, ws, shift, *(P[q + k] for k in (
                "norm1.weight", "norm1.bias", "attn.q.weight", "attn.q.bias", "attn.k.weight", "attn.k.bias",
                "attn.v.weight", "attn.v.bias", "attn.proj.weight", "attn.proj.bias", "norm2.weight", "norm2.bias",
                "mlp.fc1.weight", "mlp.fc1.bias", "mlp.fc2.weight", "mlp.fc2.bias")))
        c = f"{p}layers.{l}.attention."
        pad = (P[c + "padding_tokens"], P[c + "padding_guidance"]) if a.pad_len > 0 else (None, None)
        X = ClassLayerFn.apply(X, tg, geo, tuple(a.pooling_size), a.pad_len, *(P[c + k] for k in (
            "norm1.weight", "norm1.bias", "attention.q.weight", "attention.q.bias", "attention.k.weight",
            "attention.k.bias", "attention.v.weight", "attention.v.bias", "norm2.weight", "norm2.bias",
            "MLP.0.weight", "MLP.0.bias", "MLP.2.weight", "MLP.2.bias")), *pad)
    y, h = X, G
    for i in (1, 2):
        q = f"{p}decoder{i}."
        y = UpBlockFn.apply(y, gd[i - 1], geo, h, *(P[q + k] for k in (
            "up.weight", "up.bias", "conv.double_conv.0.weight", "conv.double_conv.1.weight",
            "conv.double_conv.1.bias", "conv.double_conv.3.weight", "conv.double_conv.4.weight",
            "conv.double_conv.4.bias")))
        h *= 2
    return HeadConvFn.apply(y, P[p + "head.weight"], P[p + "head.bias"], geo, h)
