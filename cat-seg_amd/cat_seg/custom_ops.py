"""torch.library custom ops over the C ABI ("Python side: torch.library.custom_op wrappers
on torch.cuda.current_stream(), raising RuntimeError on nonzero status").

Each op is a functional wrapper (fresh output, no mutation) around the ctypes entry point of `ops` /
`train_ops`, registered under the `catseg::` namespace with a fake (meta) implementation, so the
dispatcher, FakeTensor tracing, `torch.compile` (fullgraph) and `torch.library.opcheck` see them as
ordinary operators.  The engine keeps calling the ctypes layer directly (its hipGraph capture does not
need the dispatcher); these are the registered surface for code that composes the kernels with torch.

  catseg::gemm             nn.Linear / ConvTranspose GEMMs (catseg_gemm; model_vpt.py:193-236, model.py:77-112)
  catseg::layernorm        LayerNorm (catseg_layernorm; model_vpt.py:156-162, model.py:152,158,368-369)
  catseg::attention        softmax attention, dense / causal / Swin window (catseg_attention)
  catseg::class_attention  fused norm1 + q/k/v + linear class attention (catseg_class_attention)
  catseg::postprocess      sigmoid + bilinear resize (catseg_postprocess; cat_seg_model.py:222-228)
  catseg::linear           y = act(x W^T + b) with a registered backward (catseg_gemm forward,
                           catseg_gemm_ex / catseg_colsum backward): the training kernels through autograd
  catseg::head_logits      the whole eval forward of a registered CATSeg model up to the logits
                           (CLIP dense encode + Aggregator, cat_seg_model.py:155-188): one opaque operator,
                           so `torch.compile(model, fullgraph=True)` traces CATSeg.forward with no break
"""
from __future__ import annotations

import itertools
import weakref
from typing import Optional, Tuple

import torch

from . import _lib as L
from . import ops, train_ops as TO

_DT = {0: torch.float32, 1: torch.bfloat16}


def _code(dtype: torch.dtype) -> int:
    return 1 if dtype == torch.bfloat16 else 0


# ------------------------------------------------------------------------------------- gemm
@torch.library.custom_op("catseg::gemm", mutates_args=())
def gemm(A: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], act: int, res: Optional[torch.Tensor],
         out_dtype: int) -> torch.Tensor:
    """out = act(A . W^T + bias) + res; A (M, K) and W (N, K) of one dtype (fp32 / bf16), bias fp32,
    res and out of out_dtype (0 fp32, 1 bf16)."""
    out = torch.empty(A.shape[0], W.shape[0], device=A.device, dtype=_DT[out_dtype])
    ops.gemm(A.contiguous(), W.contiguous(), out, bias=None if bias is None else bias.contiguous(), act=act,
             res=None if res is None else res.contiguous())
    return out


@gemm.register_fake
def _(A, W, bias, act, res, out_dtype):
    return A.new_empty((A.shape[0], W.shape[0]), dtype=_DT[out_dtype])


# ------------------------------------------------------------------------------------- layernorm
@torch.library.custom_op("catseg::layernorm", mutates_args=())
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, out_dtype: int) -> torch.Tensor:
    out = torch.empty(x.shape, device=x.device, dtype=_DT[out_dtype])
    ops.layernorm(x.contiguous(), gamma.contiguous(), beta.contiguous(), out, eps=eps)
    return out


@layernorm.register_fake
def _(x, gamma, beta, eps, out_dtype):
    return x.new_empty(x.shape, dtype=_DT[out_dtype])


# ------------------------------------------------------------------------------------- attention
@torch.library.custom_op("catseg::attention", mutates_args=())
def attention(qkv: torch.Tensor, n_seq: int, seq_len: int, n_heads: int, causal: bool, mode: int, img_h: int,
              img_w: int, window: int, shift: int) -> torch.Tensor:
    """Softmax attention over the q | k | v columns of qkv (R, 3W): mode 0 dense (causal optional),
    mode 1 Swin windows with the cyclic shift and -100 region mask.  Returns (R, W)."""
    W = qkv.shape[1] // 3
    hd = W // n_heads
    qkv = qkv.contiguous()
    out = torch.empty(qkv.shape[0], W, device=qkv.device, dtype=qkv.dtype)
    ops.attention(qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:], out, n_seq=n_seq, seq_len=seq_len, n_heads=n_heads,
                  head_dim=hd, scale=hd ** -0.5, causal=causal, mode=mode, img_hw=(img_h, img_w), window=window,
                  shift=shift)
    return out


@attention.register_fake
def _(qkv, n_seq, seq_len, n_heads, causal, mode, img_h, img_w, window, shift):
    return qkv.new_empty((qkv.shape[0], qkv.shape[1] // 3))


# ------------------------------------------------------------------------------------- class attention
@torch.library.custom_op("catseg::class_attention", mutates_args=())
def class_attention(x: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, w_qkv: torch.Tensor,
                    b_qkv: torch.Tensor, tg: torch.Tensor, B: int, T: int, HW: int, n_pad: int,
                    k_pad: Optional[torch.Tensor], v_pad: Optional[torch.Tensor]) -> torch.Tensor:
    """y = x + LinearAttention(norm1(x) q/k/v + text guidance) over the (b, t, p) rows of x (bf16),
    4 heads x 32 (catseg_class_attention)."""
    y = torch.empty_like(x)
    ops.class_attention(x.contiguous(), (ln_w, ln_b), w_qkv.contiguous(), b_qkv.contiguous(), tg.contiguous(), y, B=B,
                        T=T, HW=HW, n_heads=4, head_dim=x.shape[1] // 4, n_pad=n_pad, k_pad=k_pad, v_pad=v_pad)
    return y


@class_attention.register_fake
def _(x, ln_w, ln_b, w_qkv, b_qkv, tg, B, T, HW, n_pad, k_pad, v_pad):
    return torch.empty_like(x)


# ------------------------------------------------------------------------------------- postprocess
@torch.library.custom_op("catseg::postprocess", mutates_args=())
def postprocess(logits: torch.Tensor, H: int, W: int, crop_h: int, crop_w: int) -> torch.Tensor:
    """sigmoid, crop to (crop_h, crop_w), bilinear (align_corners=False) to H x W: (B, T, h, w) fp32 ->
    (B, T, H, W) fp32 (catseg_postprocess)."""
    out = torch.empty(logits.shape[0], logits.shape[1], H, W, device=logits.device, dtype=torch.float32)
    ops.postprocess(logits.contiguous(), out, crop=(crop_h, crop_w))
    return out


@postprocess.register_fake
def _(logits, H, W, crop_h, crop_w):
    return logits.new_empty((logits.shape[0], logits.shape[1], H, W), dtype=torch.float32)


# ------------------------------------------------------------------------------------- linear (+ backward)
@torch.library.custom_op("catseg::linear", mutates_args=())
def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, act: int) -> torch.Tensor:
    """y = act(x . w^T + b), fp32; act NONE or RELU; differentiable through the training kernels."""
    y = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
    ops.gemm(x.contiguous(), w.contiguous(), y, bias=b.contiguous(), act=act)
    return y


@linear.register_fake
def _(x, w, b, act):
    return x.new_empty((x.shape[0], w.shape[0]))


def _linear_setup(ctx, inputs, output):
    x, w, b, act = inputs
    ctx.save_for_backward(x, w, output)
    ctx.act = act


def _linear_backward(ctx, dy):
    x, w, y = ctx.saved_tensors
    dy = dy.contiguous()
    if ctx.act == L.ACT_RELU:
        dy = torch.ops.catseg.act_backward(y, dy, L.ACT_RELU)
    dx = torch.ops.catseg.mm(dy, w, False, False)
    dw = torch.ops.catseg.mm(dy, x, True, False)
    db = torch.ops.catseg.colsum(dy)
    return dx, dw, db, None


@torch.library.custom_op("catseg::mm", mutates_args=())
def mm(a: torch.Tensor, b: torch.Tensor, trans_a: bool, trans_b: bool) -> torch.Tensor:
    """op(a) @ op(b) in fp32 (catseg_gemm_ex: no operand is transposed in memory)."""
    a, b = a.contiguous(), b.contiguous()
    A = a.t() if trans_a else a
    Bm = b.t() if trans_b else b
    return TO.mm(A, Bm)


@mm.register_fake
def _(a, b, trans_a, trans_b):
    M = a.shape[1] if trans_a else a.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    return a.new_empty((M, N))


@torch.library.custom_op("catseg::colsum", mutates_args=())
def colsum(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.shape[1], device=x.device, dtype=torch.float32)
    return TO.colsum(x.contiguous(), out)


@colsum.register_fake
def _(x):
    return x.new_empty((x.shape[1],))


@torch.library.custom_op("catseg::act_backward", mutates_args=())
def act_backward(u: torch.Tensor, dy: torch.Tensor, act: int) -> torch.Tensor:
    return TO.act_backward(u.contiguous(), dy.contiguous(), act)


@act_backward.register_fake
def _(u, dy, act):
    return torch.empty_like(u)


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


# ------------------------------------------------------------------------------------- whole-model forward
# CATSeg models register themselves here (an int handle, so the operator's schema stays plain); the op
# runs the model's engine eagerly, the fake kernel only needs the output geometry.
_MODELS: "dict[int, weakref.ref]" = {}
_next_handle = itertools.count(1)


def register_model(model) -> int:
    h = next(_next_handle)
    _MODELS[h] = weakref.ref(model)
    return h


def _model(handle: int):
    m = _MODELS.get(handle)
    m = m() if m is not None else None
    if m is None:
        raise RuntimeError(f"catseg: no live CATSeg model with handle {handle}")
    return m


@torch._dynamo.assume_constant_result
def head_meta(handle: int) -> Tuple[int, int]:
    """(T0, logit resolution) of a registered model, with its engine built and its test-class text
    embeddings cached: run eagerly when dynamo traces CATSeg.forward (a constant of the graph)."""
    m = _model(handle)
    eng = m.engine
    m.sem_seg_head.predictor.get_text_embeds()
    return int(eng.n_classes), int(4 * m.arch.grid)


@torch.library.custom_op("catseg::head_logits", mutates_args=())
def head_logits(raw: torch.Tensor, sizes: torch.Tensor, handle: int, n_classes: int, res: int) -> torch.Tensor:
    """fp32 logits (B, T0, res, res) of the registered model's eval forward (CatSegEngine.head_logits)
    for the zero-padded image canvas raw (B, 3, H, W) fp32 and the per-image sizes (B, 2) int32."""
    m = _model(handle)
    eng = m.engine
    m.sem_seg_head.predictor.get_text_embeds()
    out = eng.head_logits(raw.contiguous(), sizes.contiguous())
    if tuple(out.shape) != (raw.shape[0], n_classes, res, res):
        raise RuntimeError(f"catseg::head_logits: logits {tuple(out.shape)} != the traced geometry "
                           f"{(raw.shape[0], n_classes, res, res)} (class set changed after tracing?)")
    return out.clone()


@head_logits.register_fake
def _(raw, sizes, handle, n_classes, res):
    return raw.new_empty((raw.shape[0], n_classes, res, res))
