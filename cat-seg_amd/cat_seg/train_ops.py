"""Python mirror of the training-side C ABI (include/catseg_hip_train.h): one thin wrapper per
entry point, as `ops.py` is for the forward kernels.

Every wrapper takes fp32 device tensors, sizes its workspace from the library's own query (caching
allocator, graph-capturable), launches on `torch.cuda.current_stream()` and raises RuntimeError on a
non-zero status.  No wrapper has a fallback: a missing library or device raises.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _lib as L
from ._lib import IDENTITY
from .ops import _rec, _stream, call

_f32 = torch.float32


def _ws(nbytes: int, device) -> Optional[torch.Tensor]:
    if nbytes <= 0:
        return None
    return torch.empty((nbytes + 3) // 4, device=device, dtype=_f32)


def _chk(*ts):
    for t in ts:
        if t is not None:
            assert t.dtype == _f32 and t.is_cuda, f"fp32 device tensor expected, got {t.dtype} on {t.device}"


def gemm_ex(A, a_sm, a_sk, B, b_sk, b_sn, out, *, M, N, K, ldc=None, alpha=1.0, beta=0, flops_name="gemm_ex",
            act_u=None, act=L.ACT_NONE):
    """out[m][n] = alpha * sum_k A[m*a_sm + k*a_sk] * B[k*b_sk + n*b_sn] + beta * out (catseg_gemm_ex);
    with act: out = alpha * (A B) * act'(act_u) (the activation backward fused, beta 0).
    A / B / out may be views: their data_ptr() is the element (0, 0)."""
    _chk(A, B, out, act_u)
    a = L.GemmExArgs()
    a.A, a.a_sm, a.a_sk = A.data_ptr(), a_sm, a_sk
    a.B, a.b_sk, a.b_sn = B.data_ptr(), b_sk, b_sn
    a.M, a.N, a.K = M, N, K
    a.C, a.ldc = out.data_ptr(), ldc if ldc is not None else out.stride(-2)
    a.alpha, a.beta = alpha, int(beta)
    if act != L.ACT_NONE:
        a.act_u, a.ld_u, a.act = act_u.data_ptr(), act_u.stride(-2), int(act)
    ws = None if act != L.ACT_NONE else _ws(L.load().catseg_gemm_ex_workspace(M, N, K), out.device)
    if ws is not None:
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    with _rec(flops_name, 2 * M * N * K, 4 * (M * K + K * N + M * N),
              shape=(M, N, K, "m" if a_sm == 1 else "k", "n" if b_sn == 1 else "k")):
        call("catseg_gemm_ex", a, _stream())
    return out


def mm(A, B, out=None, *, beta=0, alpha=1.0, act_u=None, act=L.ACT_NONE):
    """out = alpha * A @ B (+ out): A (M, K), B (K, N) strided 2-D views with a unit stride each;
    act: out = (A @ B) * act'(act_u), the activation's backward fused into the GEMM's epilogue."""
    M, K = A.shape
    N = B.shape[1]
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=_f32)
    return gemm_ex(A, A.stride(0), A.stride(1), B, B.stride(0), B.stride(1), out, M=M, N=N, K=K, alpha=alpha,
                   beta=beta, act_u=act_u, act=act)


def colsum(x, out, *, rows=None, cols=None, ld=None, alpha=1.0, beta=0):
    """out[c] = alpha * sum_r x[r][c] (+ out[c]) (catseg_colsum)."""
    _chk(x, out)
    rows = rows if rows is not None else x.shape[0]
    cols = cols if cols is not None else x.shape[-1]
    ld = ld if ld is not None else x.stride(-2)
    ws = _ws(L.load().catseg_colsum_workspace(rows, cols), x.device)
    with _rec("colsum", 0, 4 * rows * cols):
        call("catseg_colsum", x.data_ptr(), ld, rows, cols, out.data_ptr(), alpha, int(beta), ws.data_ptr(),
             ws.numel() * 4, _stream())
    return out


def layernorm_backward(x, gamma, dy, dx, *, acc_dx=False, dgamma=None, dbeta=None, acc_param=False, eps=1e-5):
    """catseg_layernorm_backward over rows (x, dy, dx: 2-D row-major views)."""
    _chk(x, gamma, dy, dx, dgamma, dbeta)
    rows, cols = x.shape
    ws = None
    if dgamma is not None:
        ws = _ws(L.load().catseg_layernorm_backward_workspace(rows, cols), x.device)
    with _rec("layernorm_backward", 0, 4 * rows * cols * 3):
        call("catseg_layernorm_backward", x.data_ptr(), x.stride(0), gamma.data_ptr(), dy.data_ptr(), dy.stride(0),
             dx.data_ptr(), dx.stride(0), int(acc_dx), rows, cols, eps,
             None if dgamma is None else dgamma.data_ptr(), None if dbeta is None else dbeta.data_ptr(),
             int(acc_param), None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel() * 4, _stream())
    return dx


def act_forward(u, act, out=None):
    _chk(u)
    out = torch.empty_like(u) if out is None else out
    with _rec("act_forward", 0, 8 * u.numel()):
        call("catseg_act_forward", u.data_ptr(), out.data_ptr(), u.numel(), act, _stream())
    return out


def act_backward(u, dy, act, out=None):
    _chk(u, dy)
    out = torch.empty_like(u) if out is None else out
    with _rec("act_backward", 0, 12 * u.numel()):
        call("catseg_act_backward", u.data_ptr(), dy.data_ptr(), out.data_ptr(), u.numel(), act, _stream())
    return out


def groupnorm_stats_rows(x, S, HW, C_, cpg, mean, rstd, eps=1e-5):
    _chk(x, mean, rstd)
    ws = _ws(L.load().catseg_groupnorm_stats_rows_workspace(S, HW, C_, cpg), x.device)
    with _rec("groupnorm_stats_rows", 0, 4 * x.numel()):
        call("catseg_groupnorm_stats_rows", x.data_ptr(), S, HW, C_, cpg, eps, mean.data_ptr(), rstd.data_ptr(),
             None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel() * 4, _stream())
    return mean, rstd


def groupnorm_relu_backward(x, dy, dx, *, S, HW, C_, cpg, mean, rstd, gamma, beta, dgamma, dbeta, acc_param=False):
    _chk(x, dy, dx, mean, rstd, gamma, beta, dgamma, dbeta)
    ws = _ws(L.load().catseg_groupnorm_relu_backward_workspace(S, HW, C_), x.device)
    with _rec("groupnorm_relu_backward", 0, 4 * x.numel() * 5):   # x, dy read twice, dx written
        call("catseg_groupnorm_relu_backward", x.data_ptr(), dy.data_ptr(), dx.data_ptr(), S, HW, C_, cpg,
             mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(),
             int(acc_param), None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel() * 4, _stream())
    return dx


def l2normalize_backward(x, dy, dx, *, rows, cols, inmap=None, outmap=None, beta=0, eps=1e-12):
    _chk(x, dy, dx)
    call("catseg_l2normalize_backward", x.data_ptr(), x.stride(-2), inmap or IDENTITY, dy.data_ptr(), dy.stride(-2),
         dx.data_ptr(), dx.stride(-2), outmap or IDENTITY, int(beta), rows, cols, eps, _stream())
    return dx


def axpby(x, y, out, alpha=1.0, beta=1.0):
    """out = alpha * x + beta * y (y None: out = alpha * x) over whole contiguous tensors."""
    _chk(x, y, out)
    assert x.is_contiguous() and out.is_contiguous() and (y is None or y.is_contiguous())
    call("catseg_axpby", x.data_ptr(), None if y is None else y.data_ptr(), out.data_ptr(), x.numel(), alpha, beta,
         _stream())
    return out


def scatter_rows(x, idx, out):
    """out[idx[r]] = x[r] (catseg_scatter_rows); idx int32 on the device."""
    _chk(x, out)
    call("catseg_scatter_rows", x.data_ptr(), x.stride(-2), idx.data_ptr(), x.shape[0], x.shape[1], out.data_ptr(),
         out.stride(-2), _stream())
    return out


def corr_embed_backward_input(dX, weight, dcorr, *, S, H, W):
    """dcorr [S][H*W] of corr_embed's conv (catseg_corr_embed_backward_input); weight (D, 1, k, k)."""
    _chk(dX, weight, dcorr)
    D, _, k, _ = weight.shape
    with _rec("corr_embed_backward_input", 2 * S * H * W * D * k * k):
        call("catseg_corr_embed_backward_input", dX.data_ptr(), weight.data_ptr(), dcorr.data_ptr(), S, H, W, D, k,
             _stream())
    return dcorr


def add_dev_scalar(x, s):
    _chk(x, s)
    call("catseg_add_dev_scalar", x.data_ptr(), x.numel(), s.data_ptr(), _stream())
    return x


def sum_classes(x, out, *, B, T, HW, C_, beta=0):
    """out[b*HW + p] (+)= sum_t x[(b*T + t)*HW + p] over the first C_ columns (catseg_sum_classes)."""
    _chk(x, out)
    with _rec("sum_classes", 0, 4 * B * T * HW * C_):
        call("catseg_sum_classes", x.data_ptr(), x.stride(-2), B, T, HW, C_, out.data_ptr(), out.stride(-2), int(beta),
             _stream())
    return out


def sum_pixels(x, out, *, B, T, HW, C_, beta=0):
    """out[t] (+)= sum_{b,p} x[(b*T + t)*HW + p] over the first C_ columns (catseg_sum_pixels)."""
    _chk(x, out)
    with _rec("sum_pixels", 0, 4 * B * T * HW * C_):
        call("catseg_sum_pixels", x.data_ptr(), x.stride(-2), B, T, HW, C_, out.data_ptr(), out.stride(-2), int(beta),
             _stream())
    return out


def avgpool_backward_rows(dxp, dx, *, S, H, W, C_, pool, beta=0):
    _chk(dxp, dx)
    call("catseg_avgpool_backward_rows", dxp.data_ptr(), S, H, W, C_, pool[0], pool[1], dx.data_ptr(), int(beta),
         _stream())
    return dx


def upsample_ac_backward_rows(dy, dxp, *, S, H, W, C_, Hp, Wp, beta=0):
    _chk(dy, dxp)
    call("catseg_upsample_ac_backward_rows", dy.data_ptr(), S, H, W, C_, Hp, Wp, dxp.data_ptr(), int(beta), _stream())
    return dxp


def convt_gather(dout, g, *, S, hin, win, k, cout, ld=None):
    _chk(dout, g)
    ld = ld if ld is not None else dout.stride(-2)
    with _rec("convt_gather", 0, 8 * g.numel()):
        call("catseg_convt_gather", dout.data_ptr(), ld, S, hin, win, k, cout, g.data_ptr(), _stream())
    return g


def window_attention_backward(qkv, o, dout, dqkv, *, S, img_hw, window, shift, n_heads, head_dim, scale):
    """dq | dk | dv of the Swin window attention (catseg_window_attention_backward); qkv / dqkv are the
    [R][3D] row buffers of the forward projections and their gradients."""
    _chk(qkv, o, dout, dqkv)
    D = n_heads * head_dim
    a = L.WinAttnBwdArgs()
    a.q, a.k, a.v, a.ld_qkv = qkv.data_ptr(), qkv[:, D:].data_ptr(), qkv[:, 2 * D:].data_ptr(), qkv.stride(0)
    a.o, a.ld_o = o.data_ptr(), o.stride(0)
    a.dout, a.ld_dout = dout.data_ptr(), dout.stride(0)
    a.dq, a.dk, a.dv, a.ld_dqkv = dqkv.data_ptr(), dqkv[:, D:].data_ptr(), dqkv[:, 2 * D:].data_ptr(), dqkv.stride(0)
    a.S, a.img_h, a.img_w, a.window, a.shift = S, img_hw[0], img_hw[1], window, shift
    a.n_heads, a.head_dim, a.scale = n_heads, head_dim, scale
    R = S * img_hw[0] * img_hw[1]
    with _rec("window_attention_backward", 8 * R * window * window * D):
        call("catseg_window_attention_backward", a, _stream())
    return dqkv


def attention_backward(qkv, o, dout, dqkv, *, n_seq, seq_len, n_heads, head_dim, scale, causal=False):
    """dq | dk | dv of the dense (CLIP) attention (catseg_attention_backward); qkv / dqkv are [R][3W]
    row buffers (q, k, v at column offsets 0, W, 2W)."""
    _chk(qkv, o, dout, dqkv)
    W = n_heads * head_dim
    a = L.AttnBwdArgs()
    a.q, a.k, a.v, a.ld_qkv = qkv.data_ptr(), qkv[:, W:].data_ptr(), qkv[:, 2 * W:].data_ptr(), qkv.stride(0)
    a.o, a.ld_o = o.data_ptr(), o.stride(0)
    a.dout, a.ld_dout = dout.data_ptr(), dout.stride(0)
    a.dq, a.dk, a.dv, a.ld_dqkv = dqkv.data_ptr(), dqkv[:, W:].data_ptr(), dqkv[:, 2 * W:].data_ptr(), dqkv.stride(0)
    a.n_seq, a.seq_len, a.n_heads, a.head_dim, a.scale, a.causal = n_seq, seq_len, n_heads, head_dim, scale, int(causal)
    ws = _ws(L.load().catseg_attention_backward_workspace(n_seq, seq_len, n_heads), qkv.device)
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    with _rec("attention_backward", 10 * n_seq * n_heads * seq_len * seq_len * head_dim):
        call("catseg_attention_backward", a, _stream())
    return dqkv


def linear_attention_backward(qkv, dy, dqkv, *, B, T, HW, n_heads, head_dim, n_pad=0, k_pad=None, v_pad=None,
                              dk_pad=None, dv_pad=None, eps=1e-6):
    _chk(qkv, dy, dqkv, k_pad, v_pad, dk_pad, dv_pad)
    D = n_heads * head_dim
    a = L.LinAttnBwdArgs()
    a.q, a.k, a.v, a.ld_qkv = qkv.data_ptr(), qkv[:, D:].data_ptr(), qkv[:, 2 * D:].data_ptr(), qkv.stride(0)
    a.dy, a.ld_dy = dy.data_ptr(), dy.stride(0)
    a.dq, a.dk, a.dv, a.ld_dqkv = dqkv.data_ptr(), dqkv[:, D:].data_ptr(), dqkv[:, 2 * D:].data_ptr(), dqkv.stride(0)
    a.B, a.T, a.HW, a.n_heads, a.head_dim = B, T, HW, n_heads, head_dim
    a.n_pad, a.eps = n_pad, eps
    ws = None
    if n_pad > 0:
        a.k_pad, a.v_pad, a.dk_pad, a.dv_pad = k_pad.data_ptr(), v_pad.data_ptr(), dk_pad.data_ptr(), dv_pad.data_ptr()
        ws = _ws(L.load().catseg_linear_attention_backward_workspace(B, HW), qkv.device)
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    with _rec("linear_attention_backward", 12 * B * HW * T * D * head_dim):
        call("catseg_linear_attention_backward", a, _stream())
    return dqkv


def _conv_args(x, w, y, *, S, H, W, cin, cout, ksize, bias=None, act=L.ACT_NONE, alpha=1.0, beta=0, ld_x=None,
               ld_y=None, ld_w=None, dw=None):
    a = L.Conv2dArgs()
    a.x, a.ld_x = x.data_ptr(), ld_x if ld_x is not None else x.stride(-2)
    a.S, a.H, a.W, a.cin = S, H, W, cin
    if w is not None:
        a.w, a.ld_w = w.data_ptr(), ld_w if ld_w is not None else w.stride(-2)
    a.cout, a.ksize, a.pad = cout, ksize, ksize // 2
    a.bias = None if bias is None else bias.data_ptr()
    a.act = act
    a.y, a.ld_y = y.data_ptr(), ld_y if ld_y is not None else y.stride(-2)
    a.alpha, a.beta = alpha, int(beta)
    a.dw = None if dw is None else dw.data_ptr()
    return a


def conv2d(x, w, y, *, S, H, W, cin, cout, ksize=3, bias=None, act=L.ACT_NONE, alpha=1.0, beta=0, ld_x=None,
           ld_y=None):
    """y = alpha * act(conv(x, w) + bias) + beta * y over NHWC rows; w: [k*k*cin][cout] (catseg_conv2d_nhwc)."""
    _chk(x, w, y, bias)
    a = _conv_args(x, w, y, S=S, H=H, W=W, cin=cin, cout=cout, ksize=ksize, bias=bias, act=act, alpha=alpha,
                   beta=beta, ld_x=ld_x, ld_y=ld_y)
    with _rec("conv2d", 2 * S * H * W * cout * cin * ksize * ksize, shape=(S * H * W, cin, cout, ksize)):
        call("catseg_conv2d_nhwc", a, _stream())
    return y


def conv2d_wgrad(x, dy, dw, *, S, H, W, cin, cout, ksize=3, alpha=1.0, beta=0, ld_x=None, ld_y=None):
    """dw[(tap, ci)][co] = sum_p x[p + tap][ci] dy[p][co] (catseg_conv2d_wgrad)."""
    _chk(x, dy, dw)
    a = _conv_args(x, None, dy, S=S, H=H, W=W, cin=cin, cout=cout, ksize=ksize, alpha=alpha, beta=beta, ld_x=ld_x,
                   ld_y=ld_y, dw=dw)
    ws = _ws(L.load().catseg_conv2d_wgrad_workspace(C.byref(a)), x.device)
    if ws is not None:
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    with _rec("conv2d_wgrad", 2 * S * H * W * cout * cin * ksize * ksize, shape=(S * H * W, cin, cout, ksize)):
        call("catseg_conv2d_wgrad", a, _stream())
    return dw


def head_conv_backward(x, dlogits, weight, dx, dw, *, S, H, W, C_):
    _chk(x, dlogits, weight, dx, dw)
    ws = _ws(L.load().catseg_head_conv_backward_workspace(S, H, W, C_), x.device)
    with _rec("head_conv_backward", 4 * S * H * W * C_ * 9):
        call("catseg_head_conv_backward", x.data_ptr(), dlogits.data_ptr(), weight.data_ptr(), dx.data_ptr(),
             dw.data_ptr(), S, H, W, C_, ws.data_ptr(), ws.numel() * 4, _stream())
    return dx, dw
