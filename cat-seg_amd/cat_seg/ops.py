"""Python mirror of the C ABI (include/catseg_hip.h): one thin wrapper per entry point.

Every wrapper takes device tensors, derives pointers / strides / dtypes, launches on
`torch.cuda.current_stream()` and raises RuntimeError on a non-zero status.  No
wrapper has a fallback: a missing library or device raises.
"""
from __future__ import annotations

from typing import Optional

import torch

import ctypes as C

from . import _lib as L
from ._lib import rowmap, IDENTITY


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


# Optional launch recorder (bench.py's roofline pass): when a list, every wrapped launch
# appends {"kernel", "flops", "bytes", "start", "end"} with HIP events recorded on the
# launch stream around it.
PROFILE: Optional[list] = None


class _rec:
    """flops = the work the launch executes; ref_flops = the reference's count for the same module
    (class padding rows, guidance halves recomputed per class and the
    ConvTranspose maps are algorithmic work the build skips); defaults to flops."""

    def __init__(self, kernel, flops=0, nbytes=0, ref_flops=None, shape=None):
        self.kernel, self.flops, self.nbytes, self.shape = kernel, flops, nbytes, shape
        self.ref_flops = flops if ref_flops is None else ref_flops

    def __enter__(self):
        if PROFILE is not None:
            _ACTIVE[0] = True
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record(torch.cuda.current_stream())
        return self

    def __exit__(self, *exc):
        if PROFILE is not None:
            _ACTIVE[0] = False
            if exc[0] is None:
                self.e1.record(torch.cuda.current_stream())
                PROFILE.append({"kernel": self.kernel, "flops": self.flops, "ref_flops": self.ref_flops,
                                "bytes": self.nbytes, "start": self.e0, "end": self.e1, "shape": self.shape})
        return False


_ACTIVE = [False]


def call(name, *args):
    """Launch through the C ABI; under PROFILE, launches without their own record get one."""
    if PROFILE is None or _ACTIVE[0]:
        return L.call(name, *args)
    with _rec(name[len("catseg_"):]):
        return L.call(name, *args)


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return L.F32
    if t.dtype == torch.bfloat16:
        return L.BF16
    if t.dtype == torch.float8_e4m3fn:
        return L.FP8
    raise TypeError(f"unsupported dtype {t.dtype}")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ld(t: torch.Tensor) -> int:
    assert t.dim() >= 2 and t.stride(-1) == 1, "row-major rows expected"
    return t.stride(-2)


def gemm(A, W, out, *, M=None, K=None, bias=None, act=L.ACT_NONE, alpha=1.0,
         add=None, addmap=None, add_ncols=None, res=None, res2=None, amap=None,
         lda=None, ldo=None, store=None):
    """out = act(A[amap(m)] . W^T + bias + add) * alpha + res + res2   (catseg_gemm)."""
    N = W.shape[0]
    K = K if K is not None else W.shape[1]
    M = M if M is not None else A.shape[0]
    a = L.GemmArgs()
    a.A, a.lda, a.amap = A.data_ptr(), lda if lda is not None else _ld(A), amap or IDENTITY
    a.W, a.ldw = W.data_ptr(), _ld(W)
    a.M, a.N, a.K = M, N, K
    a.bias = _p(bias)
    if add is not None:
        a.add, a.ld_add = add.data_ptr(), _ld(add)
        a.addmap = addmap or IDENTITY
        a.add_ncols = add_ncols if add_ncols is not None else N
    else:
        a.addmap = IDENTITY
    a.act, a.alpha = act, alpha
    if res is not None:
        a.res, a.ld_res = res.data_ptr(), _ld(res)
    if res2 is not None:
        a.res2, a.ld_res2 = res2.data_ptr(), _ld(res2)
    a.out = out.data_ptr()
    a.ldo = ldo if ldo is not None else (_ld(out) if store is None else 0)
    if store is not None:
        a.store_mode = 1
        a.cvt_k, a.cvt_hin, a.cvt_win, a.cvt_cout = store
    a.dtype_a, a.dtype_out = _dt(A), _dt(out)
    kname = "gemm_bf16" if a.dtype_a == L.BF16 else "gemm_f32"
    with _rec(kname, 2 * M * N * K, A.element_size() * (M * K + N * K) + out.element_size() * M * N,
              shape=(M, N, K)):
        call("catseg_gemm", a, _stream())
    return out


def quant_fp8_rows(x, q, scale, *, rows=None, cols=None):
    """Per-row e4m3 quantization (catseg_quant_fp8_rows): scale[r] = max|x[r]| / 448,
    q[r] = e4m3(x[r] / scale[r]).  q: torch.float8_e4m3fn, scale: fp32 [rows]."""
    rows = rows if rows is not None else x.shape[0]
    cols = cols if cols is not None else x.shape[1]
    with _rec("quant_fp8", 0, rows * cols * (x.element_size() + 1) + 4 * rows):
        call("catseg_quant_fp8_rows", x.data_ptr(), _dt(x), _ld(x), rows, cols, q.data_ptr(), _ld(q),
             scale.data_ptr(), _stream())
    return q, scale


def layernorm_fp8(x, gamma, beta, q, scale, *, rows=None, inmap=None, eps=1e-5):
    """LayerNorm straight to per-row e4m3 (catseg_layernorm_fp8)."""
    cols = gamma.shape[0]
    rows = rows if rows is not None else q.shape[0]
    with _rec("layernorm_fp8", 0, rows * cols * (x.element_size() + 1) + 4 * rows):
        call("catseg_layernorm_fp8", x.data_ptr(), _ld(x), inmap or IDENTITY, _dt(x), q.data_ptr(), _ld(q),
             scale.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rows, cols, eps, _stream())
    return q, scale


def gemm_fp8(A, sa, W, sw, out, *, bias=None, act=L.ACT_NONE, alpha=1.0, add=None, addmap=None,
             add_ncols=None, res=None, res2=None, amap=None, M=None):
    """out = epilogue((A8[amap(m)] . W8^T) * sa[amap(m)] * sw[n]) (catseg_gemm_fp8): the config-5 ViT GEMMs.
    A, W: torch.float8_e4m3fn rows; sa [M], sw [N] fp32 dequant scales."""
    N, K = W.shape
    M = M if M is not None else A.shape[0]
    a = L.GemmArgs()
    a.A, a.lda, a.amap = A.data_ptr(), _ld(A), amap or IDENTITY
    a.W, a.ldw = W.data_ptr(), _ld(W)
    a.M, a.N, a.K = M, N, K
    a.bias = _p(bias)
    if add is not None:
        a.add, a.ld_add = add.data_ptr(), _ld(add)
        a.addmap = addmap or IDENTITY
        a.add_ncols = add_ncols if add_ncols is not None else N
    else:
        a.addmap = IDENTITY
    a.act, a.alpha = act, alpha
    if res is not None:
        a.res, a.ld_res = res.data_ptr(), _ld(res)
    if res2 is not None:
        a.res2, a.ld_res2 = res2.data_ptr(), _ld(res2)
    a.out, a.ldo = out.data_ptr(), _ld(out)
    a.dtype_a, a.dtype_out = L.FP8, _dt(out)
    with _rec("gemm_fp8", 2 * M * N * K, M * K + N * K + out.element_size() * M * N):
        call("catseg_gemm_fp8", a, sa.data_ptr(), sw.data_ptr(), _stream())
    return out


def layernorm(x, gamma, beta, out, *, rows=None, inmap=None, eps=1e-5, cols=None):
    cols = cols if cols is not None else gamma.shape[0]
    rows = rows if rows is not None else out.shape[0]
    with _rec("layernorm", 0, rows * cols * (x.element_size() + out.element_size())):
      call("catseg_layernorm", x.data_ptr(), _ld(x), inmap or IDENTITY, _dt(x), out.data_ptr(), _ld(out), _dt(out),
         gamma.data_ptr(), beta.data_ptr(), rows, cols, eps, _stream())
    return out


def l2normalize(x, out, *, rows=None, cols=None, inmap=None, eps=1e-12):
    cols = cols if cols is not None else out.shape[-1]
    rows = rows if rows is not None else out.shape[0]
    with _rec("l2normalize", 0, rows * cols * (x.element_size() + out.element_size())):
        call("catseg_l2normalize", x.data_ptr(), _ld(x), inmap or IDENTITY, _dt(x), out.data_ptr(), _ld(out),
             _dt(out), rows, cols, eps, _stream())
    return out


def convert(x, out, *, rows=None, cols=None, inmap=None):
    cols = cols if cols is not None else out.shape[-1]
    rows = rows if rows is not None else out.shape[0]
    with _rec("convert", 0, rows * cols * (x.element_size() + out.element_size())):
        call("catseg_convert", x.data_ptr(), _ld(x), inmap or IDENTITY, _dt(x), out.data_ptr(), _ld(out), _dt(out),
             rows, cols, _stream())
    return out


def attention(q, k, v, out, *, n_seq, seq_len, n_heads, head_dim, scale, causal=False,
              mode=0, img_hw=(0, 0), window=0, shift=0):
    a = L.AttnArgs()
    a.q, a.k, a.v, a.ld_qkv = q.data_ptr(), k.data_ptr(), v.data_ptr(), _ld(q)
    assert _ld(k) == a.ld_qkv and _ld(v) == a.ld_qkv
    a.out, a.ld_out = out.data_ptr(), _ld(out)
    a.n_seq, a.seq_len, a.n_heads, a.head_dim = n_seq, seq_len, n_heads, head_dim
    a.scale, a.causal = scale, int(causal)
    a.mode, a.img_h, a.img_w, a.window, a.shift = mode, img_hw[0], img_hw[1], window, shift
    a.dtype = _dt(q)
    # algorithmic bytes: q, k, v read once, the output written once
    nbytes = n_seq * seq_len * n_heads * head_dim * (3 * q.element_size() + out.element_size())
    with _rec("attention_window" if mode == 1 else "attention", 4 * n_seq * n_heads * seq_len * seq_len * head_dim,
              nbytes):
        call("catseg_attention", a, _stream())
    return out


def swin_window_attention(x, ln, w_qkv, b_qkv, gqk, gmap, out, *, S, img_hw, window, shift, n_heads, head_dim,
                          scale, eps=1e-5):
    """Fused norm1 + q/k/v (+ guidance half) + shifted-window attention (catseg_swin_window_attention)."""
    a = L.SwinAttnArgs()
    a.x, a.ld_x = x.data_ptr(), _ld(x)
    a.ln_g, a.ln_b, a.eps = ln[0].data_ptr(), ln[1].data_ptr(), eps
    a.w_qkv, a.b_qkv = w_qkv.data_ptr(), b_qkv.data_ptr()
    a.gqk, a.ld_g, a.gmap = gqk.data_ptr(), _ld(gqk), gmap
    a.out, a.ld_out = out.data_ptr(), _ld(out)
    a.S, a.img_h, a.img_w, a.window, a.shift = S, img_hw[0], img_hw[1], window, shift
    a.n_heads, a.head_dim, a.scale, a.dtype = n_heads, head_dim, scale, _dt(x)
    R = S * img_hw[0] * img_hw[1]
    C = n_heads * head_dim
    L_ = window * window
    flops = 2 * R * C * 3 * C + 4 * R * L_ * C
    ref = 2 * R * (2 * 2 * C * C + C * C) + 4 * R * L_ * C        # q, k = Linear(2C -> C) on [x | g] (model.py:94-96)
    with _rec("swin_window_attention", flops, x.element_size() * R * 2 * C, ref_flops=ref):
        call("catseg_swin_window_attention", a, _stream())
    return out


def class_attention(x, ln, w_qkv, b_qkv, tg, y, *, B, T, HW, n_heads, head_dim, tg_bstride=0, n_pad=0,
                    k_pad=None, v_pad=None, eps=1e-5, attn_eps=1e-6, tgk_t=None):
    """Fused norm1 + q/k/v (+ text-guidance half) + linear class attention + residual
    (catseg_class_attention): y = x + LinearAttention(...).  tgk_t: the transposed k half of tg
    (class_attention_kt), made here when not given."""
    if tgk_t is None:
        tgk_t = class_attention_kt(tg if tg_bstride == 0 else tg[:B * T], T, 1 if tg_bstride == 0 else B)
    a = L.ClassAttnArgs()
    a.x, a.ld_x = x.data_ptr(), _ld(x)
    a.ln_g, a.ln_b, a.eps = ln[0].data_ptr(), ln[1].data_ptr(), eps
    a.w_qkv, a.b_qkv = w_qkv.data_ptr(), b_qkv.data_ptr()
    a.tg, a.ld_tg, a.tg_bstride = tg.data_ptr(), _ld(tg), tg_bstride
    a.n_pad, a.k_pad, a.v_pad, a.attn_eps = n_pad, _p(k_pad), _p(v_pad), attn_eps
    a.y, a.ld_y = y.data_ptr(), _ld(y)
    a.B, a.T, a.HW, a.n_heads, a.head_dim, a.dtype = B, T, HW, n_heads, head_dim, _dt(x)
    a.tgk_t, a.ld_tgk_t = tgk_t.data_ptr(), tgk_t.shape[-1]
    a.tgk_t_bstride = tgk_t.shape[-2] * tgk_t.shape[-1] if tgk_t.shape[0] > 1 else 0
    R = B * T * HW
    C = n_heads * head_dim
    flops = 2 * R * C * 3 * C + 4 * R * n_heads * head_dim * head_dim
    Rp = B * HW * (T + n_pad)                 # the reference pads T to pad_len (model.py:397-409)
    ref = 2 * Rp * (2 * 2 * C * C + C * C) + 4 * Rp * n_heads * head_dim * head_dim
    with _rec("class_attention", flops, x.element_size() * R * 2 * C, ref_flops=ref):
        call("catseg_class_attention", a, _stream())
    return y


def linear_attention(q, k, v, x, y, *, B, T, HW, n_heads, head_dim, n_pad=0, k_pad=None, v_pad=None, eps=1e-6):
    a = L.LinAttnArgs()
    a.q, a.k, a.v, a.ld_qkv = q.data_ptr(), k.data_ptr(), v.data_ptr(), _ld(q)
    a.x, a.y, a.ld_xy = x.data_ptr(), y.data_ptr(), _ld(x)
    assert _ld(y) == a.ld_xy
    a.B, a.T, a.HW, a.n_heads, a.head_dim = B, T, HW, n_heads, head_dim
    a.n_pad, a.k_pad, a.v_pad, a.eps = n_pad, _p(k_pad), _p(v_pad), eps
    a.dtype = _dt(q)
    with _rec("linear_attention", 4 * B * HW * T * n_heads * head_dim * head_dim):
        call("catseg_linear_attention", a, _stream())
    return y


def full_attention(qkv, x, y, *, B, T, HW, n_heads, head_dim, n_pad=0, k_pad=None, v_pad=None):
    """ATTENTION_TYPE "full" (FullAttention, model.py:300-320): y = x + softmax(q k^T / sqrt(d)) v over
    every pixel's T classes plus the n_pad learned padding tokens (model.py:397-410).
    qkv: class-major rows (b*T + t)*HW + p, [q | k | v].  catseg_class_seq_pack -> catseg_attention
    (mode 0, the MFMA flash kernel) -> catseg_class_seq_unpack_add."""
    C_ = n_heads * head_dim
    Lp = T + n_pad
    n_seq = B * HW
    packed = torch.empty(n_seq * Lp, 3 * C_, device=qkv.device, dtype=qkv.dtype)
    o = torch.empty(n_seq * Lp, C_, device=qkv.device, dtype=qkv.dtype)
    a = L.ClassSeqArgs()
    a.qkv, a.ld_qkv = qkv.data_ptr(), _ld(qkv)
    a.packed, a.ld_packed = packed.data_ptr(), _ld(packed)
    a.o, a.ld_o = o.data_ptr(), _ld(o)
    a.x, a.y, a.ld_xy = x.data_ptr(), y.data_ptr(), _ld(x)
    assert _ld(y) == a.ld_xy and x.dtype == y.dtype == qkv.dtype
    a.B, a.T, a.HW, a.C = B, T, HW, C_
    a.n_pad, a.k_pad, a.v_pad = n_pad, _p(k_pad), _p(v_pad)
    a.dtype = _dt(qkv)
    es = qkv.element_size()
    with _rec("class_seq_pack", 0, es * (B * T * HW + n_seq * Lp) * 3 * C_):
        call("catseg_class_seq_pack", a, _stream())
    attention(packed[:, :C_], packed[:, C_:2 * C_], packed[:, 2 * C_:], o, n_seq=n_seq, seq_len=Lp,
              n_heads=n_heads, head_dim=head_dim, scale=head_dim ** -0.5)
    with _rec("class_seq_unpack_add", 0, es * 3 * B * T * HW * C_):
        call("catseg_class_seq_unpack_add", a, _stream())
    return y


def _conv_args(src1, weight, out, S, H, W, c1, s1_slice_stride, s1_offset, src2, c2, s2_slice_stride, s2_offset,
               src2_div, bias, act, gn, stats, stats_cpg, addend, addend_div):
    a = L.ConvArgs()
    a.src1, a.s1_slice_stride, a.s1_offset, a.c1 = (src1.data_ptr(),
                                                   s1_slice_stride if s1_slice_stride is not None else H * W * c1,
                                                   s1_offset, c1)
    if src2 is not None:
        a.src2, a.s2_slice_stride, a.s2_offset, a.c2, a.src2_div = (src2.data_ptr(), s2_slice_stride or H * W * c2,
                                                                   s2_offset, c2, src2_div)
    else:
        a.src2_div = 1
    a.S, a.H, a.W = S, H, W
    a.weight, a.c_out = weight.data_ptr(), weight.shape[0]
    a.bias, a.act = _p(bias), act
    if gn is not None:
        mean, rstd, gamma, beta, cpg = gn
        a.gn_mean, a.gn_rstd, a.gn_gamma, a.gn_beta, a.gn_cpg = (mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
                                                                 beta.data_ptr(), cpg)
    a.out = _p(out)
    a.stats, a.stats_cpg = _p(stats), stats_cpg
    a.dtype = _dt(out if out is not None else weight)
    if addend is not None:
        assert addend.dtype == torch.float32 and addend.is_contiguous()
        a.addend, a.addend_slice_stride, a.addend_div = addend.data_ptr(), H * W * weight.shape[0], addend_div
    return a


def _conv_bytes(src1, weight, out, S, HW, c1, src2, c2, src2_div, addend, addend_div, out_px=None, out_ch=None):
    """Algorithmic bytes of a 3x3 conv launch: each input pixel read once (the per-image src2 and
    addend once per image), each output pixel written once, the weights read once."""
    out_px = HW if out_px is None else out_px
    out_ch = weight.shape[0] if out_ch is None else out_ch
    n = S * HW * c1 * src1.element_size() + weight.numel() * weight.element_size()
    if src2 is not None:
        n += (S // max(src2_div, 1)) * HW * c2 * src2.element_size()
    if out is not None:
        n += S * out_px * out_ch * out.element_size()
    if addend is not None:
        n += (S // max(addend_div, 1)) * out_px * out_ch * 4
    return n


def conv3x3(src1, weight, out, *, S, H, W, c1, s1_slice_stride=None, s1_offset=0,
            src2=None, c2=0, s2_slice_stride=0, s2_offset=0, src2_div=1,
            bias=None, act=L.ACT_NONE, gn=None, stats=None, stats_cpg=16, addend=None, addend_div=1):
    """3x3 / pad-1 conv over NHWC (catseg_conv3x3).  `stats` receives GroupNorm partials per
    conv3x3_stats_tile(...) pixels (query it with the same arguments to size the buffer)."""
    a = _conv_args(src1, weight, out, S, H, W, c1, s1_slice_stride, s1_offset, src2, c2, s2_slice_stride, s2_offset,
                   src2_div, bias, act, gn, stats, stats_cpg, addend, addend_div)
    ws_bytes = L.load().catseg_conv3x3_workspace(C.byref(a))
    ws = None
    if ws_bytes > 0:   # split-K scratch of small-grid convs (caching allocator; graph-capturable)
        ws = torch.empty(ws_bytes // 4, device=out.device, dtype=torch.float32)
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws_bytes
    with _rec("conv3x3", 2 * S * H * W * weight.shape[0] * weight.shape[1],
              _conv_bytes(src1, weight, out, S, H * W, c1, src2, c2, src2_div, addend, addend_div)):
        call("catseg_conv3x3", a, _stream())
    return out


def conv3x3_stats_tile(src1, weight, *, S, H, W, c1, s1_slice_stride=None, s1_offset=0,
                       src2=None, c2=0, s2_slice_stride=0, s2_offset=0, src2_div=1,
                       bias=None, act=L.ACT_NONE, gn=None, stats_cpg=16, addend=None, addend_div=1) -> int:
    """Pixels per GroupNorm partial of the conv kernel catseg_conv3x3 picks for these arguments."""
    a = _conv_args(src1, weight, None, S, H, W, c1, s1_slice_stride, s1_offset, src2, c2, s2_slice_stride, s2_offset,
                   src2_div, bias, act, gn, None, stats_cpg, addend, addend_div)
    a.stats = 1   # any non-null: the query only inspects whether statistics are requested
    return L.load().catseg_conv3x3_stats_tile(C.byref(a))


def conv3x3_partial(g, weight, out, *, B, H, W):
    """out[b][pix][co] = conv3x3 of g (NHWC [B][H][W][cin]) with fp32 weight [cout][9][cin], no bias:
    the per-image guidance half of a conv over [x | g] (catseg_conv3x3_partial)."""
    cout, k = weight.shape
    cin = k // 9
    assert g.shape[-1] == cin and out.dtype == torch.float32 and weight.dtype == torch.float32
    with _rec("conv3x3_partial", 2 * B * H * W * cout * k,
              B * H * W * (cin * g.element_size() + 4 * cout) + 4 * cout * k):
        call("catseg_conv3x3_partial", g.data_ptr(), B, H, W, cin, weight.data_ptr(), cout, out.data_ptr(), _dt(g),
             _stream())
    return out


def upconv3x3(src1, weight, out, *, S, H, W, c1, s1_slice_stride=None, gn=None, stats=None, stats_cpg=16,
              addend=None, addend_div=1, ref_convt_out=None, ref_guid=0):
    """ConvTranspose2d(k=2, s=2) + conv3x3 folded into one 4-parity conv over the ConvTranspose
    input (catseg_upconv3x3): src1 [S][H][W][c1] -> out [S][2H][2W][c_out/4] with the composite
    weight [4 * cout][9 * c1] (CatSegEngine._upconv_weights) and the parity-layout addend
    (upconv_addend).  `stats` receives [S][4 * H*W / upconv3x3_stats_tile()][cout/16][2]."""
    a = _conv_args(src1, weight, out, S, H, W, c1, s1_slice_stride, 0, None, 0, 0, 0, 1, None, L.ACT_NONE, gn,
                   stats, stats_cpg, addend, addend_div)
    cout = weight.shape[0] // 4
    # reference: ConvTranspose2d(c1 -> m, k=2, s=2) then conv3x3 over [up (m) | guidance (ref_guid)]
    m = ref_convt_out or 0
    ref = (2 * S * H * W * 4 * m * c1 + 2 * S * 4 * H * W * cout * 9 * (m + ref_guid)) if m else None
    nbytes = _conv_bytes(src1, weight, out, S, H * W, c1, None, 0, 1, addend, addend_div, out_px=4 * H * W,
                         out_ch=cout)
    with _rec("upconv3x3", 2 * S * H * W * weight.shape[0] * 4 * c1, nbytes, ref_flops=ref):
        call("catseg_upconv3x3", a, _stream())
    return out


def upconv3x3_stats_tile() -> int:
    return L.load().catseg_upconv3x3_stats_tile()


def upconv_addend(g, weight, tap_bias, out, *, B, H2, W2):
    """catseg_upconv_addend: the guidance half of the Up conv on the 2H x 2W grid (fp32 weight
    [cout][9 * cin]) + the ConvTranspose bias through the in-image taps (tap_bias [9][cout]), in
    the parity layout [B][H2/2 * W2/2][4 * cout] of upconv3x3's addend."""
    cout, k = weight.shape
    cin = k // 9
    assert g.shape[-1] == cin and out.dtype == torch.float32 and weight.dtype == torch.float32
    with _rec("conv3x3_partial", 2 * B * H2 * W2 * cout * k,
              B * H2 * W2 * (cin * g.element_size() + 4 * cout) + 4 * cout * k, ref_flops=0):   # in upconv3x3's reference count
        call("catseg_upconv_addend", g.data_ptr(), B, H2, W2, cin, weight.data_ptr(), _p(tap_bias), cout,
             out.data_ptr(), _dt(g), _stream())
    return out


def conv_tile_rows() -> int:
    return L.load().catseg_conv_tile_rows()


def groupnorm_stats(partials, S, tiles, groups, tile_count, mean, rstd, eps=1e-5):
    with _rec("groupnorm_stats", 0, 4 * (S * tiles * groups * 2 + 2 * S * groups)):
        call("catseg_groupnorm_stats", partials.data_ptr(), S, tiles, groups, tile_count, eps, mean.data_ptr(),
             rstd.data_ptr(), _stream())


def groupnorm_relu(x, y, *, S, HW, C, cpg, mean, rstd, gamma, beta):
    call("catseg_groupnorm_relu", x.data_ptr(), y.data_ptr(), S, HW, C, cpg, mean.data_ptr(), rstd.data_ptr(),
         gamma.data_ptr(), beta.data_ptr(), _dt(x), _stream())
    return y


def conv3x3_head(x, *, B, T, H, W, C, weight, bias, out, T_out, classes=None, gn=None):
    if gn is None:
        call("catseg_conv3x3_head", x.data_ptr(), B, T, H, W, C, weight.data_ptr(), bias, _p(classes), T_out,
             out.data_ptr(), _dt(x), _stream())
    else:
        mean, rstd, gamma, beta, cpg = gn
        # one output channel: 9 taps x C MACs per pixel; x read once, the fp32 logit plane written once
        with _rec("conv3x3_head_gn", 2 * B * T * H * W * C * 9, B * T * H * W * (C * x.element_size() + 4)):
            call("catseg_conv3x3_head_gn", x.data_ptr(), B, T, H, W, C, weight.data_ptr(), bias, mean.data_ptr(),
                 rstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), cpg, _p(classes), T_out, out.data_ptr(),
                 _dt(x), _stream())
    return out


def corr_embed(corr, *, t_stride, b_stride, B, T, H, W, weight, bias, out, classes=None):
    hidden = weight.shape[0]
    # Conv2d(1, hidden, 7, pad 3): 49 MACs per output channel; each fp32 cost slice read once, X written once
    with _rec("corr_embed", 2 * B * T * H * W * hidden * 49, B * T * H * W * (4 + hidden * out.element_size())):
        call("catseg_corr_embed", corr.data_ptr(), t_stride, b_stride, _p(classes), B, T, H, W, weight.data_ptr(),
             bias.data_ptr(), hidden, out.data_ptr(), _dt(out), _stream())
    return out


def topk_classes(corr, *, t_stride, b_stride, B, T, HW, k, out):
    """The k classes of largest max-over-pixels cost per image, sorted (catseg_topk_classes)."""
    ws = torch.empty(B * T, device=corr.device, dtype=torch.float32)
    call("catseg_topk_classes", corr.data_ptr(), t_stride, b_stride, B, T, HW, k, out.data_ptr(), ws.data_ptr(),
         _stream())
    return out


def transpose_rows(x, out, *, rows, batch=1, in_bstride=0):
    """out[b][c][r] = x[b*in_bstride + r][c] (r < rows), zero for rows <= r < out.shape[-1]
    (catseg_transpose_rows); x (., cols) with any row stride, out (batch, cols, ld) contiguous."""
    cols = out.shape[-2]
    call("catseg_transpose_rows", x.data_ptr(), _ld(x), rows, cols, batch, in_bstride, out.data_ptr(),
         out.shape[-1], _dt(x), _stream())
    return out


def class_attention_kt(tg, T, batch=1):
    """The k half of the class-attention text guidance transposed per image: (batch, 128, Tp),
    Tp = T rounded up to 16, zero past T (catseg_class_attention's tgk_t)."""
    Tp = (T + 15) // 16 * 16
    out = torch.empty(batch, tg.shape[1] // 2, Tp, device=tg.device, dtype=tg.dtype)
    return transpose_rows(tg[:, tg.shape[1] // 2:], out, rows=T, batch=batch, in_bstride=T if batch > 1 else 0)


def gather_rows(x, idx, out):
    call("catseg_gather_rows", x.data_ptr(), _ld(x), idx.data_ptr(), idx.numel(), out.shape[-1], out.data_ptr(),
         _ld(out), _dt(x), _stream())
    return out


def fill(out, value):
    call("catseg_fill_f32", out.data_ptr(), out.numel(), value, _stream())
    return out


def preprocess_im2col(raw, sizes, *, mean, std, res, patch, out):
    B, _, Hp, Wp = raw.shape
    # the padded fp32 canvas read once, the patch matrix (with its zero K padding) written once
    G = res // patch
    with _rec("preprocess_im2col", 0, raw.numel() * 4 + B * G * G * _ld(out) * out.element_size()):
        call("catseg_preprocess_im2col", raw.data_ptr(), sizes.data_ptr(), B, Hp, Wp, mean.data_ptr(),
             std.data_ptr(), res, patch, out.data_ptr(), _ld(out), _dt(out), _stream())
    return out


def vit_embed(patches, cls, pos, gamma, beta, out, *, B, G2, width):
    # fp32 patch rows read, the fp32 residual stream written (pos / cls / LN params are L2-resident)
    with _rec("vit_embed", 0, 4 * width * (B * G2 + B * (G2 + 1))):
        call("catseg_vit_embed", patches.data_ptr(), cls.data_ptr(), pos.data_ptr(), gamma.data_ptr(),
             beta.data_ptr(), B, G2, width, out.data_ptr(), _stream())
    return out


def bicubic_resize(grid, S_in, D, out, S_out):
    call("catseg_bicubic_resize", grid.data_ptr(), S_in, D, out.data_ptr(), S_out, _stream())
    return out


def postprocess(logits, out, *, crop=None):
    B, T, h, w = logits.shape
    H, W = out.shape[-2:]
    ch, cw = crop if crop is not None else (h, w)
    with _rec("postprocess", 0, 4 * B * T * (ch * cw + H * W)):
        call("catseg_postprocess", logits.data_ptr(), B, T, h, w, ch, cw, out.data_ptr(), H, W, _stream())
    return out


def resize_bilinear(x, out, *, crop=None):
    """Bilinear (align_corners=False) of fp32 planes [B][T][h][w] cropped to `crop` -> out [B][T][H][W]."""
    B, T, h, w = x.shape
    H, W = out.shape[-2:]
    ch, cw = crop if crop is not None else (h, w)
    with _rec("resize_bilinear", 0, 4 * (B * T * (ch * cw + H * W))):
        call("catseg_resize_bilinear", x.data_ptr(), B, T, h, w, ch, cw, out.data_ptr(), H, W, _stream())
    return out


def avgpool_rows(x, out, *, S, H, W, C, pool):
    """nn.AvgPool2d(pool) over [S][H][W][C] rows -> out [S][H/ph][W/pw][C] (catseg_avgpool_rows)."""
    ph, pw = pool
    with _rec("avgpool_rows", 0, x.element_size() * S * C * (H * W + (H // ph) * (W // pw))):
        call("catseg_avgpool_rows", x.data_ptr(), S, H, W, C, ph, pw, out.data_ptr(), _dt(x), _stream())
    return out


def upsample_add_rows(xp, x, *, S, Hp, Wp, C, H, W):
    """x += bilinear_align_corners(xp -> H x W) on [S][.][.][C] rows (catseg_upsample_add_rows)."""
    assert xp.dtype == x.dtype
    with _rec("upsample_add_rows", 0, x.element_size() * S * C * (Hp * Wp + 2 * H * W)):
        call("catseg_upsample_add_rows", xp.data_ptr(), S, Hp, Wp, C, x.data_ptr(), H, W, _dt(x), _stream())
    return x


def sliding_crops(raw, sizes, out, *, out_res, kernel, stride):
    """Unfold crops + global crop of each image, fp32 0-255 (catseg_sliding_crops)."""
    N, _, Hc, Wc = raw.shape
    with _rec("sliding_crops", 0, 4 * out.numel()):
        call("catseg_sliding_crops", raw.data_ptr(), sizes.data_ptr(), N, Hc, Wc, out_res, kernel, stride,
             out.data_ptr(), _stream())
    return out


def sliding_merge(logits, out, *, kernel, stride, out_res):
    """(Fold(sigmoid(interp tiles))/count + interp(global)) / 2 (catseg_sliding_merge)."""
    N, T = out.shape[:2]
    h, w = logits.shape[-2:]
    with _rec("sliding_merge", 0, 4 * (logits.numel() + out.numel())):
        call("catseg_sliding_merge", logits.data_ptr(), N, T, h, w, kernel, stride, out_res, out.data_ptr(),
             _stream())
    return out


def token_embed(tokens, tok_emb, pos, out):
    n, ctx = tokens.shape
    call("catseg_token_embed", tokens.data_ptr(), n, ctx, tok_emb.data_ptr(), pos.data_ptr(), tok_emb.shape[1],
         out.data_ptr(), _stream())
    return out


def eot_gather(x, tokens, out):
    n, ctx = tokens.shape
    call("catseg_eot_gather", x.data_ptr(), tokens.data_ptr(), n, ctx, out.shape[-1], out.data_ptr(), _stream())
    return out


def _rows_epi(out, bias, add, addmap, add_ncols, act, res, res2, store):
    e = L.RowsEpi()
    e.bias = _p(bias)
    e.addmap = addmap or IDENTITY
    if add is not None:
        e.add, e.ld_add = add.data_ptr(), _ld(add)
        e.add_ncols = add_ncols if add_ncols is not None else add.shape[-1]
    e.act = act
    if res is not None:
        e.res, e.ld_res = res.data_ptr(), _ld(res)
    if res2 is not None:
        e.res2, e.ld_res2 = res2.data_ptr(), _ld(res2)
    e.out = out.data_ptr()
    if store is None:
        e.ldo = _ld(out)
    else:
        e.store_mode = 1
        e.cvt_k, e.cvt_hin, e.cvt_win, e.cvt_cout = store
    return e


def rows_gemm(x, w, out, *, ln=None, eps=1e-5, bias=None, add=None, addmap=None, add_ncols=None,
              act=L.ACT_NONE, res=None, res2=None, store=None, M=None):
    """out = epi(LN?(x) . w^T) over 128-wide rows (catseg_rows_gemm)."""
    M = M if M is not None else x.shape[0]
    N = w.shape[0]
    if x.dtype == torch.float32 and out.dtype == torch.float32:
        # fp32 (config 2): catseg_layernorm + catseg_gemm (same epilogue order: bias, add, act, res, res2)
        # run at ~76 TF/s on these K = 128 GEMMs against the fused row kernel's ~55 (64-row workgroups,
        # 4 MFMAs per k-step per wave)
        a = x
        if ln is not None:
            a = torch.empty(M, w.shape[1], device=x.device, dtype=torch.float32)
            layernorm(x, ln[0], ln[1], a, rows=M, eps=eps)
        ncols = add_ncols if add_ncols is not None else (add.shape[-1] if add is not None else None)
        gemm(a, w, out, M=M, bias=bias, add=add, addmap=addmap, add_ncols=ncols, act=act, res=res, res2=res2,
             store=store)
        return out
    e = _rows_epi(out, bias, add, addmap, add_ncols, act, res, res2, store)
    g, b = (ln if ln is not None else (None, None))
    with _rec("rows_gemm", 2 * M * N * w.shape[1], x.element_size() * M * (w.shape[1] + N)):
        call("catseg_rows_gemm", x.data_ptr(), _ld(x), M, _p(g), _p(b), eps, w.data_ptr(), N, e, _dt(x), _stream())
    return out


def convt64_gn(x, w, out, *, HW, gn, bias, store):
    """out = ConvT_k2(relu(GN(x))) over 64-channel rows (catseg_convt64_gn, bf16)."""
    mean, rstd, gamma, beta, cpg = gn
    e = _rows_epi(out, bias, None, None, None, L.ACT_NONE, None, None, store)
    M = x.shape[0]
    with _rec("convt64_gn", 2 * M * w.shape[0] * w.shape[1], x.element_size() * M * (w.shape[1] + w.shape[0])):
        call("catseg_convt64_gn", x.data_ptr(), M, HW, mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
             beta.data_ptr(), cpg, w.data_ptr(), w.shape[0], e, _stream())
    return out


def rows_mlp(y, w1, b1, w2, out, *, ln, b2=None, act=L.ACT_GELU, res=None, res2=None, eps=1e-5, M=None,
             ref_rows=None):
    """out = act(LN(y) . w1^T + b1) . w2^T + b2 + res + res2 (catseg_rows_mlp).  ref_rows: the
    reference's row count when it computes padded rows (the class MLP, model.py:413)."""
    M = M if M is not None else y.shape[0]
    hidden = w1.shape[0]
    if y.dtype == torch.float32 and out.dtype == torch.float32:
        # fp32 (config 2): LayerNorm + two GEMM launches beat the fused row kernel, whose one workgroup
        # per 64 rows re-stages the 2 x 256 KB of fp32 weights per hidden chunk at one wave per SIMD
        # (1.67 ms per launch at 345,600 rows); the hidden tensor round-trips HBM instead (M x 512 fp32)
        h = torch.empty(M, w1.shape[1], device=y.device, dtype=torch.float32)
        layernorm(y, ln[0], ln[1], h, rows=M, eps=eps)
        u = torch.empty(M, hidden, device=y.device, dtype=torch.float32)
        gemm(h, w1, u, M=M, bias=b1, act=act)
        gemm(u, w2, out, M=M, bias=b2, res=res, res2=res2)
        return out
    e = _rows_epi(out, b2, None, None, None, L.ACT_NONE, res, res2, None)
    ref = 4 * ref_rows * hidden * w1.shape[1] if ref_rows else None
    with _rec("rows_mlp", 4 * M * hidden * w1.shape[1], y.element_size() * M * 2 * w1.shape[1], ref_flops=ref):
        call("catseg_rows_mlp", y.data_ptr(), _ld(y), M, ln[0].data_ptr(), ln[1].data_ptr(), eps, w1.data_ptr(),
             b1.data_ptr(), hidden, act, w2.data_ptr(), e, _dt(y), _stream())
    return out


def swin_proj_mlp(attn, x, w_proj, b_proj, w1, b1, w2, b2, out, *, ln, eps=1e-5):
    """out = x1 + GELU(LN(x1) . w1^T + b1) . w2^T + b2, x1 = x + attn . w_proj^T + b_proj (bf16 rows of
    128; the Swin block after its window attention, catseg_swin_proj_mlp).  out may be x."""
    M, C_ = x.shape
    hidden = w1.shape[0]
    flops = 2 * M * C_ * C_ + 4 * M * hidden * C_
    with _rec("swin_proj_mlp", flops, x.element_size() * M * 3 * C_):
        call("catseg_swin_proj_mlp", attn.data_ptr(), _ld(attn), x.data_ptr(), _ld(x), M, w_proj.data_ptr(),
             b_proj.data_ptr(), ln[0].data_ptr(), ln[1].data_ptr(), eps, w1.data_ptr(), b1.data_ptr(), hidden,
             w2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), _stream())
    return out


def bce_onehot_loss(logits, targets, ignore_value=255):
    """The training branch's loss (cat_seg_model.py:189-203) on the device: BCE-with-logits of
    logits (B, T, h, w) fp32 bilinearly upsampled to targets' (B, H, W) size, one-hot targets
    (ignore_value -> zeros), mean over every element.  Returns a 0-d fp32 device tensor (no grad)."""
    B, T, h, w = logits.shape
    Bt, H, W = targets.shape
    assert Bt == B and logits.dtype == torch.float32 and logits.is_contiguous()
    tg = targets.to(torch.int32).contiguous()
    ws = torch.empty(B * H, device=logits.device, dtype=torch.float64)
    loss = torch.empty((), device=logits.device, dtype=torch.float32)
    with _rec("bce_onehot_loss", 0, logits.numel() * 4 + tg.numel() * 4):
        call("catseg_bce_onehot_loss", logits.data_ptr(), B, T, h, w, tg.data_ptr(), H, W, ignore_value, ws.data_ptr(),
             loss.data_ptr(), _stream())
    return loss


def bce_onehot_loss_backward(logits, targets, ignore_value=255, grad_loss=None):
    """d bce_onehot_loss / d logits on the device (catseg_bce_onehot_loss_backward): what autograd
    computes for cat_seg_model.py:192-203 (BCE mean backward through the bilinear upsample's
    backward), times grad_loss (0-d device fp32 tensor, None = 1).  Returns (B, T, h, w) fp32."""
    B, T, h, w = logits.shape
    Bt, H, W = targets.shape
    assert Bt == B and logits.dtype == torch.float32 and logits.is_contiguous()
    tg = targets.to(torch.int32).contiguous()
    gl = None if grad_loss is None else grad_loss.to(device=logits.device, dtype=torch.float32).contiguous()
    ws = torch.empty(B * T * H * w, device=logits.device, dtype=torch.float32)
    grad = torch.empty_like(logits)
    with _rec("bce_onehot_loss_backward", 0, logits.numel() * 8 + tg.numel() * 4 + ws.numel() * 8):
        call("catseg_bce_onehot_loss_backward", logits.data_ptr(), B, T, h, w, tg.data_ptr(), H, W, ignore_value,
             None if gl is None else gl.data_ptr(), ws.data_ptr(), grad.data_ptr(), _stream())
    return grad


class BCEOneHotLoss(torch.autograd.Function):
    """bce_onehot_loss with its HIP backward: loss = BCEOneHotLoss.apply(logits, targets, ignore);
    loss.backward() fills logits.grad through catseg_bce_onehot_loss_backward (targets get none)."""

    @staticmethod
    def forward(ctx, logits, targets, ignore_value=255):
        logits = logits.contiguous()
        ctx.save_for_backward(logits, targets)
        ctx.ignore_value = ignore_value
        return bce_onehot_loss(logits, targets, ignore_value)

    @staticmethod
    def backward(ctx, grad_loss):
        logits, targets = ctx.saved_tensors
        return bce_onehot_loss_backward(logits, targets, ctx.ignore_value, grad_loss), None, None


def semseg_confusion(probs, gt, conf, n_invalid, *, num_classes, ignore_label=255, clamp_pred=-1):
    """conf += bincount((N+1) * argmax(probs) + gt') on the device (catseg_semseg_confusion).
    probs (T, H, W) fp32, gt (H, W) int32, conf ((N+1)^2,) int64, n_invalid (1,) int64."""
    T, H, W = probs.shape
    assert probs.is_contiguous() and gt.is_contiguous() and gt.shape == (H, W) and gt.dtype == torch.int32
    assert conf.dtype == torch.int64 and conf.numel() == (num_classes + 1) ** 2 and n_invalid.dtype == torch.int64
    with _rec("semseg_confusion", 0, probs.numel() * 4 + gt.numel() * 4):
        call("catseg_semseg_confusion", probs.data_ptr(), T, H, W, gt.data_ptr(), num_classes, ignore_label,
             clamp_pred, conf.data_ptr(), n_invalid.data_ptr(), _stream())
    return conf
