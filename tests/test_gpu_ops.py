"""Per-kernel parity of the HIP C-ABI entry points against fp32/fp64 PyTorch and the
oracle's functions, on seeded inputs.  Marked gpu: runs on the MI355X box only."""
import math

import pytest
import torch
import torch.nn.functional as F

from cat_seg import ops
from cat_seg import _lib as L
from cat_seg._lib import rowmap
from oracle import catseg_oracle as O

pytestmark = pytest.mark.gpu

dev = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


def close(got, ref, atol, rtol=0.0, what=""):
    got = got.float().cpu()
    ref = ref.float().cpu()
    err = (got - ref).abs().max().item()
    tol = atol + rtol * ref.abs().max().item()
    assert err <= tol, f"{what}: max abs err {err:.3e} > {tol:.3e}"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    L.require_gpu()


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(300, 384, 128), (577, 1024, 1024), (33, 64, 96), (130, 32, 288), (1, 384, 128)])
def test_gemm_plain(dt, M, N, K):
    A = rnd(M, K, seed=1)
    W = rnd(N, K, seed=2) / math.sqrt(K)
    b = rnd(N, seed=3)
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    ops.gemm(A.to(dev, dt), W.to(dev, dt), out, bias=b.to(dev))
    ref = A.to(dt).double() @ W.to(dt).double().T + b.double()
    close(out, ref, atol=2e-5 if dt == torch.float32 else 1e-3, what="gemm")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dt):
    M, N, K = 2 * 3 * 20, 384, 128      # rows (b=2, t=3, p=20)
    A = rnd(M, K, seed=4)
    W = rnd(N, K, seed=5) / math.sqrt(K)
    b = rnd(N, seed=6)
    add = rnd(2 * 20, 256, seed=7)       # per (b, p), first 256 columns
    res = rnd(M, N, seed=8)
    res2 = rnd(M, N, seed=9)
    amap = rowmap(d1=1, m1=M, s1=1)
    gmap = rowmap(d1=3 * 20, s1=20, d2=1, m2=20, s2=1)
    outs = {}
    for act in (L.ACT_NONE, L.ACT_RELU, L.ACT_GELU, L.ACT_QUICKGELU):
        out = torch.empty(M, N, device=dev, dtype=dt)
        ops.gemm(A.to(dev, dt), W.to(dev, dt), out, bias=b.to(dev), act=act, add=add.to(dev, dt), addmap=gmap,
                 add_ncols=256, res=res.to(dev, dt), res2=res2.to(dev, dt), amap=amap)
        v = A.to(dt).double() @ W.to(dt).double().T + b.double()
        rows = torch.arange(M)
        arow = (rows // 60) * 20 + rows % 20
        v[:, :256] += add.to(dt).double()[arow]
        fn = {L.ACT_NONE: lambda x: x, L.ACT_RELU: F.relu, L.ACT_GELU: F.gelu,
              L.ACT_QUICKGELU: lambda x: x * torch.sigmoid(1.702 * x)}[act]
        ref = fn(v) + res.to(dt).double() + res2.to(dt).double()
        close(out, ref, atol=2e-5 if dt == torch.float32 else 3e-2, rtol=0 if dt == torch.float32 else 1e-2,
              what=f"gemm act {act}")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_convtranspose_store(dt):
    S, H, Wd, cin, cout, k = 3, 6, 5, 64, 48, 2
    x = rnd(S, cin, H, Wd, seed=10)
    w = rnd(cin, cout, k, k, seed=11) / 8
    b = rnd(cout, seed=12)
    ref = F.conv_transpose2d(x.to(dt).double(), w.to(dt).double(), b.double(), stride=k)   # (S, cout, kH, kW)
    A = x.permute(0, 2, 3, 1).reshape(S * H * Wd, cin)
    Wg = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
    out = torch.empty(S * H * k * Wd * k, cout, device=dev, dtype=dt)
    ops.gemm(A.to(dev, dt).contiguous(), Wg.to(dev, dt).contiguous(), out, bias=b.repeat(k * k).to(dev),
             store=(k, H, Wd, cout))
    got = out.reshape(S, H * k, Wd * k, cout).permute(0, 3, 1, 2)
    close(got, ref, atol=1e-5 if dt == torch.float32 else 2e-2, what="convT")


@pytest.mark.parametrize("cout,k", [(256, 2), (128, 4)])
def test_gemm_convtranspose_store_pipelined(cout, k):
    """The guidance upsamplers' shapes (cat_seg_model.py:81-82, ViT-L/14 hooks: 1024 -> 256 / 128
    channels, k = 2 / 4): ConvTranspose scatter from the pipelined kernel's 8-wide epilogue."""
    S, H, Wd, cin = 2, 24, 24, 1024
    x = rnd(S, cin, H, Wd, seed=20)
    w = rnd(cin, cout, k, k, seed=21) / 32
    b = rnd(cout, seed=22)
    ref = F.conv_transpose2d(x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double(), b.double(), stride=k)
    A = x.permute(0, 2, 3, 1).reshape(S * H * Wd, cin)
    Wg = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
    out = torch.full((S * H * k * Wd * k, cout), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.gemm(A.to(dev, torch.bfloat16).contiguous(), Wg.to(dev, torch.bfloat16).contiguous(), out,
             bias=b.repeat(k * k).to(dev), store=(k, H, Wd, cout))
    got = out.reshape(S, H * k, Wd * k, cout).permute(0, 3, 1, 2)
    close(got, ref, atol=2e-2, rtol=1e-2, what=f"convT pipelined cout {cout} k {k}")


@pytest.mark.parametrize("variant", [0, 15, 17, 20, 24])
def test_gemm_epilogue_prefetch(variant):
    """The lean gemm3 epilogue with the next round's residual rows in flight and the bias loaded once
    (tuning knob epi_prefetch 1, the default) equals the per-round form (0) bit for bit: bias + fp32 residual (out-proj /
    fc2) and bias + QuickGELU to bf16 (fc1), ragged M."""
    M, K, N = 1210, 512, 512
    A = rnd(M, K, seed=44).to(dev, torch.bfloat16)
    W = (rnd(N, K, seed=45) / math.sqrt(K)).to(dev, torch.bfloat16)
    b = rnd(N, seed=46).to(dev)
    res = rnd(M, N, seed=47).to(dev)
    lib = L.load()
    outs = {}
    try:
        L.tune("gemm_variant", variant)
        for pf in (0, 1):
            L.tune("epi_prefetch", pf)
            o1 = torch.full((M, N), float("nan"), device=dev)
            ops.gemm(A, W, o1, bias=b, res=res)
            o2 = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            ops.gemm(A, W, o2, bias=b, act=L.ACT_QUICKGELU)
            torch.cuda.synchronize()
            outs[pf] = (o1, o2)
    finally:
        L.tune("gemm_variant", 0)
        L.tune("epi_prefetch", 1)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert not torch.isnan(outs[1][0]).any()


@pytest.mark.parametrize("variant", [1, 15, 17, 19, 20, 24])
def test_gemm_pipelined_variants(variant):
    """Every LDS-DMA pipelined bf16 tile (gemm.hip gemm3_kernel) against fp64: ragged M
    (sliver tile), a CLS-dropping row map, bias + QuickGELU + fp32 residual epilogue."""
    B, L_, K, N = 3, 401, 512, 512
    M = B * (L_ - 1)                                      # 1200 rows: 4 full 256-tiles + a sliver
    A = rnd(B * L_, K, seed=40)
    W = rnd(N, K, seed=41) / math.sqrt(K)
    b = rnd(N, seed=42)
    res = rnd(M, N, seed=43)
    amap = rowmap(d1=L_ - 1, s1=L_, d2=1, m2=L_ - 1, s2=1, off=1)
    arow = A.reshape(B, L_, K)[:, 1:].reshape(-1, K)
    lib = L.load()
    try:
        L.tune("gemm_variant", variant)
        for act, odt in ((L.ACT_QUICKGELU, torch.bfloat16), (L.ACT_NONE, torch.float32)):
            out = torch.full((M, N), float("nan"), device=dev, dtype=odt)
            r = res.to(dev, odt)
            ops.gemm(A.to(dev, torch.bfloat16), W.to(dev, torch.bfloat16), out, M=M, bias=b.to(dev), act=act,
                     res=r, amap=amap)
            v = arow.to(torch.bfloat16).double() @ W.to(torch.bfloat16).double().T + b.double()
            if act == L.ACT_QUICKGELU:
                v = v * torch.sigmoid(1.702 * v)
            ref = v + r.double().cpu()
            close(out, ref, atol=1e-4 if odt == torch.float32 else 2e-2, rtol=0 if odt == torch.float32 else 1e-2,
                  what=f"gemm3 variant {variant} act {act}")
    finally:
        L.tune("gemm_variant", 0)


# ----------------------------------------------------------------------------- fp8 (config 5)
def _quant_ref(x):
    """Per-row e4m3 quantization as catseg_quant_fp8_rows defines it (fp32 arithmetic, RNE)."""
    x = x.float()
    amax = x.abs().amax(dim=1).clamp_min(1e-30)
    inv = torch.tensor(448.0) / amax
    q = (x * inv[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q, amax / 448.0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(1, 8), (37, 1024), (300, 4096), (5, 264)])
def test_quant_fp8_rows_bit_exact(dt, rows, cols):
    """catseg_quant_fp8_rows vs torch's RNE float8_e4m3fn conversion: identical bytes and scales;
    a zero row and a row with a single huge value included."""
    x = rnd(rows, cols, seed=70, scale=3.0)
    x[0, :4] = torch.tensor([1e4, -2.0, 0.5, 3.0])
    if rows > 2:
        x[2] = 0.0
    x = x.to(dt)
    q = torch.empty(rows, cols, device=dev, dtype=torch.float8_e4m3fn)
    sc = torch.empty(rows, device=dev, dtype=torch.float32)
    ops.quant_fp8_rows(x.to(dev), q, sc)
    qr, sr = _quant_ref(x)
    assert torch.equal(sc.cpu(), sr), (sc.cpu() - sr).abs().max()
    assert torch.equal(q.cpu().view(torch.uint8), qr.view(torch.uint8))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_fp8(dt):
    """catseg_layernorm_fp8 (LN in fp32, then per-row e4m3) vs fp64 LayerNorm through a
    CLS-dropping row map: scales to fp32 rounding, values within one e4m3 rounding step."""
    B, L_, C = 3, 7, 1024
    x = rnd(B * L_, C, seed=80, scale=2.0) + 0.5
    g = rnd(C, seed=81) + 1.0
    b = rnd(C, seed=82) * 0.1
    M = B * (L_ - 1)
    amap = rowmap(d1=L_ - 1, s1=L_, d2=1, m2=L_ - 1, s2=1, off=1)
    q = torch.empty(M, C, device=dev, dtype=torch.float8_e4m3fn)
    sc = torch.empty(M, device=dev)
    ops.layernorm_fp8(x.to(dev, dt), g.to(dev), b.to(dev), q, sc, rows=M, inmap=amap)
    xr = x.to(dt).double().reshape(B, L_, C)[:, 1:].reshape(-1, C)
    ln = F.layer_norm(xr, (C,), g.double(), b.double(), eps=1e-5)
    sref = ln.abs().amax(dim=1) / 448
    close(sc, sref, atol=0, rtol=1e-5, what="layernorm_fp8 scale")
    deq = q.cpu().double() * sc.cpu().double()[:, None]
    err = (deq - ln).abs()
    tol = ln.abs() * 2.0 ** -4 + sref[:, None] * 2.0 ** -9 * 1.01
    assert (err <= tol).all(), (err - tol).max()


@pytest.mark.parametrize("variant", [0, 1, 15, 17, 19, 20, 21, 23, 24])
def test_gemm_fp8_variants(variant):
    """catseg_gemm_fp8 (block-scaled K=128 MFMA over e4m3 rows) against fp64 products of the
    dequantized operands: ragged M with a CLS-dropping row map, bias + QuickGELU / fp32 residual."""
    B, L_, K, N = 3, 401, 1024, 768
    M = B * (L_ - 1)
    A = rnd(B * L_, K, seed=50)
    W = rnd(N, K, seed=51) / math.sqrt(K)
    b = rnd(N, seed=52)
    res = rnd(M, N, seed=53)
    qa, sa = _quant_ref(A)
    qw, sw = _quant_ref(W)
    amap = rowmap(d1=L_ - 1, s1=L_, d2=1, m2=L_ - 1, s2=1, off=1)
    ad = (qa.double() * sa.double()[:, None]).reshape(B, L_, K)[:, 1:].reshape(-1, K)
    wd = qw.double() * sw.double()[:, None]
    lib = L.load()
    try:
        L.tune("gemm_fp8_variant", variant)
        for act, odt in ((L.ACT_QUICKGELU, torch.bfloat16), (L.ACT_NONE, torch.float32)):
            out = torch.full((M, N), float("nan"), device=dev, dtype=odt)
            r = res.to(dev, odt)
            ops.gemm_fp8(qa.to(dev), sa.to(dev), qw.to(dev), sw.to(dev), out, M=M, bias=b.to(dev), act=act,
                         res=r, amap=amap)
            v = ad @ wd.T + b.double()
            if act == L.ACT_QUICKGELU:
                v = v * torch.sigmoid(1.702 * v)
            ref = v + r.double().cpu()
            close(out, ref, atol=1e-4 if odt == torch.float32 else 2e-2, rtol=0 if odt == torch.float32 else 1e-2,
                  what=f"gemm_fp8 variant {variant} act {act}")
    finally:
        L.tune("gemm_fp8_variant", 0)


@pytest.mark.parametrize("variant", [15, 17, 20])
def test_gemm_fp8_epilogue_prefetch(variant):
    """fp8 GEMM with the lean prefetching epilogue (per-column scales once, per-row scale and fp32
    residual of the next round in flight; epi_prefetch 1, default) vs the per-round form, with a
    CLS-dropping row map: bias + residual and bias + QuickGELU.  The dequant multiply and the bias add
    may contract into one FMA in one form and not the other: an ulp of the fp32 result."""
    B, L_, K, N = 3, 401, 1024, 768
    M = B * (L_ - 1)
    qa, sa = _quant_ref(rnd(B * L_, K, seed=54))
    qw, sw = _quant_ref(rnd(N, K, seed=55) / math.sqrt(K))
    b = rnd(N, seed=56).to(dev)
    res = rnd(M, N, seed=57).to(dev)
    amap = rowmap(d1=L_ - 1, s1=L_, d2=1, m2=L_ - 1, s2=1, off=1)
    lib = L.load()
    outs = {}
    try:
        L.tune("gemm_fp8_variant", variant)
        for pf in (0, 1):
            L.tune("epi_prefetch", pf)
            o1 = torch.full((M, N), float("nan"), device=dev)
            ops.gemm_fp8(qa.to(dev), sa.to(dev), qw.to(dev), sw.to(dev), o1, M=M, bias=b, res=res, amap=amap)
            o2 = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            ops.gemm_fp8(qa.to(dev), sa.to(dev), qw.to(dev), sw.to(dev), o2, M=M, bias=b, act=L.ACT_QUICKGELU,
                         amap=amap)
            torch.cuda.synchronize()
            outs[pf] = (o1, o2)
    finally:
        L.tune("gemm_fp8_variant", 0)
        L.tune("epi_prefetch", 1)
    d1 = (outs[0][0] - outs[1][0]).abs()                  # O(1) values: a few fp32 ulps of the sum
    assert d1.max().item() <= 4e-6, d1.max().item()
    d2 = (outs[0][1].float() - outs[1][1].float()).abs()
    assert d2.max().item() <= 2 ** -7 * outs[0][1].float().abs().max().item()     # a bf16 ulp at most
    assert not torch.isnan(outs[1][0]).any()


def test_gemm_fp8_vit_shapes_vs_bf16():
    """The ViT-L/14 block shapes (M = 8 x 577) through the automatic fp8 tile choice: the
    dequantized-operand product to fp32 accuracy, and within e4m3 error of the bf16 GEMM."""
    M = 8 * 577
    for N, K in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        A = rnd(M, K, seed=N + K)
        W = rnd(N, K, seed=N + K + 1) / math.sqrt(K)
        qa = torch.empty(M, K, device=dev, dtype=torch.float8_e4m3fn)
        sa = torch.empty(M, device=dev)
        qw = torch.empty(N, K, device=dev, dtype=torch.float8_e4m3fn)
        sw = torch.empty(N, device=dev)
        ops.quant_fp8_rows(A.to(dev, torch.bfloat16), qa, sa)
        ops.quant_fp8_rows(W.to(dev), qw, sw)
        out = torch.empty(M, N, device=dev)
        ops.gemm_fp8(qa, sa, qw, sw, out)
        ref = (qa.cpu().double() * sa.cpu().double()[:, None]) @ (qw.cpu().double() * sw.cpu().double()[:, None]).T
        close(out, ref, atol=1e-4, what=f"gemm_fp8 {M}x{N}x{K}")
        exact = A.to(torch.bfloat16).double() @ W.double().T
        rel = ((out.cpu().double() - exact).norm() / exact.norm()).item()
        assert rel < 0.05, f"fp8 vs exact relative error {rel}"


def test_gemm_amap_cls_drop():
    B, L_, C = 2, 5, 16
    A = rnd(B * L_, C, seed=13)
    W = rnd(8, C, seed=14)
    out = torch.empty(B * (L_ - 1), 8, device=dev)
    ops.gemm(A.to(dev), W.to(dev), out, M=B * (L_ - 1), amap=rowmap(d1=L_ - 1, s1=L_, d2=1, m2=L_ - 1, s2=1, off=1))
    ref = A.reshape(B, L_, C)[:, 1:].reshape(-1, C).double() @ W.double().T
    close(out, ref, atol=1e-5, what="amap")


# ----------------------------------------------------------------------------- norms
@pytest.mark.parametrize("cols", [128, 768, 1024, 96])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_l2(cols, dt):
    x = rnd(77, cols, seed=15) * 3 + 0.5
    g, b = rnd(cols, seed=16) + 1, rnd(cols, seed=17)
    out = torch.empty(77, cols, device=dev, dtype=dt)
    ops.layernorm(x.to(dev), g.to(dev), b.to(dev), out)
    close(out, F.layer_norm(x.double(), (cols,), g.double(), b.double(), 1e-5),
          atol=2e-5 if dt == torch.float32 else 2e-2, what="LN")
    ops.l2normalize(x.to(dev), out)
    close(out, F.normalize(x.double(), dim=-1), atol=1e-6 if dt == torch.float32 else 4e-3, what="l2")


@pytest.mark.parametrize("rows", [4616, 2308, 2049])
def test_layernorm_pipelined_rows(rows):
    """The ViT's ln_1 / ln_2 / ln_post shape (fp32 rows of 1024 -> bf16): the persistent pipelined
    kernel (tuning knob ln_variant 0, default) equals the one-row-per-wave kernel bit for bit and
    meets fp64 LayerNorm to bf16 rounding (model_vpt.py:156-162)."""
    cols = 1024
    x = rnd(rows, cols, seed=18) * 3 + 0.5
    x[::97, :7] *= 40.0                     # CLIP-like outlier channels
    g, b = rnd(cols, seed=19) + 1, rnd(cols, seed=20)
    lib = L.load()
    outs = []
    for v in (0, 1):
        L.tune("ln_variant", v)
        o = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
        ops.layernorm(x.to(dev), g.to(dev), b.to(dev), o)
        outs.append(o)
    L.tune("ln_variant", 0)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    close(outs[0], F.layer_norm(x.double(), (cols,), g.double(), b.double(), 1e-5), atol=3e-2, rtol=1e-2, what="LN pipe")


# ----------------------------------------------------------------------------- attention
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("L_,H,causal", [(577, 4, False), (77, 2, True), (50, 3, False), (64, 2, False),
                                         (129, 2, False), (14, 12, True)])
def test_attention_dense(dt, L_, H, causal):
    B, d = 2, 64
    qkv = rnd(B * L_, 3 * H * d, seed=18) * 2
    out = torch.empty(B * L_, H * d, device=dev, dtype=dt)
    q = qkv.to(dev, dt)
    ops.attention(q[:, :H * d], q[:, H * d:2 * H * d], q[:, 2 * H * d:], out, n_seq=B, seq_len=L_, n_heads=H,
                  head_dim=d, scale=d ** -0.5, causal=causal)
    x = qkv.to(dt).double().reshape(B, L_, 3, H, d).permute(2, 0, 3, 1, 4)
    s = (x[0] @ x[1].transpose(-1, -2)) * d ** -0.5
    if causal:
        s = s + torch.full((L_, L_), float("-inf")).triu(1).double()
    ref = (torch.softmax(s, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B * L_, H * d)
    close(out, ref, atol=2e-5 if dt == torch.float32 else 1.5e-2, what="attn")


@pytest.mark.parametrize("L_,spike", [(577, None), (50, None), (129, None), (577, 300), (577, 5)])
def test_attention_dense_log2_scaled_q(L_, spike):
    """Mode 2 (the ViT blocks: q rows carry scale * log2(e), folded into the q projection; the
    running max enters the S MFMA as its accumulator): vs fp64 softmax attention of the unscaled q,
    including a spike key that forces the defer-max rescale in block 0 / a middle block."""
    B, H, d = 2, 4, 64
    qkv = rnd(B * L_, 3 * H * d, seed=31) * 2
    if spike is not None:
        qkv[spike, H * d:H * d + d] += 4 * qkv[200, :d]
    c = d ** -0.5 * 1.4426950408889634
    q = qkv.clone()
    q[:, :H * d] *= c
    qb = q.to(dev, torch.bfloat16)
    out = torch.empty(B * L_, H * d, device=dev, dtype=torch.bfloat16)
    ops.attention(qb[:, :H * d], qb[:, H * d:2 * H * d], qb[:, 2 * H * d:], out, n_seq=B, seq_len=L_,
                  n_heads=H, head_dim=d, scale=0.0, mode=2)
    x = q.to(torch.bfloat16).double().reshape(B, L_, 3, H, d).permute(2, 0, 3, 1, 4)
    s = (x[0] @ x[1].transpose(-1, -2)) * math.log(2.0)
    ref = (torch.softmax(s, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B * L_, H * d)
    close(out, ref, atol=1.5e-2, what=f"attn mode 2 L={L_} spike={spike}")
    with pytest.raises(RuntimeError):     # fp32 / causal are not mode-2 shapes
        ops.attention(qb[:, :H * d].float(), qb[:, H * d:2 * H * d].float(), qb[:, 2 * H * d:].float(),
                      out.float(), n_seq=B, seq_len=L_, n_heads=H, head_dim=d, scale=0.0, mode=2)


@pytest.mark.parametrize("variant", [7])
def test_attention_dense_tilings(variant):
    """The generic tiling of the dense path (tuning knob attn_variant 7) == the default ViT kernel."""
    B, L_, H, d = 2, 577, 4, 64
    q = (rnd(B * L_, 3 * H * d, seed=19) * 2).to(dev, torch.bfloat16)
    args = (q[:, :H * d], q[:, H * d:2 * H * d], q[:, 2 * H * d:])
    kw = dict(n_seq=B, seq_len=L_, n_heads=H, head_dim=d, scale=d ** -0.5)
    ref = torch.empty(B * L_, H * d, device=dev, dtype=torch.bfloat16)
    ops.attention(*args, ref, **kw)
    lib = L.load()
    try:
        L.tune("attn_variant", variant)
        out = torch.empty_like(ref)
        ops.attention(*args, out, **kw)
    finally:
        L.tune("attn_variant", 0)
    close(out, ref, atol=8e-3, what=f"attention tiling {variant}")


@pytest.mark.parametrize("spike_key", [5, 300, 576])
def test_attention_dense_defer_max_rescale(spike_key):
    """The ViT kernel's defer-max branch (cdna_hip_programming.md rule 26): one key made to
    dominate some queries' scores so the running max jumps by far more than the threshold in the
    block holding it (block 0, a middle block, the 1-key tail block); every other query keeps
    its ordinary scores.  Checked against fp64 over the full tensor, and the rescale threshold's
    two extremes (always / first block only) must agree with the default to rounding."""
    B, L_, H, d = 1, 577, 2, 64
    qkv = rnd(B * L_, 3 * H * d, seed=23) * 2
    k_cols = slice(H * d, 2 * H * d)
    for qrow in (3, 200, 576):                        # k[spike] ~ 12 * q[qrow] for head 0 only
        qkv[spike_key, H * d:H * d + d] += 12 * qkv[qrow, :d] / 3
    q = qkv.to(dev, torch.bfloat16)
    out = torch.empty(B * L_, H * d, device=dev, dtype=torch.bfloat16)
    ops.attention(q[:, :H * d], q[:, k_cols], q[:, 2 * H * d:], out, n_seq=B, seq_len=L_, n_heads=H,
                  head_dim=d, scale=d ** -0.5)
    x = qkv.to(torch.bfloat16).double().reshape(B, L_, 3, H, d).permute(2, 0, 3, 1, 4)
    s = (x[0] @ x[1].transpose(-1, -2)) * d ** -0.5
    if spike_key >= 64:                               # the jump the branch must handle
        assert s[0, 0].max(-1).values.max() - s[0, 0, :, :64].max() > 30
    ref = (torch.softmax(s, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B * L_, H * d)
    close(out, ref, atol=1.5e-2, what=f"attn defer-max spike at key {spike_key}")
    alt = torch.empty_like(out)
    try:
        L.tune("attn_variant", 7)                     # the exact-max kernel (rescales every block)
        ops.attention(q[:, :H * d], q[:, k_cols], q[:, 2 * H * d:], alt, n_seq=B, seq_len=L_, n_heads=H,
                      head_dim=d, scale=d ** -0.5)
    finally:
        L.tune("attn_variant", 0)
    close(out, alt, atol=8e-3, what="defer-max vs exact-max kernel")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shift", [0, 6])
def test_attention_swin_windows(dt, shift):
    S, Hh, Ww, ws, nh, hd = 3, 24, 24, 12, 4, 32
    D = nh * hd
    qkv = rnd(S * Hh * Ww, 3 * D, seed=19) * 2
    out = torch.empty(S * Hh * Ww, D, device=dev, dtype=dt)
    q = qkv.to(dev, dt)
    ops.attention(q[:, :D], q[:, D:2 * D], q[:, 2 * D:], out, n_seq=S * 4, seq_len=ws * ws, n_heads=nh,
                  head_dim=hd, scale=hd ** -0.5, mode=1, img_hw=(Hh, Ww), window=ws, shift=shift)
    # reference: roll -> partition -> masked softmax attention -> reverse -> roll back (model.py:185-219)
    x = qkv.to(dt).double().reshape(S, Hh, Ww, 3 * D)
    if shift:
        x = torch.roll(x, (-shift, -shift), (1, 2))
    xw = O.window_partition(x, ws).reshape(-1, ws * ws, 3, nh, hd).permute(2, 0, 3, 1, 4)
    a = (xw[0] * hd ** -0.5) @ xw[1].transpose(-1, -2)
    if shift:
        m = O.shift_mask(Hh, Ww, ws, shift).double()
        a = (a.view(S, 4, nh, ws * ws, ws * ws) + m.unsqueeze(1).unsqueeze(0)).view(-1, nh, ws * ws, ws * ws)
    o = (torch.softmax(a, -1) @ xw[2]).transpose(1, 2).reshape(-1, ws, ws, D)
    o = O.window_reverse(o, ws, Hh, Ww)
    if shift:
        o = torch.roll(o, (shift, shift), (1, 2))
    close(out, o.reshape(S * Hh * Ww, D), atol=2e-5 if dt == torch.float32 else 1.5e-2, what="swin attn")


# ----------------------------------------------------------------------------- linear attention
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T,n_pad", [(20, 236), (150, 106), (256, 0), (37, 0)])
def test_linear_attention(dt, T, n_pad):
    B, HW, D = 2, 9, 128
    qkv = rnd(B * T * HW, 3 * D, seed=20)
    x = rnd(B * T * HW, D, seed=21)
    kp, vp = rnd(D, seed=22), rnd(D, seed=23)
    qd, xd = qkv.to(dev, dt), x.to(dev, dt)
    y = torch.empty_like(xd)
    ops.linear_attention(qd[:, :D], qd[:, D:2 * D], qd[:, 2 * D:], xd, y, B=B, T=T, HW=HW, n_heads=4, head_dim=32,
                         n_pad=n_pad, k_pad=kp.to(dev), v_pad=vp.to(dev))
    z = qkv.to(dt).double().reshape(B, T, HW, 3, 4, 32).permute(3, 0, 2, 1, 4, 5).reshape(3, B * HW, T, 4, 32)
    q, k, v = z[0], z[1], z[2]
    if n_pad:
        k = torch.cat([k, kp.double().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
        v = torch.cat([v, vp.double().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
    o = O.linear_attention(q, k, v).reshape(B, HW, T, D).permute(0, 2, 1, 3).reshape(-1, D)
    close(y, x.to(dt).double() + o, atol=2e-5 if dt == torch.float32 else 3e-2, what="linattn")


# ----------------------------------------------------------------------------- full class attention
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T,n_pad", [(20, 236), (150, 106), (256, 0), (37, 0), (10, 6)])
def test_full_class_attention(dt, T, n_pad):
    """ATTENTION_TYPE "full": pack -> MFMA flash attention (mode 0, head_dim 32) -> unpack + residual,
    against FullAttention (model.py:300-320) in fp64 over the padded class axis."""
    B, HW, D = 2, 9, 128
    qkv = rnd(B * T * HW, 3 * D, seed=24)
    x = rnd(B * T * HW, D, seed=25)
    kp, vp = rnd(D, seed=26), rnd(D, seed=27)
    qd, xd = qkv.to(dev, dt), x.to(dev, dt)
    y = torch.empty_like(xd)
    ops.full_attention(qd, xd, y, B=B, T=T, HW=HW, n_heads=4, head_dim=32, n_pad=n_pad, k_pad=kp.to(dev),
                       v_pad=vp.to(dev))
    z = qkv.to(dt).double().reshape(B, T, HW, 3, 4, 32).permute(3, 0, 2, 1, 4, 5).reshape(3, B * HW, T, 4, 32)
    q, k, v = z[0], z[1], z[2]
    if n_pad:
        k = torch.cat([k, kp.to(dt).double().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
        v = torch.cat([v, vp.to(dt).double().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
    o = O.full_attention(q, k, v).reshape(B, HW, T, D).permute(0, 2, 1, 3).reshape(-1, D)
    close(y, x.to(dt).double() + o, atol=2e-5 if dt == torch.float32 else 3e-2, what="fullattn")


@pytest.mark.parametrize("T,n_pad,per_image", [(150, 106, False), (20, 236, False), (256, 0, True), (37, 0, False),
                                               (33, 5, True)])
def test_class_attention_fused(T, n_pad, per_image):
    """catseg_class_attention == norm1 + AttentionLayer q/k/v (+ text guidance) + LinearAttention
    + residual (model.py:397-413, 338-354, 256-286) against an fp64 restatement on the same bf16
    inputs, and against the unfused rows_gemm + linear_attention pair.  per_image: guidance rows
    gathered per image (the top-k path, tg_bstride = T)."""
    B, HW, D = 2, 24, 128
    dt = torch.bfloat16
    R = B * T * HW
    X = rnd(R, D, seed=61, scale=2.0).to(dev, dt)
    g1, b1 = (1 + rnd(D, seed=62, scale=0.2)).to(dev), rnd(D, seed=63, scale=0.2).to(dev)
    W = (rnd(3 * D, D, seed=64) / math.sqrt(D)).to(dev, dt)
    bias = rnd(3 * D, seed=65, scale=0.1).to(dev)
    ntg = B * T if per_image else T
    tg = rnd(ntg, 2 * D, seed=66, scale=0.5).to(dev, dt)
    kp, vp = rnd(D, seed=67).to(dev), rnd(D, seed=68).to(dev)
    y = torch.empty_like(X)
    ops.class_attention(X, (g1, b1), W, bias, tg, y, B=B, T=T, HW=HW, n_heads=4, head_dim=32,
                        tg_bstride=T if per_image else 0, n_pad=n_pad, k_pad=kp, v_pad=vp)
    # fp64 restatement on the same bf16 inputs
    xf = X.double().cpu()
    h = F.layer_norm(xf, (D,), g1.double().cpu(), b1.double().cpu())
    qkv = h @ W.double().cpu().T + bias.double().cpu()
    tgf = tg.double().cpu()
    if per_image:
        tg_rows = tgf.reshape(B, T, 1, 2 * D).expand(B, T, HW, 2 * D).reshape(R, 2 * D)
    else:
        tg_rows = tgf.reshape(1, T, 1, 2 * D).expand(B, T, HW, 2 * D).reshape(R, 2 * D)
    qkv[:, :2 * D] += tg_rows
    z = qkv.reshape(B, T, HW, 3, 4, 32).permute(3, 0, 2, 1, 4, 5).reshape(3, B * HW, T, 4, 32)
    q, k, v = z[0], z[1], z[2]
    if n_pad:
        k = torch.cat([k, kp.double().cpu().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
        v = torch.cat([v, vp.double().cpu().reshape(1, 1, 4, 32).expand(B * HW, n_pad, 4, 32)], 1)
    o = O.linear_attention(q, k, v).reshape(B, HW, T, D).permute(0, 2, 1, 3).reshape(-1, D)
    ref = xf + o
    err = (y.double().cpu() - ref).abs()
    assert err.max().item() < 5e-2 and err.mean().item() < 5e-3, (err.max().item(), err.mean().item())
    # the unfused bf16 pair (q/k/v rounded to bf16 in HBM) on the same inputs
    qkv_d = torch.empty(R, 3 * D, device=dev, dtype=dt)
    tmap = rowmap(d1=HW) if per_image else rowmap(d1=HW, m1=T)
    ops.rows_gemm(X, W, qkv_d, ln=(g1, b1), bias=bias, add=tg, addmap=tmap, add_ncols=2 * D)
    y2 = torch.empty_like(X)
    ops.linear_attention(qkv_d[:, :D], qkv_d[:, D:2 * D], qkv_d[:, 2 * D:], X, y2, B=B, T=T, HW=HW, n_heads=4,
                         head_dim=32, n_pad=n_pad, k_pad=kp, v_pad=vp)
    e2 = (y.float() - y2.float()).abs()
    assert e2.max().item() < 5e-2 and e2.mean().item() < 5e-3, (e2.max().item(), e2.mean().item())
    # a second launch computes the same bits (no atomics, fixed reduction order)
    y3 = torch.empty_like(X)
    ops.class_attention(X, (g1, b1), W, bias, tg, y3, B=B, T=T, HW=HW, n_heads=4, head_dim=32,
                        tg_bstride=T if per_image else 0, n_pad=n_pad, k_pad=kp, v_pad=vp)
    torch.cuda.synchronize()
    assert torch.equal(y, y3)


# ----------------------------------------------------------------------------- conv + GN
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_dual_source_gn(dt):
    B, T, H, W, c1, c2, co = 2, 3, 16, 16, 48, 16, 32
    S = B * T
    x1 = rnd(S, c1, H, W, seed=24)
    x2 = rnd(B, c2, H, W, seed=25)
    w = rnd(co, c1 + c2, 3, 3, seed=26) / 8
    xin = torch.cat([x1, x2.repeat_interleave(T, 0)], 1)
    ref = F.conv2d(xin.to(dt).double(), w.to(dt).double(), padding=1)
    a1 = x1.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    a2 = x2.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    wk = w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
    out = torch.empty(S * H * W, co, device=dev, dtype=dt)
    tiles = H * W // ops.conv_tile_rows()
    st = torch.empty(S * tiles * (co // 16) * 2, device=dev)
    ops.conv3x3(a1, wk, out, S=S, H=H, W=W, c1=c1, src2=a2, c2=c2, src2_div=T, stats=st)
    got = out.reshape(S, H, W, co).permute(0, 3, 1, 2)
    tol = 1e-5 if dt == torch.float32 else 3e-2
    close(got, ref, atol=tol, what="conv")
    mean = torch.empty(S * (co // 16), device=dev)
    rstd = torch.empty_like(mean)
    ops.groupnorm_stats(st, S, tiles, co // 16, ops.conv_tile_rows() * 16, mean, rstd)
    g = ref.reshape(S, co // 16, -1)
    close(mean, g.mean(-1).reshape(-1), atol=1e-5 if dt == torch.float32 else 1e-3, what="gn mean")
    close(rstd, (1 / torch.sqrt(g.var(-1, unbiased=False) + 1e-5)).reshape(-1), atol=0, rtol=1e-4 if dt == torch.float32 else 2e-2,
          what="gn rstd")
    # GN+ReLU prologue feeding a second conv, and the head conv with GN on load
    gam, bet = rnd(co, seed=27) + 1, rnd(co, seed=28)
    w2 = rnd(co, co, 3, 3, seed=29) / 8
    y1 = F.relu(F.group_norm(ref, co // 16, gam.double(), bet.double(), 1e-5))
    ref2 = F.conv2d(y1, w2.to(dt).double(), padding=1)
    out2 = torch.empty_like(out)
    ops.conv3x3(out, w2.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt), out2, S=S, H=H, W=W, c1=co,
                gn=(mean, rstd, gam.to(dev), bet.to(dev), 16))
    close(out2.reshape(S, H, W, co).permute(0, 3, 1, 2), ref2, atol=1e-4 if dt == torch.float32 else 8e-2,
          what="conv gn prologue")
    z = torch.empty_like(out)
    ops.groupnorm_relu(out, z, S=S, HW=H * W, C=co, cpg=16, mean=mean, rstd=rstd, gamma=gam.to(dev), beta=bet.to(dev))
    close(z.reshape(S, H, W, co).permute(0, 3, 1, 2), y1, atol=1e-4 if dt == torch.float32 else 2e-2,
          rtol=0 if dt == torch.float32 else 1e-2, what="gn relu")
    hw_ = rnd(1, co, 3, 3, seed=30) / 8
    logits = torch.full((B, T + 2, H, W), 7.0, device=dev)
    cls = torch.tensor([[0, 2, 4], [1, 3, 0]], dtype=torch.int32)
    ops.conv3x3_head(out, B=B, T=T, H=H, W=W, C=co, weight=hw_[0].permute(1, 2, 0).reshape(-1).contiguous().to(dev),
                     bias=0.25, out=logits, T_out=T + 2, classes=cls.to(dev), gn=(mean, rstd, gam.to(dev), bet.to(dev), 16))
    rh = F.conv2d(y1, hw_.double(), torch.tensor([0.25]).double(), padding=1).reshape(B, T, H, W)
    for bi in range(B):
        for t in range(T):
            close(logits[bi, cls[bi, t]], rh[bi, t], atol=1e-4 if dt == torch.float32 else 5e-2, what="head")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("S,H,c1,co", [(2, 24, 768, 128), (3, 48, 256, 32), (1, 24, 512, 128)])
def test_conv3x3_splitk_guidance_projection(dt, S, H, c1, co):
    """The per-image guidance projections (model.py:616-630: conv3x3 + bias + ReLU on res3/4/5):
    small grids over long K run split-K (fp32 partials + reduce) when the op provides the
    workspace; equal to fp64 conv2d."""
    lib = L.load()
    x = rnd(S, c1, H, H, seed=81)
    w = rnd(co, c1, 3, 3, seed=82) / math.sqrt(9 * c1)
    b = rnd(co, seed=83) * 0.1
    ref = F.relu(F.conv2d(x.to(dt).double(), w.to(dt).double(), b.double(), padding=1))
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    wk = w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
    out = torch.empty(S * H * H, co, device=dev, dtype=dt)
    a = ops._conv_args(xd, wk, out, S, H, H, c1, None, 0, None, 0, 0, 0, 1, b.to(dev), L.ACT_RELU, None, None, 16,
                       None, 1)
    assert lib.catseg_conv3x3_workspace(ops.C.byref(a)) > 0      # these shapes do split
    ops.conv3x3(xd, wk, out, S=S, H=H, W=H, c1=c1, bias=b.to(dev), act=L.ACT_RELU)
    close(out.reshape(S, H, H, co).permute(0, 3, 1, 2), ref, atol=1e-5 if dt == torch.float32 else 2e-2,
          rtol=0 if dt == torch.float32 else 1e-2, what="split-K conv")


@pytest.mark.parametrize("c1,c2,co,H", [(96, 32, 64, 48), (48, 16, 32, 96), (64, 0, 64, 48), (32, 0, 32, 96)])
def test_conv3x3_ring_guidance_split(c1, c2, co, H):
    """The decoder convs on the ring kernel (bf16): conv over [x | g] (g per image, repeated over
    T; model.py:551-554) computed as conv(x) + the per-image fp32 partial conv of g
    (catseg_conv3x3_partial) joined as the epilogue addend, vs fp64 and vs the unsplit path;
    GroupNorm partial statistics included."""
    B, T, W = 2, 3, H
    S = B * T
    dt = torch.bfloat16
    x1 = rnd(S, c1, H, W, seed=71)
    x2 = rnd(B, max(c2, 1), H, W, seed=72)[:, :c2]
    w = rnd(co, c1 + c2, 3, 3, seed=73) / 8
    xin = torch.cat([x1, x2.repeat_interleave(T, 0)], 1) if c2 else x1
    ref = F.conv2d(xin.to(dt).double(), w.to(dt).double(), padding=1)
    a1 = x1.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    out = torch.empty(S * H * W, co, device=dev, dtype=dt)
    if c2:
        a2 = x2.permute(0, 2, 3, 1).contiguous().to(dev, dt)
        wx = w[:, :c1].permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
        wg = w[:, c1:].to(dt).float().permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev)
        part = torch.empty(B * H * W, co, device=dev)
        ops.conv3x3_partial(a2, wg, part, B=B, H=H, W=W)
        refp = F.conv2d(x2.to(dt).double(), w[:, c1:].to(dt).double(), padding=1)
        close(part.reshape(B, H, W, co).permute(0, 3, 1, 2), refp, atol=1e-4, what="partial conv")
        kw, wc = dict(S=S, H=H, W=W, c1=c1, addend=part, addend_div=T), wx
    else:
        kw, wc = dict(S=S, H=H, W=W, c1=c1), w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
    tile = ops.conv3x3_stats_tile(a1, wc, **kw)
    tiles = H * W // tile
    st = torch.empty(S * tiles * (co // 16) * 2, device=dev)
    ops.conv3x3(a1, wc, out, stats=st, **kw)
    got = out.reshape(S, H, W, co).permute(0, 3, 1, 2).double().cpu()
    err = (got - ref).abs() - 2.0 ** -8 * ref.abs()
    assert err.max().item() <= 1e-5, err.max().item()
    # the one-barrier-per-chunk rings (tuning knob ring_onebar 1, default) equal the two-barrier form bit for bit
    L.load()
    out1, st1 = torch.empty_like(out), torch.empty_like(st)
    try:
        L.tune("ring_onebar", 0)
        ops.conv3x3(a1, wc, out1, stats=st1, **kw)
        torch.cuda.synchronize()
    finally:
        L.tune("ring_onebar", 1)
    assert torch.equal(out1, out) and torch.equal(st1, st)
    mean = torch.empty(S * (co // 16), device=dev)
    rstd = torch.empty_like(mean)
    ops.groupnorm_stats(st, S, tiles, co // 16, tile * 16, mean, rstd)
    g = ref.reshape(S, co // 16, -1)
    close(mean, g.mean(-1).reshape(-1), atol=1e-4, what="gn mean")
    close(rstd, (1 / torch.sqrt(g.var(-1, unbiased=False) + 1e-5)).reshape(-1), atol=0, rtol=2e-3, what="gn rstd")
    if c2:
        # the unsplit path (guidance channels read per class) on the same inputs
        out2 = torch.empty_like(out)
        wk = w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
        ops.conv3x3(a1, wk, out2, S=S, H=H, W=W, c1=c1, src2=a2, c2=c2, src2_div=T)
        e2 = (out.float() - out2.float()).abs() - 2.0 ** -7 * out2.float().abs()   # one bf16 rounding apart
        assert e2.max().item() < 1e-2, e2.max().item()


# ----------------------------------------------------------------------------- small ops
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_corr_embed_topk(dt):
    B, T, H, W, hid = 2, 40, 24, 24, 128
    corr = rnd(T, B * H * W, seed=31) * 0.2
    w = rnd(hid, 1, 7, 7, seed=32) / 7
    b = rnd(hid, seed=33)
    k = 16
    cls = torch.empty(B, k, device=dev, dtype=torch.int32)
    cd = corr.to(dev)
    ops.topk_classes(cd, t_stride=B * H * W, b_stride=H * W, B=B, T=T, HW=H * W, k=k, out=cls)
    m = corr.reshape(T, B, H * W).max(-1)[0].T   # (B, T)
    ref_cls = m.topk(k, -1)[1]
    assert torch.equal(torch.sort(cls.cpu().long(), -1)[0], torch.sort(ref_cls, -1)[0])
    X = torch.empty(B * k * H * W, hid, device=dev, dtype=dt)
    ops.corr_embed(cd, t_stride=B * H * W, b_stride=H * W, B=B, T=k, H=H, W=W, weight=w.reshape(hid, 49).to(dev),
                   bias=b.to(dev), out=X, classes=cls)
    c = corr.reshape(T, B, H, W).permute(1, 0, 2, 3)
    sel = torch.stack([c[bi, cls[bi].cpu().long()] for bi in range(B)])   # (B, k, H, W)
    ref = F.conv2d(sel.reshape(B * k, 1, H, W).double(), w.double(), b.double(), padding=3)
    close(X.reshape(B * k, H, W, hid).permute(0, 3, 1, 2), ref, atol=1e-5 if dt == torch.float32 else 2e-2,
          what="corr_embed")
    if dt == torch.bfloat16:
        # both bf16 kernels (MFMA hi/lo split, VALU) land within bf16 output rounding of fp64
        lib = L.load()
        try:
            for mode in (1, 0):
                L.tune("corr_mfma", mode)
                X.zero_()
                ops.corr_embed(cd, t_stride=B * H * W, b_stride=H * W, B=B, T=k, H=H, W=W,
                               weight=w.reshape(hid, 49).to(dev), bias=b.to(dev), out=X, classes=cls)
                got = X.reshape(B * k, H, W, hid).permute(0, 3, 1, 2).double().cpu()
                err = (got - ref).abs() - 2.0 ** -8 * ref.abs()
                assert err.max().item() <= 1e-6, (mode, err.max().item())
        finally:
            L.tune("corr_mfma", 1)


@pytest.mark.parametrize("B,T,HW,k", [(4, 847, 576, 256), (3, 459, 576, 256), (2, 300, 37, 256), (1, 2048, 64, 1000)])
def test_topk_classes_exact(B, T, HW, k):
    """model.py:694-702: max over (P, H, W) of the cost per class, then the k largest.  The kernel
    returns them sorted by (max descending, class index ascending) -- the set torch.topk selects,
    in a fixed order (the class aggregation is permutation-equivariant and the final scatter is by
    index).  Exact, including forced ties (one shared maximum for a run of classes)."""
    corr = rnd(T, B * HW, seed=171)
    c3 = corr.reshape(T, B, HW)
    c3[10:20, :, 5] = 7.0                   # ten classes tie at the top in every image
    c3[30:34, :, :] = -3.0                  # and four tie at a constant row
    cls = torch.empty(B, k, device=dev, dtype=torch.int32)
    ops.topk_classes(corr.to(dev), t_stride=B * HW, b_stride=HW, B=B, T=T, HW=HW, k=k, out=cls)
    m = c3.max(-1)[0].T                     # (B, T)
    for b in range(B):
        order = sorted(range(T), key=lambda t: (-m[b, t].item(), t))[:k]
        assert cls[b].cpu().tolist() == order


@pytest.mark.parametrize("p,res", [(16, 384), (14, 336), (12, 384)])
def test_preprocess_im2col(p, res):
    """Normalise + bilinear resize of ragged padded images + patch im2col vs the oracle's preprocess,
    for the two compiled patch sizes (B/16, L/14) and the runtime-patch kernel."""
    arch_mean = torch.tensor([122.7709383, 116.7460125, 104.09373615])
    arch_std = torch.tensor([68.5005327, 66.6321579, 70.3231630])
    imgs = [torch.randint(0, 256, (3, 300, 352), generator=torch.Generator().manual_seed(1)).float(),
            torch.randint(0, 256, (3, 320, 256), generator=torch.Generator().manual_seed(2)).float()]

    class A:
        clip_pixel_mean, clip_pixel_std, size_divisibility, clip_resolution = arch_mean.tolist(), arch_std.tolist(), 32, res
    ref, sizes = O.preprocess(A, imgs)
    Hp, Wp = 320, 352
    raw = torch.zeros(2, 3, Hp, Wp)
    for i, im in enumerate(imgs):
        raw[i, :, :im.shape[1], :im.shape[2]] = im
    G = res // p
    out = torch.empty(2 * G * G, 3 * p * p + 32, device=dev)
    ops.preprocess_im2col(raw.to(dev), torch.tensor(sizes, dtype=torch.int32).to(dev), mean=arch_mean.to(dev),
                          std=arch_std.to(dev), res=res, patch=p, out=out)
    cols = F.unfold(ref, p, stride=p).transpose(1, 2).reshape(-1, 3 * p * p)
    close(out[:, :3 * p * p], cols, atol=2e-5, what="preprocess")
    assert out[:, 3 * p * p:].abs().max().item() == 0


def test_bicubic_postprocess():
    S_in, S_out, D = 14, 24, 8
    g = rnd(S_in * S_in, D, seed=34)
    out = torch.empty(S_out * S_out, D, device=dev)
    ops.bicubic_resize(g.to(dev), S_in, D, out, S_out)
    pos = torch.cat([torch.zeros(1, D), g], 0)
    ref = O.resized_pos_embed(pos, S_in, S_out)[1:]
    close(out, ref, atol=2e-6, what="bicubic")
    lg = rnd(2, 3, 96, 96, seed=35) * 4
    o = torch.empty(2, 3, 333, 250, device=dev)
    ops.postprocess(lg.to(dev), o)
    ref = F.interpolate(lg.sigmoid(), size=(333, 250), mode="bilinear", align_corners=False)
    close(o, ref, atol=2e-6, what="postprocess")


@pytest.mark.parametrize("HW,crop", [(336, None), (384, None), (336, (90, 77))])
def test_postprocess_compile_time_width(HW, crop):
    """The separable band kernel (tuning knob post_variant 0, default; W = 336 / 384, the
    CAT-Seg eval outputs) vs torch (sigmoid -> bilinear, align_corners=False, sem_seg_postprocess crop)
    and bit for bit vs the direct band kernel (variant 1)."""
    lib = L.load()
    lg = (rnd(2, 5, 96, 96, seed=36) * 4).to(dev)
    outs = []
    try:
        for v in (0, 1):
            L.tune("post_variant", v)
            o = torch.empty(2, 5, HW, HW, device=dev)
            if crop is None:
                ops.postprocess(lg, o)
            else:
                ops.postprocess(lg, o, crop=crop)
            torch.cuda.synchronize()
            outs.append(o)
    finally:
        L.tune("post_variant", 0)
    src = lg.cpu() if crop is None else lg.cpu()[:, :, :crop[0], :crop[1]]
    ref = F.interpolate(src.sigmoid(), size=(HW, HW), mode="bilinear", align_corners=False)
    close(outs[0], ref, atol=2e-6, what="postprocess W=%d" % HW)
    assert torch.equal(outs[0], outs[1])


@pytest.fixture(params=["persistent", "tiled"])
def rows_variant(request):
    L.tune("persistent", 1 if request.param == "persistent" else 0)
    yield request.param
    L.tune("persistent", 1)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M", [300, 1000])
def test_rows_gemm_ln_add_res_and_convt(dt, M, rows_variant):
    D, N = 128, 384
    x = rnd(M, D, seed=40) * 2 + 0.3
    g, b = rnd(D, seed=41) + 1, rnd(D, seed=42)
    w = rnd(N, D, seed=43) / math.sqrt(D)
    bias = rnd(N, seed=44)
    add = rnd(M // 10 + 1, 256, seed=45)
    res = rnd(M, N, seed=46)
    amap = rowmap(d1=10)                        # row m -> add row m // 10
    out = torch.empty(M, N, device=dev, dtype=dt)
    ops.rows_gemm(x.to(dev, dt), w.to(dev, dt), out, ln=(g.to(dev), b.to(dev)), bias=bias.to(dev),
                  add=add.to(dev, dt), addmap=amap, add_ncols=256, act=L.ACT_GELU, res=res.to(dev, dt))
    xn = F.layer_norm(x.to(dt).double(), (D,), g.double(), b.double(), 1e-5)
    v = xn.to(dt).double() @ w.to(dt).double().T + bias.double()
    v[:, :256] += add.to(dt).double()[torch.arange(M) // 10]
    ref = F.gelu(v) + res.to(dt).double()
    close(out, ref, atol=5e-5 if dt == torch.float32 else 4e-2, rtol=0 if dt == torch.float32 else 1e-2,
          what="rows_gemm")
    # ConvTranspose scatter store, no LN
    S, H, W_, co = 3, 4, 5, 96
    xs = rnd(S * H * W_, D, seed=47)
    wt = rnd(D, co, 2, 2, seed=48) / 8
    bt = rnd(co, seed=49)
    Wg = wt.permute(2, 3, 1, 0).reshape(4 * co, D).contiguous()
    o2 = torch.empty(S * 4 * H * W_, co, device=dev, dtype=dt)
    ops.rows_gemm(xs.to(dev, dt), Wg.to(dev, dt), o2, bias=bt.repeat(4).to(dev), store=(2, H, W_, co))
    ref2 = F.conv_transpose2d(xs.to(dt).double().reshape(S, H, W_, D).permute(0, 3, 1, 2), wt.to(dt).double(),
                              bt.double(), stride=2)
    close(o2.reshape(S, 2 * H, 2 * W_, co).permute(0, 3, 1, 2), ref2, atol=2e-5 if dt == torch.float32 else 2e-2,
          what="rows convT")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [L.ACT_GELU, L.ACT_RELU])
def test_rows_mlp(dt, act, rows_variant):
    M, D, Hd = 700, 128, 512
    y = rnd(M, D, seed=50) * 2
    g, b = rnd(D, seed=51) + 1, rnd(D, seed=52)
    w1, b1 = rnd(Hd, D, seed=53) / math.sqrt(D), rnd(Hd, seed=54)
    w2, b2 = rnd(D, Hd, seed=55) / math.sqrt(Hd), rnd(D, seed=56)
    x = rnd(M, D, seed=57)
    yd, xd = y.to(dev, dt), x.to(dev, dt)
    out = torch.empty_like(xd)
    ops.rows_mlp(yd, w1.to(dev, dt), b1.to(dev), w2.to(dev, dt), out, ln=(g.to(dev), b.to(dev)), b2=b2.to(dev),
                 act=act, res=yd, res2=xd)
    yn = F.layer_norm(y.to(dt).double(), (D,), g.double(), b.double(), 1e-5).to(dt).double()
    fn = F.gelu if act == L.ACT_GELU else F.relu
    h = fn(yn @ w1.to(dt).double().T + b1.double()).to(dt).double()
    ref = h @ w2.to(dt).double().T + b2.double() + y.to(dt).double() + x.to(dt).double()
    close(out, ref, atol=5e-5 if dt == torch.float32 else 4e-2, rtol=0 if dt == torch.float32 else 1e-2,
          what="rows_mlp")
    # in place (out aliases the residual), as the engine uses it
    ops.rows_mlp(yd, w1.to(dev, dt), b1.to(dev), w2.to(dev, dt), yd, ln=(g.to(dev), b.to(dev)), b2=b2.to(dev),
                 act=act, res=yd)
    close(yd, ref - x.to(dt).double(), atol=5e-5 if dt == torch.float32 else 4e-2,
          rtol=0 if dt == torch.float32 else 1e-2, what="rows_mlp in place")


@pytest.mark.parametrize("W_,c1,c2,co,gn", [(48, 96, 32, 64, False), (48, 64, 0, 64, True), (96, 48, 16, 32, False),
                                            (96, 32, 0, 32, True)])
@pytest.mark.parametrize("lds", [2, 0])
def test_conv3x3_decoder_shapes(W_, c1, c2, co, gn, lds):
    """The decoder conv shapes (bf16): row-ring kernel (conv_mode 2), im2col (0)."""
    B, T = 2, 3
    S, H = B * T, W_
    x1 = rnd(S, H, W_, c1, seed=70) * 2
    x2 = rnd(B, H, W_, max(c2, 8), seed=71)[..., :c2]
    w = rnd(co, c1 + c2, 3, 3, seed=72) / 12
    dt = torch.bfloat16
    mean = rnd(S * (c1 // 16), seed=73) * 0.2
    rstd = rnd(S * (c1 // 16), seed=74) * 0.2 + 1
    gam, bet = rnd(c1, seed=75) + 1, rnd(c1, seed=76)
    xin = x1.to(dt).double()
    if gn:
        g = torch.arange(c1) // 16
        sc = rstd.reshape(S, -1)[:, g].double() * gam.double()
        sh = bet.double() - mean.reshape(S, -1)[:, g].double() * sc
        xin = torch.relu(xin * sc[:, None, None, :] + sh[:, None, None, :]).to(dt).double()
    if c2:
        xin = torch.cat([xin, x2.to(dt).double().repeat_interleave(T, 0)], -1)
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w.to(dt).double(), padding=1)
    L.tune("conv_mode", lds)
    try:
        out = torch.empty(S * H * W_, co, device=dev, dtype=dt)
        xs = x1.reshape(-1, c1).contiguous().to(dev, dt)
        wk = w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev, dt)
        kw = dict(S=S, H=H, W=W_, c1=c1, src2=x2.reshape(-1, c2).contiguous().to(dev, dt) if c2 else None, c2=c2,
                  src2_div=T, gn=(mean.to(dev), rstd.to(dev), gam.to(dev), bet.to(dev), 16) if gn else None)
        tile = ops.conv3x3_stats_tile(xs, wk, **kw)
        tiles = H * W_ // tile
        st = torch.empty(S * tiles * (co // 16) * 2, device=dev)
        ops.conv3x3(xs, wk, out, stats=st, **kw)
        close(out.reshape(S, H, W_, co).permute(0, 3, 1, 2), ref, atol=3e-2, rtol=1e-2, what="conv decoder")
        m_ = torch.empty(S * (co // 16), device=dev)
        r_ = torch.empty_like(m_)
        ops.groupnorm_stats(st, S, tiles, co // 16, tile * 16, m_, r_)
        gref = ref.reshape(S, co // 16, 16, H * W_)
        close(m_, gref.mean((-1, -2)).reshape(-1), atol=2e-3, what="gn mean")
    finally:
        L.tune("conv_mode", 2)


def test_convt64_gn():
    S, H, W_, C, co = 3, 8, 16, 64, 48
    x = rnd(S, H, W_, C, seed=60) * 2
    mean, rstd = rnd(S * 4, seed=61) * 0.3, rnd(S * 4, seed=62) * 0.2 + 1
    gam, bet = rnd(C, seed=63) + 1, rnd(C, seed=64)
    wt, bt = rnd(C, co, 2, 2, seed=65) / 8, rnd(co, seed=66)
    xd = x.reshape(-1, C).to(dev, torch.bfloat16)
    out = torch.empty(S * 4 * H * W_, co, device=dev, dtype=torch.bfloat16)
    Wg = wt.permute(2, 3, 1, 0).reshape(4 * co, C).contiguous()
    ops.convt64_gn(xd, Wg.to(dev, torch.bfloat16), out, HW=H * W_,
                   gn=(mean.to(dev), rstd.to(dev), gam.to(dev), bet.to(dev), 16), bias=bt.repeat(4).to(dev),
                   store=(2, H, W_, co))
    xb = x.to(torch.bfloat16).double()
    g = torch.arange(C) // 16
    sc = rstd.reshape(S, 4)[:, g].double() * gam.double()
    sh = bet.double() - mean.reshape(S, 4)[:, g].double() * sc
    z = torch.relu(xb * sc[:, None, None, :] + sh[:, None, None, :]).to(torch.bfloat16).double()
    ref = F.conv_transpose2d(z.permute(0, 3, 1, 2), wt.to(torch.bfloat16).double(), bt.double(), stride=2)
    close(out.reshape(S, 2 * H, 2 * W_, co).permute(0, 3, 1, 2), ref, atol=3e-2, rtol=1e-2, what="convt64_gn")


def test_text_helpers():
    n, ctx, Wd, vocab = 3, 16, 64, 50
    tok = torch.randint(0, vocab, (n, ctx), generator=torch.Generator().manual_seed(3)).int()
    emb, pos = rnd(vocab, Wd, seed=36), rnd(ctx, Wd, seed=37)
    x = torch.empty(n * ctx, Wd, device=dev)
    ops.token_embed(tok.to(dev), emb.to(dev), pos.to(dev), x)
    ref = emb[tok.long()] + pos
    close(x, ref.reshape(-1, Wd), atol=1e-6, what="token_embed")
    e = torch.empty(n, Wd, device=dev)
    ops.eot_gather(x, tok.to(dev), e)
    close(e, ref[torch.arange(n), tok.long().argmax(-1)], atol=1e-6, what="eot")


# ----------------------------------------------------------------------------- pooling / sliding
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pool", [(2, 2), (3, 2), (4, 4)])
def test_avgpool_and_upsample_add_rows(dt, pool):
    """ClassTransformerLayer pool_features + interpolate(align_corners=True) + residual
    (model.py:374-385,415-423) on the rows layout, vs torch on the reference layout."""
    S, H, W, C = 5, 24, 24, 128
    ph, pw = pool
    x = rnd(S, H, W, C, seed=31).to(dt)
    xp = torch.empty(S * (H // ph) * (W // pw), C, device=dev, dtype=dt)
    ops.avgpool_rows(x.to(dev).reshape(-1, C), xp, S=S, H=H, W=W, C=C, pool=pool)
    ref_p = F.avg_pool2d(x.float().permute(0, 3, 1, 2), pool)                    # (S, C, Hp, Wp)
    close(xp.reshape(S, H // ph, W // pw, C).permute(0, 3, 1, 2), ref_p,
          atol=1e-6 if dt == torch.float32 else 1e-2, what="avgpool")
    y = rnd(S, H // ph, W // pw, C, seed=32).to(dt)
    xd = x.to(dev).reshape(-1, C).clone()
    ops.upsample_add_rows(y.to(dev).reshape(-1, C), xd, S=S, Hp=H // ph, Wp=W // pw, C=C, H=H, W=W)
    up = F.interpolate(y.float().permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=True)
    ref = x.float() + up.permute(0, 2, 3, 1)
    close(xd.reshape(S, H, W, C), ref, atol=1e-5 if dt == torch.float32 else 2e-2, what="upsample_add")


def test_sliding_crops_and_merge_vs_oracle_ops():
    """catseg_sliding_crops / catseg_sliding_merge / catseg_resize_bilinear vs the reference's
    Unfold / Fold / interpolate sequence (cat_seg_model.py:158-168,204-217)."""
    k, stride, res = 384, 256, 640
    unfold = torch.nn.Unfold(kernel_size=k, stride=stride)
    fold = torch.nn.Fold([res, res], kernel_size=k, stride=stride)
    shapes = [(440, 360), (512, 640)]
    imgs = [rnd(3, h, w, seed=40 + i, scale=127.5) + 127.5 for i, (h, w) in enumerate(shapes)]
    Hc, Wc = 512, 640
    raw = torch.zeros(2, 3, Hc, Wc)
    for i, im in enumerate(imgs):
        raw[i, :, :im.shape[1], :im.shape[2]] = im
    sizes = torch.tensor(shapes, dtype=torch.int32)
    crops = torch.empty(2 * 5, 3, k, k, device=dev)
    ops.sliding_crops(raw.to(dev), sizes.to(dev), crops, out_res=res, kernel=k, stride=stride)
    for i, im in enumerate(imgs):
        x = F.interpolate(im.unsqueeze(0), size=[res, res], mode="bilinear", align_corners=False).squeeze()
        x = unfold(x).reshape(3, k, k, -1).permute(3, 0, 1, 2)
        gl = F.interpolate(im.unsqueeze(0), size=(k, k), mode="bilinear", align_corners=False)
        ref = torch.cat((x, gl), 0)
        close(crops[5 * i:5 * i + 5], ref, atol=2e-3, what=f"crops {i}")
    T = 7
    lg = rnd(2 * 5, T, 96, 96, seed=44, scale=4.0)
    merged = torch.empty(2, T, res, res, device=dev)
    ops.sliding_merge(lg.to(dev), merged, kernel=k, stride=stride, out_res=res)
    for i in range(2):
        o = F.interpolate(lg[5 * i:5 * i + 5], size=k, mode="bilinear", align_corners=False).sigmoid()
        glob = F.interpolate(o[-1:], size=[res, res], mode="bilinear", align_corners=False)
        t = fold(o[:-1].flatten(1).T) / fold(unfold(torch.ones([1, res, res])))
        close(merged[i], ((t + glob) / 2.0)[0], atol=1e-5, what=f"merge {i}")
    # the band kernel gathering from global (1) equals the staged merge computing the row terms per
    # output (2) bit for bit; the tabulated staged merge (0, default) has the same taps and Fold order
    # but the compiler contracts its blends into FMAs differently (an ulp of a probability)
    lib = L.load()
    mv = {}
    for v in (1, 2):
        mv[v] = torch.empty_like(merged)
        try:
            L.tune("merge_variant", v)
            ops.sliding_merge(lg.to(dev), mv[v], kernel=k, stride=stride, out_res=res)
            torch.cuda.synchronize()
        finally:
            L.tune("merge_variant", 0)
    assert torch.equal(mv[1], mv[2])
    assert (merged - mv[2]).abs().max().item() <= 1e-6
    # ragged band (out_res not a multiple of the 16-row band) with another window geometry:
    # out_res 600 = 2 tiles of 360 at stride 240, 90-wide logits
    k2, s2, r2 = 360, 240, 600
    lg2 = rnd(1 * 5, 3, 90, 90, seed=45, scale=4.0)
    m2 = {}
    for v in (0, 2):
        m2[v] = torch.empty(1, 3, r2, r2, device=dev)
        try:
            L.tune("merge_variant", v)
            ops.sliding_merge(lg2.to(dev), m2[v], kernel=k2, stride=s2, out_res=r2)
            torch.cuda.synchronize()
        finally:
            L.tune("merge_variant", 0)
    assert (m2[0] - m2[2]).abs().max().item() <= 1e-6
    out = torch.empty(1, T, 480, 400, device=dev)
    ops.resize_bilinear(merged[:1], out, crop=(res, res))
    ref = F.interpolate(merged[:1].cpu(), size=(480, 400), mode="bilinear", align_corners=False)
    close(out, ref, atol=1e-6, what="resize")


@pytest.mark.parametrize("variant", [0, 3])
@pytest.mark.parametrize("shift", [0, 6, 3])
def test_swin_window_attention_fused_vs_unfused(shift, variant):
    """catseg_swin_window_attention == catseg_rows_gemm(LN1 + q/k/v + guidance) followed by
    catseg_attention mode 1 (model.py:191-199, 86-114), bf16, on the 24x24 / 12x12 geometry.
    variant 0 = the register-resident kernel (default, swin_window.hip swin_win5: two 4-wave
    workgroups per CU), 3 = the head-per-SIMD kernel (swin_win3, the fallback for other guidance row
    maps); S = 7 slices = 28 windows over the persistent grid (window location varies per workgroup)."""
    B, T, HW, D = 1, 7, 576, 128
    S = B * T
    R = S * HW
    dt = torch.bfloat16
    X = rnd(R, D, seed=51, scale=2.0).to(dev, dt)
    g1, b1 = (1 + rnd(D, seed=52, scale=0.2)).to(dev), rnd(D, seed=53, scale=0.2).to(dev)
    W = (rnd(3 * D, D, seed=54) / math.sqrt(D)).to(dev, dt)
    bias = rnd(3 * D, seed=55, scale=0.1).to(dev)
    gqk = rnd(B * HW, 2 * D, seed=56, scale=0.5).to(dev, dt)
    gmap = rowmap(d1=T * HW, s1=HW, d2=1, m2=HW, s2=1)
    qkv = torch.empty(R, 3 * D, device=dev, dtype=dt)
    ops.rows_gemm(X, W, qkv, ln=(g1, b1), bias=bias, add=gqk, addmap=gmap, add_ncols=2 * D)
    ref = torch.empty(R, D, device=dev, dtype=dt)
    ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], ref, n_seq=S * 4, seq_len=144, n_heads=4,
                  head_dim=32, scale=32 ** -0.5, mode=1, img_hw=(24, 24), window=12, shift=shift)
    out = torch.empty(R, D, device=dev, dtype=dt)
    try:
        L.tune("swin_variant", variant)
        ops.swin_window_attention(X, (g1, b1), W, bias, gqk, gmap, out, S=S, img_hw=(24, 24), window=12, shift=shift,
                                  n_heads=4, head_dim=32, scale=32 ** -0.5)
    finally:
        L.tune("swin_variant", 0)
    err = (out.float() - ref.float()).abs()
    # both are bf16 pipelines over the same math (q/k/v rounded to bf16 in both): equal to bf16 noise
    assert err.max().item() < 3e-2 and err.mean().item() < 2e-3, (err.max().item(), err.mean().item())
    # and against an fp32 torch restatement of the reference ops on the same bf16 inputs
    from oracle import catseg_oracle as O
    xf = X.float().cpu().reshape(S, 24, 24, D)
    h = F.layer_norm(xf, (D,), g1.cpu(), b1.cpu())
    gi = gqk.float().cpu().reshape(B, 1, 24, 24, 2 * D).expand(B, T, 24, 24, 2 * D).reshape(S, 24, 24, 2 * D)
    qkv_f = h @ W.float().cpu().T + bias.cpu()
    qkv_f[..., :2 * D] += gi
    if shift:
        qkv_f = torch.roll(qkv_f, shifts=(-shift, -shift), dims=(1, 2))
    win = O.window_partition(qkv_f, 12).reshape(-1, 144, 3, 4, 32).permute(2, 0, 3, 1, 4)   # (3, nW*S, H, L, d)
    q, k, v = win[0] * 32 ** -0.5, win[1], win[2]
    attn = q @ k.transpose(-2, -1)
    if shift:
        m = O.shift_mask(24, 24, 12, shift)                  # (nW, L, L)
        attn = attn.reshape(S, 4, 4, 144, 144) + m.reshape(1, 4, 1, 144, 144)
        attn = attn.reshape(-1, 4, 144, 144)
    o = (attn.softmax(-1) @ v).transpose(1, 2).reshape(-1, 12, 12, D)
    o = O.window_reverse(o, 12, 24, 24)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    e2 = (out.float().cpu().reshape(S, 24, 24, D) - o).abs()
    assert e2.max().item() < 5e-2 and e2.mean().item() < 5e-3, (e2.max().item(), e2.mean().item())


@pytest.mark.parametrize("glin", [True, False])
@pytest.mark.parametrize("shift", [0, 6])
def test_swin_window_attention_persistent_variants_agree(shift, glin):
    """Persistent grid over several windows per workgroup (S = 200 slices = 800 windows > the
    grid, guidance map of 2 images): the register-resident default (variant 0, swin_win5) equals the
    head-per-SIMD kernel (variant 3, swin_win3: same LayerNorm, projection, mask and softmax
    arithmetic) bit for bit; both retire the window's opaque LDS-DMA with a counted window-start wait
    that lets the previous window's stores stay in flight.  glin=False stores the guidance pixel-major
    (row = pixel * B + image), which no slice maps to one base + pixel: both then run swin_win3's
    per-tile row-map path."""
    B, T, HW, D = 2, 100, 576, 128
    S = B * T
    R = S * HW
    dt = torch.bfloat16
    X = rnd(R, D, seed=61, scale=2.0).to(dev, dt)
    g1, b1 = (1 + rnd(D, seed=62, scale=0.2)).to(dev), rnd(D, seed=63, scale=0.2).to(dev)
    W = (rnd(3 * D, D, seed=64) / math.sqrt(D)).to(dev, dt)
    bias = rnd(3 * D, seed=65, scale=0.1).to(dev)
    gqk = rnd(B * HW, 2 * D, seed=66, scale=0.5).to(dev, dt)
    gmap = rowmap(d1=T * HW, s1=HW, d2=1, m2=HW, s2=1) if glin else rowmap(d1=T * HW, s1=1, d2=1, m2=HW, s2=B)
    outs = []
    try:
        for variant in (3, 0):
            L.tune("swin_variant", variant)
            o = torch.full((R, D), float("nan"), device=dev, dtype=dt)
            ops.swin_window_attention(X, (g1, b1), W, bias, gqk, gmap, o, S=S, img_hw=(24, 24), window=12,
                                      shift=shift, n_heads=4, head_dim=32, scale=32 ** -0.5)
            torch.cuda.synchronize()
            outs.append(o.float())
    finally:
        L.tune("swin_variant", 0)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[1], outs[0]), (outs[1] - outs[0]).abs().max().item()


def test_swin_window_attention_repeat_launches_bit_identical():
    """Regression for an intermittent wrong tile: the register-resident kernel's first masked form
    (16x16x16 mask MFMA) returned one wave's query tile 0 wrong in ~1 launch of 5 when LDS was idle.
    Twelve launches of the default (variant 0) at shift 6 over 800 windows (224 workgroups with a
    single window) must all equal swin_win3 (variant 3) bit for bit."""
    B, T, HW, D = 2, 100, 576, 128
    S, R = B * T, B * T * HW
    dt = torch.bfloat16
    X = rnd(R, D, seed=61, scale=2.0).to(dev, dt)
    g1, b1 = (1 + rnd(D, seed=62, scale=0.2)).to(dev), rnd(D, seed=63, scale=0.2).to(dev)
    W = (rnd(3 * D, D, seed=64) / math.sqrt(D)).to(dev, dt)
    bias = rnd(3 * D, seed=65, scale=0.1).to(dev)
    gqk = rnd(B * HW, 2 * D, seed=66, scale=0.5).to(dev, dt)
    gmap = rowmap(d1=T * HW, s1=HW, d2=1, m2=HW, s2=1)

    def run(variant):
        L.tune("swin_variant", variant)
        o = torch.full((R, D), float("nan"), device=dev, dtype=dt)
        ops.swin_window_attention(X, (g1, b1), W, bias, gqk, gmap, o, S=S, img_hw=(24, 24), window=12, shift=6,
                                  n_heads=4, head_dim=32, scale=32 ** -0.5)
        return o

    try:
        ref = run(3)
        bad = [i for i in range(12) if not torch.equal(run(0), ref)]
    finally:
        L.tune("swin_variant", 0)
    assert not bad, f"launches {bad} of 12 differ from swin_win3"


@pytest.mark.parametrize("ci,m,cg,co,H,gn_src", [(64, 48, 16, 32, 48, True), (64, 48, 16, 32, 48, False),
                                                   (128, 96, 32, 64, 24, False)])
def test_upconv3x3_folded_convtranspose(ci, m, cg, co, H, gn_src):
    """catseg_upconv3x3 + catseg_upconv_addend (Up blocks, model.py:546-555):
    ConvTranspose2d(ci -> m, k=2, s=2) of z (relu(GN(z)) in the second block), concat the
    per-image guidance (cg ch, repeated over T), conv3x3 (m + cg -> co, no bias) == one 4-parity
    composite conv over z plus the addend; vs the unfused composition in fp64 (bf16 operands),
    GroupNorm partials too.  Shapes of the second (48 -> 96) and first (24 -> 48) block."""
    from cat_seg.engine import CatSegEngine
    B, T = 2, 3
    S = B * T
    z = rnd(S, ci, H, H, seed=81)
    wt = rnd(ci, m, 2, 2, seed=82) / 8
    bt = rnd(m, seed=83)
    wc = rnd(co, m + cg, 3, 3, seed=84) / 16
    g = rnd(B, cg, 2 * H, 2 * H, seed=85)
    dt = torch.bfloat16
    if gn_src:
        mean = rnd(S * (ci // 16), seed=86) * 0.1
        rstd = 1 + rnd(S * (ci // 16), seed=87).abs()
        gam, bet = 1 + rnd(ci, seed=88) * 0.2, rnd(ci, seed=89) * 0.1
        zb = z.to(dt).double().reshape(S, ci // 16, 16, H, H)
        zz = torch.relu(((zb - mean.double().reshape(S, -1, 1, 1, 1)) * rstd.double().reshape(S, -1, 1, 1, 1)
                         ).reshape(S, ci, H, H) * gam.double().reshape(1, ci, 1, 1) + bet.double().reshape(1, ci, 1, 1))
        # the kernel applies GN+ReLU in fp32 and rounds to bf16 before the MFMA
        zz = zz.float().to(dt).double()
    else:
        zz = z.to(dt).double()
    up = F.conv_transpose2d(zz, wt.double(), bt.double(), stride=2)
    xin = torch.cat([up, g.to(dt).double().repeat_interleave(T, 0)], 1)
    ref = F.conv2d(xin, wc.double(), padding=1)                              # (S, co, 2H, 2H)
    comp, tap_b = CatSegEngine._upconv_weights(wt, bt, wc[:, :m])
    wg = wc[:, m:].to(dt).float().permute(0, 2, 3, 1).reshape(co, -1).contiguous().to(dev)
    part = torch.empty(B * H * H, 4 * co, device=dev)
    ops.upconv_addend(g.permute(0, 2, 3, 1).contiguous().to(dev, dt), wg, tap_b.to(dev), part, B=B, H2=2 * H, W2=2 * H)
    out = torch.empty(S * 4 * H * H, co, device=dev, dtype=dt)
    tile = ops.upconv3x3_stats_tile()
    ntl = 4 * H * H // tile
    st = torch.empty(S * ntl * (co // 16) * 2, device=dev)
    gn = None
    if gn_src:
        gn = (mean.to(dev), rstd.to(dev), gam.to(dev), bet.to(dev), 16)
    ops.upconv3x3(z.permute(0, 2, 3, 1).contiguous().to(dev, dt), comp.to(dev, dt), out, S=S, H=H, W=H, c1=ci, gn=gn,
                  stats=st, addend=part, addend_div=T)
    got = out.reshape(S, 2 * H, 2 * H, co).permute(0, 3, 1, 2).double().cpu()
    # bf16 composite weights vs the exact composition: a few bf16 roundings of an O(1) sum
    err = (got - ref).abs()
    assert err.max().item() <= 2e-2 + 2 ** -7 * ref.abs().max().item(), err.max().item()
    assert err.mean().item() <= 2e-3, err.mean().item()
    # the one-barrier-per-chunk ring (tuning knob ring_onebar 1, default) equals the two-barrier form bit for bit
    L.load()
    out1, st1 = torch.empty_like(out), torch.empty_like(st)
    try:
        L.tune("ring_onebar", 0)
        ops.upconv3x3(z.permute(0, 2, 3, 1).contiguous().to(dev, dt), comp.to(dev, dt), out1, S=S, H=H, W=H, c1=ci,
                      gn=gn, stats=st1, addend=part, addend_div=T)
        torch.cuda.synchronize()
    finally:
        L.tune("ring_onebar", 1)
    assert torch.equal(out1, out) and torch.equal(st1, st)
    mean1 = torch.empty(S * (co // 16), device=dev)
    rstd1 = torch.empty_like(mean1)
    ops.groupnorm_stats(st, S, ntl, co // 16, tile * 16, mean1, rstd1)
    gref = got.reshape(S, co // 16, -1)
    close(mean1, gref.mean(-1).reshape(-1), atol=1e-4, what="gn mean")
    close(rstd1, (1 / torch.sqrt(gref.var(-1, unbiased=False) + 1e-5)).reshape(-1), atol=0, rtol=2e-3, what="gn rstd")


def test_swin_proj_mlp_equals_separate_kernels():
    """catseg_swin_proj_mlp (model.py:112 proj, :222-223 shortcut + Mlp(norm2)) is the separate
    catseg_rows_gemm(proj + residual) -> catseg_rows_mlp pair, bit for bit, on ragged M; and both
    match an fp64 restatement to bf16 rounding."""
    M, C, Hd = 3 * 577 + 5, 128, 512
    dt = torch.bfloat16
    x = rnd(M, C, seed=91).to(dev, dt)
    attn = rnd(M, C, seed=92).to(dev, dt)
    wp, bp = (rnd(C, C, seed=93) / 11).to(dev, dt), rnd(C, seed=94).to(dev)
    g, b = (1 + rnd(C, seed=95) * 0.2).to(dev), (rnd(C, seed=96) * 0.1).to(dev)
    w1, b1 = (rnd(Hd, C, seed=97) / 11).to(dev, dt), rnd(Hd, seed=98).to(dev)
    w2, b2 = (rnd(C, Hd, seed=99) / 22).to(dev, dt), rnd(C, seed=100).to(dev)
    ref = x.clone()
    ops.rows_gemm(attn, wp, ref, bias=bp, res=ref)
    ops.rows_mlp(ref, w1, b1, w2, ref, ln=(g, b), b2=b2, act=L.ACT_GELU, res=ref)
    got = x.clone()
    ops.swin_proj_mlp(attn, got, wp, bp, w1, b1, w2, b2, got, ln=(g, b))
    torch.cuda.synchronize()
    assert torch.equal(got, ref), (got.float() - ref.float()).abs().max().item()
    x1 = x.double().cpu() + attn.double().cpu() @ wp.double().cpu().T + bp.double().cpu()
    h = F.gelu(F.layer_norm(x1, (C,), g.double().cpu(), b.double().cpu(), 1e-5) @ w1.double().cpu().T + b1.double().cpu())
    y = x1 + h @ w2.double().cpu().T + b2.double().cpu()
    close(got, y, atol=0.08, rtol=0.02, what="swin proj+mlp vs fp64")


@pytest.mark.parametrize("H,W", [(96, 96), (50, 96), (50, 37)])
def test_head_conv_band(H, W):
    """The head conv (model.py:634, 32 -> 1, 3x3, GroupNorm+ReLU on load) vs fp64, with the top-k
    class scatter: at W = 96 the MFMA tap-product kernel (head_variant 0, the default; 24-row bands,
    ragged last band at H = 50) and the v_dot2c band kernel with the compile-time width (variant 1),
    which equals the runtime-width band kernel (variant 2, also the W = 37 path) bit for bit."""
    B, T, C = 2, 3, 32
    S = B * T
    lib = L.load()
    x = rnd(S, C, H, W, seed=111)
    mean, rstd = rnd(S * 2, seed=112) * 0.2, 1 + rnd(S * 2, seed=113).abs()
    gam, bet = 1 + rnd(C, seed=114) * 0.2, rnd(C, seed=115) * 0.2
    hw_ = rnd(1, C, 3, 3, seed=116) / 8
    xb = x.to(torch.bfloat16)
    y1 = torch.relu(((xb.double().reshape(S, 2, 16, H, W) - mean.double().reshape(S, 2, 1, 1, 1))
                     * rstd.double().reshape(S, 2, 1, 1, 1)).reshape(S, C, H, W) * gam.double().reshape(1, C, 1, 1)
                    + bet.double().reshape(1, C, 1, 1))
    rh = F.conv2d(y1, hw_.double(), torch.tensor([0.25]).double(), padding=1).reshape(B, T, H, W)
    xin = xb.permute(0, 2, 3, 1).contiguous().to(dev)
    cls = torch.tensor([[0, 2, 4], [1, 3, 0]], dtype=torch.int32).to(dev)
    outs = {}
    try:
        for v in (0, 1, 2, 3):
            L.tune("head_variant", v)
            logits = torch.full((B, T + 2, H, W), -100.0, device=dev)
            ops.conv3x3_head(xin, B=B, T=T, H=H, W=W, C=C, weight=hw_[0].permute(1, 2, 0).reshape(-1).contiguous().to(dev),
                             bias=0.25, out=logits, T_out=T + 2, classes=cls,
                             gn=(mean.to(dev), rstd.to(dev), gam.to(dev), bet.to(dev), 16))
            outs[v] = logits.cpu()
    finally:
        L.tune("head_variant", 0)
    assert torch.equal(outs[3], outs[0])     # tap kernel with one input step in flight instead of two
    for v in (0, 1):
        for bi in range(B):
            for t in range(T):
                # fp16 relu(GN(x)) operands: ~5e-4 per product, 288 terms
                close(outs[v][bi, cls[bi, t]], rh[bi, t], atol=6e-3, what=f"head variant {v} vs fp64")
        assert (outs[v] == -100.0).sum() == B * 2 * H * W        # the unselected class planes stay untouched
    # the band kernel with the compile-time width (W = 96) is the runtime-width one, bit for bit
    assert torch.equal(outs[1], outs[2])


@pytest.mark.parametrize("M", [2 * 577 + 9, 300 * 32 + 17, 40])
@pytest.mark.parametrize("act", [L.ACT_GELU, L.ACT_RELU])
def test_mlp_barrier_lean_bit_identical(act, M):
    """The barrier-lean persistent MLP (tuning knob mlp_variant 0, the default: the epilogue of one
    tile beside the first GEMM of the next, residual rows in LDS) equals pmlp_kernel (1) bit for
    bit -- the Swin MLP (GELU), the class MLP (ReLU, + res2), the fused Swin proj + MLP -- on ragged
    M with one tile per workgroup (40 rows), a few, and many (> 2 tiles per workgroup).  pmlp_kernel
    has the segment-table GELU only, so the comparison runs with gelu_form 0; the default 7-VALU form
    is gated against fp64 in test_mlp_gelu_forms_vs_fp64."""
    C, Hd = 128, 512
    dt = torch.bfloat16
    y = (rnd(M, C, seed=130) * 2).to(dev, dt)
    x = rnd(M, C, seed=131).to(dev, dt)
    g, b = (1 + rnd(C, seed=132) * 0.2).to(dev), (rnd(C, seed=133) * 0.1).to(dev)
    w1, b1 = (rnd(Hd, C, seed=134) / 11).to(dev, dt), rnd(Hd, seed=135).to(dev)
    w2, b2 = (rnd(C, Hd, seed=136) / 22).to(dev, dt), rnd(C, seed=137).to(dev)
    wp, bp = (rnd(C, C, seed=138) / 11).to(dev, dt), rnd(C, seed=139).to(dev)
    outs = {}
    form = L.tuning("gelu_form")
    L.tune("gelu_form", 0)
    try:
        for v in (0, 1):
            L.tune("mlp_variant", v)
            o1 = torch.empty_like(y)
            ops.rows_mlp(y, w1, b1, w2, o1, ln=(g, b), b2=b2, act=act, res=y,
                         res2=x if act == L.ACT_RELU else None)
            o2 = x.clone()
            ops.swin_proj_mlp(y, o2, wp, bp, w1, b1, w2, b2, o2, ln=(g, b))
            torch.cuda.synchronize()
            outs[v] = (o1, o2)
    finally:
        L.tune("mlp_variant", 0)
        L.tune("gelu_form", form)
    assert torch.equal(outs[0][0], outs[1][0]), (outs[0][0].float() - outs[1][0].float()).abs().max().item()
    assert torch.equal(outs[0][1], outs[1][1]), (outs[0][1].float() - outs[1][1].float()).abs().max().item()


@pytest.mark.parametrize("M", [300 * 32 + 17, 40])
def test_mlp_gelu_forms_vs_fp64(M):
    """Both GELU forms of the persistent MLPs (gelu_form 0: gelu_seg, 9 VALU; 1: gelu_x7, 7 VALU, the
    default) against the fp64 composition of the Swin MLP and the fused Swin proj + MLP: each within the
    same bf16 gate, and the two forms' outputs within a few bf16 ulps of each other."""
    C, Hd = 128, 512
    dt = torch.bfloat16
    y = (rnd(M, C, seed=140) * 2).to(dev, dt)
    x = rnd(M, C, seed=141).to(dev, dt)
    g, b = (1 + rnd(C, seed=142) * 0.2).to(dev), (rnd(C, seed=143) * 0.1).to(dev)
    w1, b1 = (rnd(Hd, C, seed=144) / 4).to(dev, dt), rnd(Hd, seed=145).to(dev)   # hidden spans the GELU range
    w2, b2 = (rnd(C, Hd, seed=146) / 22).to(dev, dt), rnd(C, seed=147).to(dev)
    wp, bp = (rnd(C, C, seed=148) / 11).to(dev, dt), rnd(C, seed=149).to(dev)
    D = lambda t: t.double().cpu()
    ref_mlp = D(y) + F.gelu(F.layer_norm(D(y), (C,), D(g), D(b), 1e-5) @ D(w1).T + D(b1)) @ D(w2).T + D(b2)
    x1 = (D(x) + D(y) @ D(wp).T + D(bp)).to(dt).double()
    ref_pm = x1 + F.gelu(F.layer_norm(x1, (C,), D(g), D(b), 1e-5) @ D(w1).T + D(b1)) @ D(w2).T + D(b2)
    outs = {}
    form = L.tuning("gelu_form")
    try:
        for f in (0, 1):
            L.tune("gelu_form", f)
            o1 = torch.empty_like(y)
            ops.rows_mlp(y, w1, b1, w2, o1, ln=(g, b), b2=b2, act=L.ACT_GELU, res=y)
            o2 = x.clone()
            ops.swin_proj_mlp(y, o2, wp, bp, w1, b1, w2, b2, o2, ln=(g, b))
            torch.cuda.synchronize()
            outs[f] = (D(o1), D(o2))
            e1 = (outs[f][0] - ref_mlp).abs().max().item()
            e2 = (outs[f][1] - ref_pm).abs().max().item()
            assert e1 < 0.1 and e2 < 0.1, (f, e1, e2)
    finally:
        L.tune("gelu_form", form)
    for k in range(2):
        d = (outs[0][k] - outs[1][k]).abs()
        scale = ref_mlp.abs().max().item() if k == 0 else ref_pm.abs().max().item()
        assert d.max().item() <= 2 ** -6 * scale, (k, d.max().item(), scale)
