"""Training-side HIP kernels (include/catseg_hip_train.h) against torch fp64 autograd of the
reference ops (cat_seg/modeling/transformer/model.py, cat_seg/cat_seg_model.py).

Gate: max |hip - ref| <= 1e-4 * max |ref| (+ a 1e-6 floor) for every gradient (fp32 kernels vs fp64).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from cat_seg import _lib as L  # noqa: E402
from cat_seg import ops, train_ops as TO  # noqa: E402
from oracle import catseg_oracle as O  # noqa: E402

DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def close(a, b, tol=1e-4):
    e = rel(a, b)
    assert e <= tol, f"rel err {e:.3e} > {tol}"


def g(*shape, seed=0, scale=1.0):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=gen, dtype=torch.float64) * scale


def dev(t):
    return t.float().to(DEV).contiguous()


@pytest.mark.parametrize("M,N,K", [(300, 132, 68), (96, 512, 40000), (2304, 768, 171), (5, 4, 8)])
def test_gemm_ex_layouts(M, N, K):
    A = g(M, K, seed=1)
    B = g(K, N, seed=2)
    ref = A @ B
    for a_t in (False, True):
        for b_t in (False, True):
            Ad = dev(A.t() if a_t else A)              # a_t: stored [K][M] (m-contiguous)
            Bd = dev(B.t() if b_t else B)              # b_t: stored [N][K] (k-contiguous)
            a_sm, a_sk = (1, M) if a_t else (K, 1)
            b_sk, b_sn = (1, K) if b_t else (N, 1)
            if (a_t and M % 4) or (not a_t and K % 4) or (b_t and K % 4) or (not b_t and N % 4):
                continue
            out = torch.full((M, N), 3.0, device=DEV)
            TO.gemm_ex(Ad, a_sm, a_sk, Bd, b_sk, b_sn, out, M=M, N=N, K=K, alpha=0.5, beta=1)
            close(out, 0.5 * ref + 3.0)


@pytest.mark.parametrize("terms,tol", [(0, 2e-6), (6, 2e-6), (3, 3e-5)])
@pytest.mark.parametrize("M,N,K", [(300, 132, 68), (128, 384, 20000), (7, 12, 100)])
def test_gemm_ex_split_bf16_forms(terms, tol, M, N, K):
    """The product forms of catseg_gemm_ex (tuning knob gemm_ex_terms): exact-f32 MFMA, the six-pair
    split-bf16 form (automatic for K >= 8192: fp32-class error) and the three-pair form (~2^-17),
    in every operand layout, against fp64 at fp32-scale gates."""
    A = g(M, K, seed=11)
    B = g(K, N, seed=12)
    ref = A @ B
    L.tune("gemm_ex_terms", terms)
    try:
        for a_t in (False, True):
            for b_t in (False, True):
                if (a_t and M % 4) or (not a_t and K % 4) or (b_t and K % 4) or (not b_t and N % 4):
                    continue
                a_sm, a_sk = (1, M) if a_t else (K, 1)
                b_sk, b_sn = (1, K) if b_t else (N, 1)
                out = torch.empty(M, N, device=DEV)
                TO.gemm_ex(dev(A.t() if a_t else A), a_sm, a_sk, dev(B.t() if b_t else B), b_sk, b_sn, out,
                           M=M, N=N, K=K)
                close(out, ref, tol)
    finally:
        L.tune("gemm_ex_terms", -1)


@pytest.mark.parametrize("act,fn", [(L.ACT_GELU, F.gelu), (L.ACT_RELU, F.relu),
                                    (L.ACT_QUICKGELU, lambda t: t * torch.sigmoid(1.702 * t))])
def test_gemm_ex_activation_backward_epilogue(act, fn):
    """dU = (dY . W2) * act'(U) in the GEMM's epilogue (the MLP backward's fused form) vs fp64 autograd,
    in place (the epilogue writes over U) and into a fresh buffer."""
    M, N, K = 1000, 512, 128
    dY, W2, U = g(M, K, seed=40), g(K, N, seed=41) / math.sqrt(K), g(M, N, seed=42, scale=2)
    ur = U.clone().requires_grad_(True)
    fn(ur).backward(dY @ W2)
    out = TO.mm(dev(dY), dev(W2), act_u=dev(U), act=act)
    close(out, ur.grad)
    Ud = dev(U)
    TO.mm(dev(dY), dev(W2), out=Ud, act_u=Ud, act=act)
    close(Ud, ur.grad)


@pytest.mark.parametrize("rows,cols,ld", [(5000, 132, 132),      # 16-byte loads, 33 vectors in a 64-wide block
                                          (5000, 130, 130),      # scalar path (cols % 4 != 0)
                                          (3001, 96, 100),       # strided rows, vectors
                                          (300000, 32, 32),      # 2048 chunks, 8 vectors x 32 row lanes
                                          (77, 3072, 3072),      # 12 column blocks, one chunk per 64 rows
                                          (9, 1, 1)])
def test_colsum(rows, cols, ld):
    x = g(rows, ld, seed=3)
    out = torch.ones(cols, device=DEV)
    TO.colsum(dev(x), out, rows=rows, cols=cols, ld=ld, beta=1, alpha=2.0)
    ref = x[:, :cols].double().sum(0)
    close(out, 2 * ref.float() + 1)


@pytest.mark.parametrize("cols", [128, 768])
def test_layernorm_backward(cols):
    x = g(777, cols, seed=4)
    w = 1 + 0.1 * g(cols, seed=5)
    b = 0.1 * g(cols, seed=6)
    dy = g(777, cols, seed=7)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    F.layer_norm(xr, (cols,), wr, br, 1e-5).backward(dy)
    dx = dev(torch.ones_like(x))
    dg = torch.zeros(cols, device=DEV)
    db = torch.zeros(cols, device=DEV)
    TO.layernorm_backward(dev(x), dev(w), dev(dy), dx, acc_dx=True, dgamma=dg, dbeta=db)
    close(dx, xr.grad + 1)
    close(dg, wr.grad)
    close(db, br.grad)


@pytest.mark.parametrize("act,fn", [(L.ACT_GELU, F.gelu), (L.ACT_RELU, F.relu),
                                    (L.ACT_QUICKGELU, lambda t: t * torch.sigmoid(1.702 * t))])
def test_act_forward_backward(act, fn):
    u = g(4096, seed=8, scale=3)
    dy = g(4096, seed=9)
    ur = u.clone().requires_grad_(True)
    a = fn(ur)
    a.backward(dy)
    close(TO.act_forward(dev(u), act), a, 1e-6)
    close(TO.act_backward(dev(u), dev(dy), act), ur.grad, 1e-6)


@pytest.mark.parametrize("S,H,W,C,cpg", [(6, 12, 10, 64, 16),    # one pixel chunk
                                         (3, 40, 37, 32, 16),    # 3 chunks of 512 pixels, the last ragged
                                         (2, 24, 24, 128, 16),   # 4.5 chunks of 128 pixels
                                         (4, 9, 7, 16, 4)])      # one group of 4 channels per quad
def test_groupnorm_relu_stats_and_backward(S, H, W, C, cpg):
    x = g(S, C, H, W, seed=10) * 2 + 0.5
    gm = 1 + 0.2 * g(C, seed=11)
    bt = 0.3 * g(C, seed=12)
    dy = g(S, C, H, W, seed=13)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gm, bt))
    F.relu(F.group_norm(xr, C // cpg, gr, br, 1e-5)).backward(dy)
    xn = dev(x.permute(0, 2, 3, 1))
    mean = torch.empty(S * C // cpg, device=DEV)
    rstd = torch.empty_like(mean)
    TO.groupnorm_stats_rows(xn, S, H * W, C, cpg, mean, rstd)
    xs = x.reshape(S, C // cpg, -1)
    close(mean, xs.mean(-1).reshape(-1), 1e-5)
    close(rstd, (1 / torch.sqrt(xs.var(-1, unbiased=False) + 1e-5)).reshape(-1), 1e-5)
    dx = torch.empty_like(xn)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    TO.groupnorm_relu_backward(xn, dev(dy.permute(0, 2, 3, 1)), dx, S=S, HW=H * W, C_=C, cpg=cpg, mean=mean, rstd=rstd,
                               gamma=dev(gm), beta=dev(bt), dgamma=dg, dbeta=db)
    close(dx, xr.grad.permute(0, 2, 3, 1))
    close(dg, gr.grad)
    close(db, br.grad)


def test_sum_classes_and_pixels():
    B, T, HW, C = 3, 7, 25, 64
    x = g(B * T * HW, 96, seed=14)
    xr = x[:, :C].reshape(B, T, HW, C)
    out = torch.ones(B * HW, C, device=DEV)
    TO.sum_classes(dev(x), out, B=B, T=T, HW=HW, C_=C, beta=1)
    close(out, xr.sum(1).reshape(B * HW, C) + 1, 1e-6)
    out2 = torch.empty(T, C, device=DEV)
    TO.sum_pixels(dev(x), out2, B=B, T=T, HW=HW, C_=C)
    close(out2, xr.sum((0, 2)), 1e-6)


def test_avgpool_and_upsample_ac_backward():
    S, H, W, C = 5, 24, 24, 16
    x = g(S, C, H, W, seed=15)
    xr = x.clone().requires_grad_(True)
    xp = F.avg_pool2d(xr, 2)
    y = F.interpolate(xp, size=(H, W), mode="bilinear", align_corners=True)
    dy = g(S, C, H, W, seed=16)
    y.backward(dy)
    # upsample backward to the pooled grid, then the pool backward
    dyn = dev(dy.permute(0, 2, 3, 1))
    dxp = torch.empty(S * 12 * 12, C, device=DEV)
    TO.upsample_ac_backward_rows(dyn, dxp, S=S, H=H, W=W, C_=C, Hp=12, Wp=12)
    dx = torch.ones(S * H * W, C, device=DEV)
    TO.avgpool_backward_rows(dxp, dx, S=S, H=H, W=W, C_=C, pool=(2, 2), beta=1)
    close(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, C) + 1)


def test_l2normalize_backward():
    x = g(300, 96, seed=17)
    dy = g(300, 96, seed=18)
    xr = x.clone().requires_grad_(True)
    F.normalize(xr, dim=-1).backward(dy)
    dx = torch.zeros(300, 96, device=DEV)
    TO.l2normalize_backward(dev(x), dev(dy), dx, rows=300, cols=96)
    close(dx, xr.grad)


@pytest.mark.parametrize("k", [2, 4])
def test_convtranspose_backward_via_gather(k):
    S, h, cin, cout = 3, 6, 32, 16
    x = g(S, cin, h, h, seed=19)
    w = g(cin, cout, k, k, seed=20) * 0.2
    b = g(cout, seed=21)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv_transpose2d(xr, wr, br, stride=k)
    dy = g(*y.shape, seed=22)
    y.backward(dy)
    G = torch.empty(S * h * h, k * k * cout, device=DEV)
    TO.convt_gather(dev(dy.permute(0, 2, 3, 1)).reshape(-1, cout), G, S=S, hin=h, win=h, k=k, cout=cout)
    Wg = dev(w.permute(2, 3, 1, 0).reshape(k * k * cout, cin))      # [(ky, kx, co)][ci]
    X = dev(x.permute(0, 2, 3, 1).reshape(-1, cin))
    dX = TO.mm(G, Wg)
    close(dX, xr.grad.permute(0, 2, 3, 1).reshape(-1, cin))
    dWg = TO.mm(G.t(), X)
    close(dWg.reshape(k, k, cout, cin).permute(3, 2, 0, 1), wr.grad)
    db = torch.empty(cout, device=DEV)
    TO.colsum(G, db, rows=S * h * h * k * k, cols=cout, ld=cout)
    close(db, br.grad)


def _window_ref(q, k, v, H, W, ws, shift, nh):
    """WindowAttention core (model.py:86-114 without the projections) over rows [S*H*W][D], the
    roll / partition / reverse of SwinTransformerBlock.forward (model.py:185-216)."""
    S = q.shape[0] // (H * W)
    D = q.shape[1]

    def part(t):
        t = t.reshape(S, H, W, D)
        if shift:
            t = torch.roll(t, (-shift, -shift), (1, 2))
        return O.window_partition(t, ws).reshape(-1, ws * ws, nh, D // nh).permute(0, 2, 1, 3)

    qw, kw, vw = part(q), part(k), part(v)
    hd = D // nh
    a = (qw * hd ** -0.5) @ kw.transpose(-2, -1)
    if shift:
        m = O.shift_mask(H, W, ws, shift).to(a.dtype)
        nw = m.shape[0]
        a = (a.view(-1, nw, nh, ws * ws, ws * ws) + m.unsqueeze(1).unsqueeze(0)).view(-1, nh, ws * ws, ws * ws)
    a = a.softmax(-1)
    o = (a @ vw).transpose(1, 2).reshape(-1, ws, ws, D)
    o = O.window_reverse(o, ws, H, W)
    if shift:
        o = torch.roll(o, (shift, shift), (1, 2))
    return o.reshape(S * H * W, D)


@pytest.mark.parametrize("shift", [0, 6])
def test_window_attention_backward(shift):
    S, H, W, ws, nh, D = 3, 24, 24, 12, 4, 128
    R = S * H * W
    qkv = g(R, 3 * D, seed=23)
    dout = g(R, D, seed=24)
    qr, kr, vr = (qkv[:, i * D:(i + 1) * D].clone().requires_grad_(True) for i in range(3))
    o = _window_ref(qr, kr, vr, H, W, ws, shift, nh)
    o.backward(dout)
    # the forward kernel's own output feeds D_q = dO . O
    qkvd = dev(qkv)
    od = torch.empty(R, D, device=DEV)
    ops.attention(qkvd[:, :D], qkvd[:, D:2 * D], qkvd[:, 2 * D:], od, n_seq=S * 4, seq_len=ws * ws, n_heads=nh,
                  head_dim=D // nh, scale=(D // nh) ** -0.5, mode=1, img_hw=(H, W), window=ws, shift=shift)
    close(od, o, 1e-5)
    dqkv = torch.empty(R, 3 * D, device=DEV)
    TO.window_attention_backward(qkvd, od, dev(dout), dqkv, S=S, img_hw=(H, W), window=ws, shift=shift, n_heads=nh,
                                 head_dim=D // nh, scale=(D // nh) ** -0.5)
    close(dqkv[:, :D], qr.grad)
    close(dqkv[:, D:2 * D], kr.grad)
    close(dqkv[:, 2 * D:], vr.grad)


@pytest.mark.parametrize("n_seq,L_,nh,causal", [(2, 577, 3, False), (5, 14, 2, True), (1, 77, 2, True),
                                                 (3, 50, 1, False)])
def test_dense_attention_backward(n_seq, L_, nh, causal):
    """CLIP nn.MultiheadAttention core (model_vpt.py:202-206; causal triu -inf mask, model_vpt.py:400-406)."""
    hd = 64
    W = nh * hd
    R = n_seq * L_
    qkv = g(R, 3 * W, seed=40)
    dout = g(R, W, seed=41)
    qr, kr, vr = (qkv[:, i * W:(i + 1) * W].clone().requires_grad_(True) for i in range(3))

    def heads(t):
        return t.reshape(n_seq, L_, nh, hd).permute(0, 2, 1, 3)

    s = (heads(qr) * hd ** -0.5) @ heads(kr).transpose(-2, -1)
    if causal:
        s = s + torch.full((L_, L_), float("-inf"), dtype=s.dtype).triu_(1)
    o = (s.softmax(-1) @ heads(vr)).permute(0, 2, 1, 3).reshape(R, W)
    o.backward(dout)
    qkvd = dev(qkv)
    od = torch.empty(R, W, device=DEV)
    ops.attention(qkvd[:, :W], qkvd[:, W:2 * W], qkvd[:, 2 * W:], od, n_seq=n_seq, seq_len=L_, n_heads=nh,
                  head_dim=hd, scale=hd ** -0.5, causal=causal)
    close(od, o, 1e-5)
    dqkv = torch.empty(R, 3 * W, device=DEV)
    TO.attention_backward(qkvd, od, dev(dout), dqkv, n_seq=n_seq, seq_len=L_, n_heads=nh, head_dim=hd,
                          scale=hd ** -0.5, causal=causal)
    close(dqkv[:, :W], qr.grad)
    close(dqkv[:, W:2 * W], kr.grad)
    close(dqkv[:, 2 * W:], vr.grad)


@pytest.mark.parametrize("T,n_pad", [(20, 236), (171, 85), (256, 0)])
def test_linear_attention_backward(T, n_pad):
    B, HW, nh, D = 2, 9, 4, 128
    hd = D // nh
    R = B * T * HW
    qkv = g(R, 3 * D, seed=25)
    kv_pad = g(2, D, seed=26)
    dy = g(R, D, seed=27)
    qr, kr, vr = (qkv[:, i * D:(i + 1) * D].clone().requires_grad_(True) for i in range(3))
    kp, vp = (kv_pad[i].clone().requires_grad_(True) for i in range(2))

    def seq(t, pad):      # rows (b, t, p) -> (b*p, T + n_pad, nh, hd)
        t = t.reshape(B, T, HW, D).permute(0, 2, 1, 3)
        if n_pad:
            t = torch.cat([t, pad.reshape(1, 1, 1, D).expand(B, HW, n_pad, D)], 2)
        return t.reshape(B * HW, T + n_pad, nh, hd)

    out = O.linear_attention(seq(qr, kp), seq(kr, kp), seq(vr, vp))[:, :T]
    out = out.reshape(B, HW, T, D).permute(0, 2, 1, 3).reshape(R, D)
    out.backward(dy)
    dqkv = torch.empty(R, 3 * D, device=DEV)
    dkp = torch.empty(D, device=DEV)
    dvp = torch.empty(D, device=DEV)
    kw = dict(k_pad=dev(kv_pad[0]), v_pad=dev(kv_pad[1]), dk_pad=dkp, dv_pad=dvp) if n_pad else {}
    TO.linear_attention_backward(dev(qkv), dev(dy), dqkv, B=B, T=T, HW=HW, n_heads=nh, head_dim=hd, n_pad=n_pad, **kw)
    close(dqkv[:, :D], qr.grad)
    close(dqkv[:, D:2 * D], kr.grad)
    close(dqkv[:, 2 * D:], vr.grad)
    if n_pad:
        close(dkp, kp.grad)
        close(dvp, vp.grad)


@pytest.mark.parametrize("cin,cout,k,relu,S", [(96, 64, 3, False, 3), (64, 32, 3, True, 3), (1, 128, 7, False, 3),
                                               (128, 16, 3, True, 3), (20, 8, 3, False, 3),
                                               (3, 16, 3, False, 3),      # scalar (cin % 4 != 0) 192-row weight tiles
                                               (32, 32, 3, True, 24),     # weight gradient split over 11 pixel ranges
                                               (96, 64, 3, False, 40)])   # 256 x 32 and 128 x 64 tiles, split-K
def test_conv2d_forward_dgrad_wgrad(cin, cout, k, relu, S):
    H, W = 24, 20
    x = g(S, cin, H, W, seed=28)
    w = g(cout, cin, k, k, seed=29) / math.sqrt(cin * k * k)
    b = g(cout, seed=30)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv2d(xr, wr, br, padding=k // 2)
    if relu:
        y = F.relu(y)
    dy = g(*y.shape, seed=31)
    y.backward(dy)
    xn = dev(x.permute(0, 2, 3, 1).reshape(-1, cin))
    wt = dev(w.permute(2, 3, 1, 0).reshape(k * k * cin, cout))         # [(tap, ci)][co]
    yd = torch.empty(S * H * W, cout, device=DEV)
    TO.conv2d(xn, wt, yd, S=S, H=H, W=W, cin=cin, cout=cout, ksize=k, bias=dev(b), act=L.ACT_RELU if relu else 0)
    close(yd, y.permute(0, 2, 3, 1).reshape(-1, cout), 1e-5)
    dyn = dev(dy.permute(0, 2, 3, 1).reshape(-1, cout))
    if relu:
        dyn = TO.act_backward(yd, dyn, L.ACT_RELU)
    dw = torch.empty(k * k * cin, cout, device=DEV)
    TO.conv2d_wgrad(xn, dyn, dw, S=S, H=H, W=W, cin=cin, cout=cout, ksize=k)
    close(dw.reshape(k, k, cin, cout).permute(3, 2, 0, 1), wr.grad)
    if cin % 4 == 0:
        # data gradient: conv of dY with the flipped, transposed weight [(tap, co)][ci]
        wf = dev(w.flip(2, 3).permute(2, 3, 0, 1).reshape(k * k * cout, cin))
        dx = torch.empty(S * H * W, cin, device=DEV)
        TO.conv2d(dyn, wf, dx, S=S, H=H, W=W, cin=cout, cout=cin, ksize=k)
        close(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, cin))


@pytest.mark.parametrize("max_norm", [0.0, 0.01, 1e6])
def test_adamw_matches_torch(max_norm):
    """cat_seg.optim.AdamW (catseg_adamw_step) vs torch.optim.AdamW behind the reference's
    FullModelGradientClippingOptimizer (train_net.py:228-253), 4 steps, three parameter groups."""
    from cat_seg.optim import AdamW
    gen = torch.Generator().manual_seed(50)
    shapes = [(128, 256), (5000,), (3, 4, 5), (1,), (4097,)]
    base = [torch.randn(*s, generator=gen) for s in shapes]
    grads = [[torch.randn(*s, generator=gen) for s in shapes] for _ in range(4)]
    mine = [b.clone().cuda().requires_grad_(True) for b in base]
    ref = [b.clone().cuda().requires_grad_(True) for b in base]

    def groups(ps):
        return [{"params": ps[:2], "lr": 2e-4, "weight_decay": 1e-4}, {"params": ps[2:4], "lr": 2e-6,
                "weight_decay": 0.0}, {"params": ps[4:], "lr": 1e-3, "weight_decay": 0.05}]

    o1 = AdamW(groups(mine), 2e-4, max_grad_norm=max_norm)
    o2 = torch.optim.AdamW(groups(ref), 2e-4)
    for st in range(4):
        for p, q, gr in zip(mine, ref, grads[st]):
            p.grad = gr.cuda()
            q.grad = gr.cuda()
        o1.step()
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(ref, max_norm)
        o2.step()
        for p, q in zip(mine, ref):
            assert (p - q).abs().max().item() <= 1e-6 * q.abs().max().item() + 1e-7
            assert (p.grad - q.grad).abs().max().item() <= 1e-6 * q.grad.abs().max().item()
    if max_norm > 0:
        tot = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g.cuda()) for g in grads[-1]]))
        assert abs(o1.last_grad_norm[0].item() - tot.item()) <= 1e-5 * tot.item()
    # the state layout is torch's: the two optimizers' state dicts load into each other
    sd = o1.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    o2.load_state_dict(sd)


def test_head_conv_backward():
    S, H, W, C = 5, 32, 24, 32
    x = g(S, C, H, W, seed=32)
    w = g(1, C, 3, 3, seed=33) / math.sqrt(9 * C)
    xr, wr = (t.clone().requires_grad_(True) for t in (x, w))
    y = F.conv2d(xr, wr, padding=1)
    dl = g(*y.shape, seed=34)
    y.backward(dl)
    dx = torch.empty(S * H * W, C, device=DEV)
    dw = torch.empty(9, C, device=DEV)
    TO.head_conv_backward(dev(x.permute(0, 2, 3, 1)), dev(dl), dev(w[0].permute(1, 2, 0).reshape(9, C)), dx, dw,
                          S=S, H=H, W=W, C_=C)
    close(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, C))
    close(dw, wr.grad[0].permute(1, 2, 0).reshape(9, C))
