"""Phase stamps of classattn2 (debug variant 16+4): per pixel LN / A / B cycles (s_memtime)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cat-seg_amd")]
from cat_seg import ops, _lib as L  # noqa: E402

dev = torch.device("cuda")
lib = L.load()
B, HW, D, T = 8, 576, 128, 150
R = B * T * HW
X = (torch.randn(R, D, device=dev) * 2).to(torch.bfloat16)
g1, b1 = 1 + 0.2 * torch.randn(D, device=dev), 0.2 * torch.randn(D, device=dev)
W = (torch.randn(3 * D, D, device=dev) / D ** 0.5).to(torch.bfloat16)
bias = 0.1 * torch.randn(3 * D, device=dev)
tg = (0.5 * torch.randn(T, 2 * D, device=dev)).to(torch.bfloat16)
kp, vp = torch.randn(D, device=dev), torch.randn(D, device=dev)
for v in (16 + 4, 16 + 4 + 3):
    L.tune("classattn_variant", v)
    for _ in range(3):
        y = torch.zeros_like(X)
        ops.class_attention(X, (g1, b1), W, bias, tg, y, B=B, T=T, HW=HW, n_heads=4, head_dim=32, n_pad=106,
                            k_pad=kp, v_pad=vp)
        torch.cuda.synchronize()
    st = y.reshape(-1).view(torch.int64)[: 512 * 64].view(512, 64)[:, :32].view(512, 8, 4).cpu().double()
    ln, A, Bq = (st[:, :, 1] - st[:, :, 0]), (st[:, :, 2] - st[:, :, 1]), (st[:, :, 3] - st[:, :, 2])
    tot = st[:, 7, 3] - st[:, 0, 0]
    print(f"variant {v}: cycles per pixel (median over WGs, pixels 1-7): LN {ln[:, 1:].median():.0f}  "
          f"A {A[:, 1:].median():.0f}  B {Bq[:, 1:].median():.0f}  8 pixels total {tot.median():.0f}", flush=True)
L.tune("classattn_variant", 0)
