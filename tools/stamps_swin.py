"""Phase stamps of the Swin window kernel (swin_variant 16): s_memtime at the window start, after the
window barrier, after P1 (LayerNorm), after the P1 barrier, after P2 (projection), after the P2
barrier and after P3 (attention), for the first 4 windows of every wave, at config 3's shape
(S = 1200 slices).  Prints the median cycles of each phase over waves and windows 1..3, split by
sub-wave (tiles 5 / 4).
usage: python tools/stamps_swin.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L
from cat_seg._lib import rowmap

lib = L.load()
B, T, HW, D = 8, 150, 576, 128
S, R = B * T, B * T * HW
dev, dt = "cuda", torch.bfloat16
torch.manual_seed(0)
X = torch.randn(R, D, device=dev).to(dt)
W = (torch.randn(3 * D, D, device=dev) / 11).to(dt)
bias = torch.randn(3 * D, device=dev) * 0.1
g1, b1 = 1 + torch.randn(D, device=dev) * 0.1, torch.randn(D, device=dev) * 0.1
gqk = (torch.randn(B * HW, 2 * D, device=dev) * 0.3).to(dt)
gmap = rowmap(d1=T * HW, s1=HW, d2=1, m2=HW, s2=1)
grid = 256
extra = grid * 8 * 32 * 8 // (2 * D) + 1               # rows of 256 bytes past the output
names = ["wait+barrier", "P1 LayerNorm", "P1 barrier", "P2 projection", "P2 barrier", "P3 attention"]
for shift in (0, 6):
    out = torch.zeros(R + extra, D, device=dev, dtype=dt)
    L.tune("swin_variant", 16)
    for _ in range(3):
        ops.swin_window_attention(X, (g1, b1), W, bias, gqk, gmap, out[:R], S=S, img_hw=(24, 24), window=12,
                                  shift=shift, n_heads=4, head_dim=32, scale=32 ** -0.5)
    torch.cuda.synchronize()
    L.tune("swin_variant", 0)
    st = out[R:].view(torch.int64).flatten()[:grid * 8 * 32].reshape(grid, 8, 4, 8).cpu()
    d = (st[..., 1:7] - st[..., 0:6]).double()            # (grid, wave, window, phase)
    tot = (st[..., 6] - st[..., 0]).double()
    for sub in (0, 1):
        sel = d[:, 4 * sub:4 * sub + 4, 1:4].reshape(-1, 6)
        med = sel.median(0).values
        print(f"shift {shift} sub {sub} ({'5' if sub == 0 else '4'} tiles): " +
              "  ".join(f"{n} {v:.0f}" for n, v in zip(names, med.tolist())) +
              f"  | window {tot[:, 4 * sub:4 * sub + 4, 1:4].median().item():.0f} cycles", flush=True)
