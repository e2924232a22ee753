"""Time catseg_corr_embed (the cost volume's 7x7 Conv2d(1, 128), bf16 out) at the headline shape
(L/14@336, bs 8, 150 classes: 1200 slices of 24 x 24) and print a checksum of the output, so that two
libraries (CATSEG_HIP_LIB) can be compared bit for bit.
usage: python tools/micro_corr.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops

torch.manual_seed(0)
B, T, G, D = 8, 150, 24, 128
HW = G * G
corr = torch.randn(T, B * HW, device="cuda") * 0.3
w = torch.randn(D, 49, device="cuda") / 7
bias = torch.randn(D, device="cuda") * 0.1
out = torch.empty(B * T * HW, D, device="cuda", dtype=torch.bfloat16)
run = lambda: ops.corr_embed(corr, t_stride=B * HW, b_stride=HW, B=B, T=T, H=G, W=G, weight=w, bias=bias, out=out)
run(); torch.cuda.synchronize()
ts = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
t = sorted(ts)[3]
print(f"corr_embed: {t:.1f} us  {out.numel() * 2 / t / 1e6:.2f} TB/s written  checksum "
      f"{out.float().double().sum().item():.6f} {out.view(torch.int16).double().abs().sum().item():.0f}")
