"""Time catseg_swin_proj_mlp (Swin proj + residual + LN + MLP) and catseg_rows_mlp (class MLP, ReLU)
at the headline's shapes (8 images x 150 classes x 576 pixels = 691200 rows of 128, bf16), print a
checksum of each output.  Run it once per library (CATSEG_HIP_LIB) on one box for an A/B.
usage: python tools/micro_mlp.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

L.load()
torch.manual_seed(0)
R, D, H = 1200 * 576, 128, 512
dev = "cuda"
bf = torch.bfloat16
attn = torch.randn(R, D, device=dev).to(bf)
x = torch.randn(R, D, device=dev).to(bf)
wp = (torch.randn(D, D, device=dev) / 11).to(bf); bp = torch.randn(D, device=dev) * 0.1
w1 = (torch.randn(H, D, device=dev) / 11).to(bf); b1 = torch.randn(H, device=dev) * 0.1
w2 = (torch.randn(D, H, device=dev) / 22).to(bf); b2 = torch.randn(D, device=dev) * 0.1
g, b = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev) * 0.1
out = torch.empty_like(x)
def swin():
    ops.swin_proj_mlp(attn, x, wp, bp, w1, b1, w2, b2, out, ln=(g, b))
def cls():
    ops.rows_mlp(x, w1, b1, w2, out, ln=(g, b), b2=b2, act=L.ACT_RELU, res=x)
for name, f in (("swin_proj_mlp", swin), ("rows_mlp relu", cls)):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    f(); torch.cuda.synchronize()
    print(f"{name}: {sorted(ts)[2] * 1e3:.1f} us  checksum {out.float().sum().item():.6e}", flush=True)
