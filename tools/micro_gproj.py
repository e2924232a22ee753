"""Time the guidance-projection convs (catseg_conv3x3 on the im2col kernel with split-K) at the bs=8
L/14@336 shapes: gp (24², 768 -> 128), dgp0 (48², 256 -> 32), dgp1 (96², 128 -> 16); weight layout
[cout][9 * cin] as the engine passes it."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

torch.manual_seed(0)
B = 8
for name, (H, cin, cout) in {"gp": (24, 768, 128), "dgp0": (48, 256, 32), "dgp1": (96, 128, 16)}.items():
    x = torch.randn(B * H * H, cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, 9 * cin, device="cuda") / (3 * cin ** 0.5)).to(torch.bfloat16)
    b = torch.randn(cout, device="cuda")
    out = torch.empty(B * H * H, cout, device="cuda", dtype=torch.bfloat16)
    ops.conv3x3(x, w, out, S=B, H=H, W=H, c1=cin, bias=b, act=L.ACT_RELU)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.conv3x3(x, w, out, S=B, H=H, W=H, c1=cin, bias=b, act=L.ACT_RELU)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    print(f"{name}: {sorted(ts)[3]:.1f} us (conv + split-K reduce)", flush=True)
