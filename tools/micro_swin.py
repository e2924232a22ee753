"""Time the fused Swin window kernel variants (tuning knob swin_variant) at config 3 (S = 1200 slices,
24x24, 12x12 windows, 4 heads x 32) for shift 0 and 6, and compare their outputs.
usage: python tools/micro_swin.py [variants, default 0,3]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L
from cat_seg._lib import rowmap

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,3").split(",")]
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
out = torch.empty(R, D, device=dev, dtype=dt)
for shift in (0, 6):
    def run():
        ops.swin_window_attention(X, (g1, b1), W, bias, gqk, gmap, out, S=S, img_hw=(24, 24), window=12, shift=shift,
                                  n_heads=4, head_dim=32, scale=32 ** -0.5)
    res, ref = {}, None
    for v in variants:
        L.tune("swin_variant", v)
        run(); torch.cuda.synchronize()
        o = out.float().clone()
        ref = o if ref is None else ref
        res[v] = {"diff": (o - ref).abs().max().item(), "t": [], "ck": out.view(torch.int16).double().abs().sum().item()}
    for r in range(5):
        for v in variants:
            L.tune("swin_variant", v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record(); torch.cuda.synchronize()
            res[v]["t"].append(e0.elapsed_time(e1) / 5)
    for v in variants:
        print(f"shift {shift} variant {v}: {sorted(res[v]['t'])[2] * 1e3:7.1f} us  max diff vs first {res[v]['diff']:.3e}"
              f"  checksum {res[v]['ck']:.0f}",
              flush=True)
L.tune("swin_variant", 0)
