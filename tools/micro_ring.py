"""Time the decoder ring-conv knobs (tuning knob ring_variant) on the config-3 decoder shapes
(1200 slices; Up1 48x48, Up2 96x96) and check every variant against variant 0.
usage: python tools/micro_ring.py [variants, default "0,1,2,3,4"]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4").split(",")]
lib = L.load()
torch.manual_seed(0)
S, B, T = 1200, 8, 150
dt = torch.bfloat16
cases = {}
for name, (H, c1, co, add) in {"up1_conv1": (48, 96, 64, True), "up1_conv2": (48, 64, 64, False),
                               "up2_conv1": (96, 48, 32, True), "up2_conv2": (96, 32, 32, False)}.items():
    x = (torch.randn(S * H * H, c1, device="cuda") * 0.5).to(dt)
    w = (torch.randn(co, 9 * c1, device="cuda") / (3 * c1 ** 0.5)).to(dt)
    out = torch.empty(S * H * H, co, device="cuda", dtype=dt)
    kw = dict(S=S, H=H, W=H, c1=c1)
    if add:
        kw.update(addend=torch.randn(B * H * H, co, device="cuda"), addend_div=T)
    else:
        g = co // 16
        kw.update(gn=(torch.zeros(S * (c1 // 16), device="cuda"), torch.ones(S * (c1 // 16), device="cuda"),
                      torch.ones(c1, device="cuda"), torch.zeros(c1, device="cuda"), 16))
    cases[name] = (x, w, out, kw)
res, outs = {}, {}
for rnd in range(3):
    for v in variants:
        pass  # one tiling per shape since round 4 (ring_variant removed)
        for name, (x, w, out, kw) in cases.items():
            tile = ops.conv3x3_stats_tile(x, w, **kw)
            st = torch.empty(S * (kw["H"] * kw["W"] // tile) * (w.shape[0] // 16) * 2, device="cuda")
            ops.conv3x3(x, w, out, stats=st, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                ops.conv3x3(x, w, out, stats=st, **kw)
            e1.record(); torch.cuda.synchronize()
            res.setdefault((name, v), []).append(e0.elapsed_time(e1) / 5)
            if rnd == 0:
                outs[(name, v)] = out.clone()

for name in cases:
    for v in variants:
        t = sorted(res[(name, v)])[1]
        d = (outs[(name, v)].float() - outs[(name, 0)].float()).abs().max().item() if 0 in variants else 0
        print(f"{name:10s} variant {v}: {t * 1e3:8.1f} us   max diff vs v0 {d:.2e}", flush=True)
