"""Time the four headline decoder convs (L/14@336, bs 8, T 150: S = 1200 slices) under values of
one tuning knob, interleaved in one process, and check each value's outputs against the first's
bit for bit: Up1 fold (24x24x128 -> 4 parities x 64), Up1 conv2 (48x48, 64 -> 64, GN+ReLU in),
Up2 fold (relu(GN(48x48x64)) -> 4 x 32), Up2 conv2 (96x96, 32 -> 32, GN+ReLU in).
usage: python tools/micro_decoder.py ring_onebar 0 1"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

knob, values = sys.argv[1], [int(v) for v in sys.argv[2:]]
L.load()
dev, dt = "cuda", torch.bfloat16
B, T = 8, 150
S = B * T
torch.manual_seed(0)


def gn_args(c):
    return (torch.rand(S * c // 16, device=dev) * 0.1, 1 + torch.rand(S * c // 16, device=dev),
            torch.rand(c, device=dev), torch.rand(c, device=dev) * 0.1, 16)


cases = {}
for name, H, ci, co, gn in (("up1_fold", 24, 128, 64, False), ("up2_fold", 48, 64, 32, True)):
    src = (torch.rand(S * H * H, ci, device=dev) - 0.5).to(dt)
    w = ((torch.rand(4 * co, 9 * ci, device=dev) - 0.5) / 16).to(dt)
    add = torch.rand(B * H * H, 4 * co, device=dev)
    out = torch.empty(S * 4 * H * H, co, device=dev, dtype=dt)
    st = torch.empty(S * (4 * H * H // ops.upconv3x3_stats_tile()) * (co // 16) * 2, device=dev)
    g = gn_args(ci) if gn else None
    cases[name] = (lambda src=src, w=w, out=out, H=H, ci=ci, g=g, st=st, add=add:
                   ops.upconv3x3(src, w, out, S=S, H=H, W=H, c1=ci, gn=g, stats=st, addend=add, addend_div=T), out)
for name, H, ci, co in (("up1_conv2", 48, 64, 64), ("up2_conv2", 96, 32, 32)):
    x = (torch.randn(S * H * H, ci, device=dev) * 0.5).to(dt)
    w = (torch.randn(co, 9 * ci, device=dev) / (3 * ci ** 0.5)).to(dt)
    out = torch.empty(S * H * H, co, device=dev, dtype=dt)
    kw = dict(S=S, H=H, W=H, c1=ci, gn=gn_args(ci))
    st = torch.empty(S * (H * H // 32) * (co // 16) * 2, device=dev)   # >= any tile's partial count
    cases[name] = (lambda x=x, w=w, out=out, kw=kw, st=st: ops.conv3x3(x, w, out, stats=st, **kw), out)

res, outs = {}, {}
for rnd in range(5):
    for v in values:
        L.tune(knob, v)
        for name, (run, out) in cases.items():
            run()
            if rnd == 0:
                torch.cuda.synchronize()
                outs[(name, v)] = out.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record(); torch.cuda.synchronize()
            res.setdefault((name, v), []).append(e0.elapsed_time(e1) / 5)
L.tune(knob, values[0])
for name in cases:
    for v in values:
        t = sorted(res[(name, v)])[2]
        same = torch.equal(outs[(name, v)], outs[(name, values[0])])
        ck = outs[(name, v)].view(torch.int16).double().abs().sum().item()
        print(f"{name:10s} {knob}={v}: {t * 1e3:8.1f} us   bit-identical to {values[0]}: {same}  checksum {ck:.0f}",
              flush=True)
