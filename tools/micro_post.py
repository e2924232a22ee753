"""Time the headline's two output kernels at bs 8, T 150 (1200 planes): catseg_conv3x3_head_gn (32 -> 1
head conv on 96^2 with GN+ReLU in, tuning knob head_variant) and catseg_postprocess (sigmoid + bilinear
96^2 -> 336^2); check every head variant against the first bit for bit.
usage: python tools/micro_post.py [head variants, default 0,3]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,3").split(",")]
L.load()
torch.manual_seed(0)
B, T, C, H, W = 8, 150, 32, 96, 96
S = B * T
x = torch.randn(S * H * W, C, device="cuda").to(torch.bfloat16)
mean, rstd = torch.randn(S * 2, device="cuda") * 0.2, torch.rand(S * 2, device="cuda") + 1
gam, bet = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
w = torch.randn(9 * C, device="cuda") / 8
logits = {v: torch.empty(B, T, H, W, device="cuda") for v in variants}
def head(v):
    L.tune("head_variant", v)
    ops.conv3x3_head(x, B=B, T=T, H=H, W=W, C=C, weight=w, bias=0.25, out=logits[v], T_out=T, classes=None,
                     gn=(mean, rstd, gam, bet, 16))
post_out = torch.empty(B, T, 336, 336, device="cuda")
def post(v):
    ops.postprocess(logits[variants[0]], post_out, crop=(96, 96))
fns = [(f"head v{v}", head, v) for v in variants] + [("postprocess", post, 0)]
for name, f, v in fns:
    f(v)
torch.cuda.synchronize()
ts = {name: [] for name, _, _ in fns}
for _ in range(5):
    for name, f, v in fns:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f(v)
        e1.record(); torch.cuda.synchronize()
        ts[name].append(e0.elapsed_time(e1) / 5 * 1e3)
L.tune("head_variant", 0)
for name, f, v in fns:
    eq = torch.equal(logits[v], logits[variants[0]]) if name.startswith("head") else ""
    print(f"{name}: {sorted(ts[name])[2]:.1f} us {eq}", flush=True)
