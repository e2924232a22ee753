"""Time catseg_sliding_merge at config 5's shape (8 images x 5 crops, T = 459, 96² logits -> 640²)
for values of tuning knob merge_variant (0 = tabulated staged merge, 1 = band kernel, 2 = staged
merge), same process, and print every value's max difference from the first's.
usage: python tools/micro_merge.py [variants, default 2,0]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,0").split(",")]
lib = L.load()
torch.manual_seed(0)
N, T = 8, 459
lg = torch.randn(N * 5, T, 96, 96, device="cuda") * 4
outs = {}
for v in variants:
    L.tune("merge_variant", v)
    outs[v] = torch.empty(N, T, 640, 640, device="cuda")
    ops.sliding_merge(lg, outs[v], kernel=384, stride=256, out_res=640)
torch.cuda.synchronize()
ts = {v: [] for v in variants}
for _ in range(5):
    for v in variants:
        L.tune("merge_variant", v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.sliding_merge(lg, outs[v], kernel=384, stride=256, out_res=640)
        e1.record(); torch.cuda.synchronize()
        ts[v].append(e0.elapsed_time(e1) / 3)
L.tune("merge_variant", 0)
gb = N * T * 640 * 640 * 4 / 1e9
for v in variants:
    t = sorted(ts[v])[2]
    print(f"merge variant {v}: {t:.3f} ms  ({gb / t:.2f} TB/s of output)  max diff vs {variants[0]}: "
          f"{(outs[v] - outs[variants[0]]).abs().max().item():.2e}", flush=True)
