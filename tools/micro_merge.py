"""Time catseg_sliding_merge at config 5's shape (8 images x 5 crops, T = 459, 96² logits -> 640²)
for tuning knob merge_variant 0 (LDS-staged tile rows) and 1 (band kernel), same process."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

lib = L.load()
torch.manual_seed(0)
N, T = 8, 459
lg = torch.randn(N * 5, T, 96, 96, device="cuda") * 4
out = torch.empty(N, T, 640, 640, device="cuda")
ts = {0: [], 1: []}
outs = {}
for v in (0, 1):
    L.tune("merge_variant", v)
    o = torch.empty_like(out) if v else out
    ops.sliding_merge(lg, o, kernel=384, stride=256, out_res=640)
    outs[v] = o
torch.cuda.synchronize()
for _ in range(5):
    for v in (0, 1):
        L.tune("merge_variant", v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.sliding_merge(lg, outs[v], kernel=384, stride=256, out_res=640)
        e1.record(); torch.cuda.synchronize()
        ts[v].append(e0.elapsed_time(e1) / 3)
L.tune("merge_variant", 0)
print(f"merge: variant 0 {sorted(ts[0])[2]:.3f} ms  variant 1 {sorted(ts[1])[2]:.3f} ms  identical {torch.equal(outs[0], outs[1])}",
      flush=True)
