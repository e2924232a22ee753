"""Time the ViT LayerNorm (fp32 rows of 1024 -> bf16) per tuning knob ln_variant at the bs=8 / bs=4
row counts, same process; check every variant against the first bit for bit.
usage: python tools/micro_ln.py [variants, default 0,1]  (back-to-back launches are launch-bound at ~10 us:
read the per-kernel times from rocprofv3 --kernel-trace --stats around it)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]
L.load()
torch.manual_seed(0)
for rows in (4616, 2308):
    x = torch.randn(rows, 1024, device="cuda") * 3
    g, b = torch.rand(1024, device="cuda") + 0.5, torch.randn(1024, device="cuda")
    outs, ts = {}, {v: [] for v in variants}
    for v in variants:
        L.tune("ln_variant", v)
        outs[v] = torch.empty(rows, 1024, device="cuda", dtype=torch.bfloat16)
        ops.layernorm(x, g, b, outs[v])
    torch.cuda.synchronize()
    for _ in range(7):
        for v in variants:
            L.tune("ln_variant", v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.layernorm(x, g, b, outs[v])
            e1.record(); torch.cuda.synchronize()
            ts[v].append(e0.elapsed_time(e1) / 20 * 1e3)
    L.tune("ln_variant", 0)
    mb = rows * 1024 * 6 / 1e6
    print(f"rows {rows}: " + "  ".join(
        f"v{v} {sorted(ts[v])[3]:.2f} us ({mb / sorted(ts[v])[3]:.2f} TB/s, equal {torch.equal(outs[v], outs[variants[0]])})"
        for v in variants), flush=True)
