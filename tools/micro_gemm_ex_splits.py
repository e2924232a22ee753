"""Split-K sweep for catseg_gemm_ex on the training step's GEMM shapes (tuning knob gemm_ex_splits):
time each forced split count against the automatic choice (0) in one process.

usage: python tools/micro_gemm_ex_splits.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch  # noqa: E402

from cat_seg import _lib as L  # noqa: E402
from cat_seg import train_ops as TO  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
shapes = [(2308, 3072, 768, "k"), (2308, 768, 3072, "k"), (2308, 768, 2304, "k"), (768, 768, 2308, "m"),
          (512, 512, 2052, "m"), (2052, 2048, 512, "k"), (2052, 512, 2048, "k"), (2052, 512, 512, "k"),
          (384, 128, 393984, "m"), (768, 3072, 2308, "m"), (3072, 768, 2308, "m")]
for M, N, K, ao in shapes:
    A = torch.randn(K, M, device=dev) if ao == "m" else torch.randn(M, K, device=dev)
    B = torch.randn(K, N, device=dev)
    Aop = A.t() if ao == "m" else A
    out = torch.empty(M, N, device=dev)
    ref = Aop.double() @ B.double()
    res = []
    for sp in (0, 1, 2, 3, 4, 6, 8, 12, 16, 32):
        L.tune("gemm_ex_splits", sp)
        TO.mm(Aop, B, out=out)
        torch.cuda.synchronize()
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                TO.mm(Aop, B, out=out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        res.append((sp, sorted(ts)[2], err))
    L.tune("gemm_ex_splits", 0)
    print(f"M={M:6d} N={N:5d} K={K:7d} A {ao}-contig: " +
          "  ".join(f"s{sp}:{t:6.1f}us" for sp, t, _ in res) + f"  max rel err {max(e for *_, e in res):.1e}",
          flush=True)
