"""gemm8 diagnostics: split the ping-pong GEMM's time into fixed (prologue + epilogue) and
per-K-tile cost.  usage: python tools/micro_gemm8.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L
lib = L.load()
M = 8 * 577
dev = "cuda"


def timeit(fn, n=20, rounds=5):
    """n launches captured in one hipGraph (no host launch overhead in the timing)."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay(); torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1e3)
    return sorted(ts)[len(ts) // 2]


for N, outdt in ((3072, torch.bfloat16), (1024, torch.float32)):
    for K in (64, 256, 1024, 4096):
        A = (torch.rand(M, K, device=dev) - 0.5).to(torch.bfloat16)
        W = (torch.rand(N, K, device=dev) - 0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=outdt)
        row = []
        for v in (9, 10, 5):
            row.append(timeit(lambda: (L.tune("gemm_variant", v), ops.gemm(A, W, out))))
        tm = timeit(lambda: torch.mm(A, W.t()))
        print(f"N={N} K={K:5d} out={str(outdt)[6:]:9s} gemm8 {row[0]:7.1f} us  mainloop-only {row[1]:7.1f} us  "
              f"128x128 {row[2]:7.1f} us  torch.mm {tm:7.1f} us", flush=True)
L.tune("gemm_variant", 0)
