"""Emulate split-K candidates for the ViT GEMMs: time gemm3 tile variants on (M', N, K') shapes whose
per-CU work equals a split-K launch (e.g. fc2 split 2 = 2M rows x K/2), next to the current automatic tile.
usage: python tools/micro_gemm_split.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

lib = L.load()
M = 8 * 577
cases = [  # name, M, N, K, variant, fp32 out
    ("fc2 auto", M, 1024, 4096, 0, True),
    ("fc2 v18 160x256 full K", M, 1024, 4096, 18, True),
    ("fc2 split2 emu v18", 2 * M, 1024, 2048, 18, True),
    ("fc2 split2 emu v1 256x256", 2 * M, 1024, 2048, 1, True),
    ("fc2 split3 emu v1 256x256", 3 * M, 1024, 1408, 1, True),
    ("fc2 split2 emu v15", 2 * M, 1024, 2048, 15, True),
    ("proj auto", M, 1024, 1024, 0, True),
    ("proj split2 emu v18", 2 * M, 1024, 512, 18, True),
    ("fc1 auto", M, 4096, 1024, 0, False),
    ("fc1 v18 160x256", M, 4096, 1024, 18, False),
    ("fc1 v1 256x256", M, 4096, 1024, 1, False),
    ("qkv auto", M, 3072, 1024, 0, False),
    ("qkv v9 pingpong", M, 3072, 1024, 9, False),
]
res = {}
for name, m, n, k, v, f32 in cases:
    A = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(n, k, device="cuda") * 2 - 1) / k ** 0.5).to(torch.bfloat16)
    out = torch.empty(m, n, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    bias = torch.rand(n, device="cuda")
    L.tune("gemm_variant", v)
    ts = []
    for r in range(7):
        ops.gemm(A, W, out, bias=bias)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.gemm(A, W, out, bias=bias)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20)
    t = sorted(ts)[3]
    print(f"{name:28s} M={m:6d} N={n:5d} K={k:5d}: {t * 1e3:7.1f} us  {2 * m * n * k / t / 1e9:7.1f} TF/s", flush=True)
L.tune("gemm_variant", 0)
