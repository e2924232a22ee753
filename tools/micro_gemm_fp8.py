"""Time the fp8 GEMM tiles (tuning knob gemm_fp8_variant) on the ViT-L/14@336 (B=8) shapes.
usage: python tools/micro_gemm_fp8.py [variants, default "0,1,15,17,19,20,21,23,24"]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,15,17,19,20,21,23,24").split(",")]
M = int(os.environ.get("MG_M", 8 * 577))     # MG_M=23080: config 5's 40 crops
shapes = {"qkv": (3072, 1024, L.ACT_NONE, False), "proj": (1024, 1024, L.ACT_NONE, True),
          "fc1": (4096, 1024, L.ACT_QUICKGELU, False), "fc2": (1024, 4096, L.ACT_NONE, True)}
dev = "cuda"
lib = L.load()
torch.manual_seed(0)
for name, (N, K, act, has_res) in shapes.items():
    A = torch.rand(M, K, device=dev) * 2 - 1
    W = (torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5
    qa = torch.empty(M, K, device=dev, dtype=torch.float8_e4m3fn); sa = torch.empty(M, device=dev)
    qw = torch.empty(N, K, device=dev, dtype=torch.float8_e4m3fn); sw = torch.empty(N, device=dev)
    ops.quant_fp8_rows(A, qa, sa); ops.quant_fp8_rows(W, qw, sw)
    bias = torch.rand(N, device=dev) - 0.5
    R = (torch.rand(M, N, device=dev) - 0.5) if has_res else None
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if has_res else torch.bfloat16)
    res = {}
    for rnd in range(5):
        for v in variants:
            L.tune("gemm_fp8_variant", v)
            try:
                ops.gemm_fp8(qa, sa, qw, sw, out, bias=bias, act=act, res=R)
            except RuntimeError:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.gemm_fp8(qa, sa, qw, sw, out, bias=bias, act=act, res=R)
            e1.record(); torch.cuda.synchronize()
            res.setdefault(v, []).append(e0.elapsed_time(e1) / 20)
    flops = 2 * M * N * K
    for v, t in res.items():
        t = sorted(t)[len(t) // 2]
        print(f"{name:5s} N={N:5d} K={K:5d} variant {v:2d}: {t * 1e3:8.1f} us {flops / t / 1e9:8.1f} TF/s")
L.tune("gemm_fp8_variant", 0)
