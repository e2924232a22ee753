"""Anatomy of the ViT residual-stream GEMMs (out-proj / fc2 at M = 4616): time the automatic tile at
the engine's epilogue and with parts removed, and at scaled K / M / N, to split a launch into
per-K-step, per-tile and epilogue time.

usage: python tools/micro_gemm_anatomy.py [variant, default 0 = automatic]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch  # noqa: E402

from cat_seg import _lib as L  # noqa: E402
from cat_seg import ops  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else 0
L.tune("gemm_variant", v)
dev = "cuda"
torch.manual_seed(0)


def case(name, M, N, K, out_dt, res):
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    bias = torch.rand(N, device=dev) - 0.5
    R = (torch.rand(M, N, device=dev) - 0.5) if res else None
    out = torch.empty(M, N, device=dev, dtype=out_dt)

    def run():
        ops.gemm(A, W, out, bias=bias, res=R)
    run()
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t() + bias + (R if res else 0)
    err = (out.float() - ref).abs().max().item()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    t = sorted(ts)[3]
    byts = M * K * 2 + N * K * 2 + M * N * (4 if out_dt == torch.float32 else 2) + (M * N * 4 if res else 0)
    print(f"{name:28s} M={M:5d} N={N:5d} K={K:5d}: {t:7.1f} us  {2 * M * N * K / t / 1e6:7.1f} TF/s  "
          f"{byts / t / 1e3:6.2f} TB/s  err {err:.2e}", flush=True)


M = 8 * 577
f32, b16 = torch.float32, torch.bfloat16
case("out-proj (engine)", M, 1024, 1024, f32, True)
case("out-proj no residual", M, 1024, 1024, f32, False)
case("out-proj bf16 out", M, 1024, 1024, b16, False)
case("out-proj K=512", M, 1024, 512, f32, True)
case("out-proj K=2048", M, 1024, 2048, f32, True)
case("out-proj M/2", M // 2, 1024, 1024, f32, True)
case("out-proj M/4", M // 4, 1024, 1024, f32, True)
case("out-proj N=512", M, 512, 1024, f32, True)
case("fc2 (engine)", M, 1024, 4096, f32, True)
case("fc2 no residual", M, 1024, 4096, f32, False)
case("fc2 M/2", M // 2, 1024, 4096, f32, True)
case("qkv", M, 3072, 1024, b16, False)
case("fc1 (no act)", M, 4096, 1024, b16, False)
L.tune("gemm_variant", 0)
