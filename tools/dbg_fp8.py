"""fp8 GEMM diagnostics: exact small-integer operands (any k-order mismatch shows) and
random operands (error vs fp64 of the dequantized product)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "cat-seg_amd"), os.path.join(os.path.dirname(__file__), "..")]
import torch
from cat_seg import ops, _lib as L

dev = "cuda"
torch.manual_seed(0)
for M, N, K in ((256, 256, 128), (1200, 768, 1024)):
    A = torch.randint(-4, 5, (M, K)).float()
    W = torch.randint(-4, 5, (N, K)).float()
    qa, qw = A.to(torch.float8_e4m3fn), W.to(torch.float8_e4m3fn)
    sa, sw = torch.ones(M), torch.ones(N)
    out = torch.empty(M, N, device=dev)
    ops.gemm_fp8(qa.to(dev), sa.to(dev), qw.to(dev), sw.to(dev), out)
    ref = A.double() @ W.double().T
    d = (out.cpu().double() - ref).abs()
    print(f"int {M}x{N}x{K}: max err {d.max().item()}, n wrong {(d > 0).sum().item()} / {d.numel()}")
    # one-hot probe: A = e_k rows
    for kk in (0, 1, 31, 32, 64, 127):
        A1 = torch.zeros(M, K); A1[:, kk] = 1.0
        W1 = torch.zeros(N, K); W1[:, kk] = 1.0
        out = torch.empty(M, N, device=dev)
        ops.gemm_fp8(A1.to(torch.float8_e4m3fn).to(dev), sa.to(dev), W1.to(torch.float8_e4m3fn).to(dev), sw.to(dev), out)
        print("  onehot k", kk, "sum", out.sum().item(), "expect", M * N)
    for scale in (1.0, 1e-3):
        A = (torch.rand(M, K) * 2 - 1) * 448 * scale
        W = (torch.rand(N, K) * 2 - 1) * 448 * scale
        qa, qw = A.to(torch.float8_e4m3fn), W.to(torch.float8_e4m3fn)
        out = torch.empty(M, N, device=dev)
        ops.gemm_fp8(qa.to(dev), sa.to(dev), qw.to(dev), sw.to(dev), out)
        ref = qa.double() @ qw.double().T
        d = (out.cpu().double() - ref).abs()
        print(f"rand scale {scale}: max err {d.max().item():.4g} rel {(d.max() / ref.abs().max()).item():.3g}")
        nz = qa.float().abs() < 2 ** -6
        print("  subnormal fraction A", nz.float().mean().item())
        # flush subnormals in the reference and compare
        qa2 = torch.where(qa.float().abs() < 2 ** -6, torch.zeros(()), qa.float()).double()
        qw2 = torch.where(qw.float().abs() < 2 ** -6, torch.zeros(()), qw.float()).double()
        d2 = (out.cpu().double() - qa2 @ qw2.T).abs()
        print(f"  vs FTZ reference: max err {d2.max().item():.4g}")
