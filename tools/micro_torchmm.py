"""torch.mm (hipBLASLt) on the ViT-L/14@336 bs=8 GEMM shapes, for kernel-name / timing
comparison under rocprofv3 --kernel-trace --stats."""
import torch
M = 8 * 577
for name, (N, K) in {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}.items():
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.nn.functional.linear(A, W, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.nn.functional.linear(A, W, b)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{name}: {t:.1f} us  {2 * M * N * K / t / 1e6:.0f} TFLOP/s", flush=True)
