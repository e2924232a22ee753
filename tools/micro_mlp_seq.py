"""ViT MLP GEMMs in sequence vs alone (L/14@336, bs 8): fc1 (QuickGELU, bf16 out) then fc2 (fp32
residual in place), each timed with HIP events, against fc2 repeated on its own.
usage: python tools/micro_mlp_seq.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

M, D, H = 8 * 577, 1024, 4096
torch.manual_seed(0)
dev = "cuda"
h = (torch.rand(M, D, device=dev) - 0.5).to(torch.bfloat16)
w1 = ((torch.rand(H, D, device=dev) - 0.5) / 16).to(torch.bfloat16)
b1 = torch.rand(H, device=dev) - 0.5
w2 = ((torch.rand(D, H, device=dev) - 0.5) / 32).to(torch.bfloat16)
b2 = torch.rand(D, device=dev) - 0.5
x = torch.rand(M, D, device=dev) - 0.5
u = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
fc1 = lambda: ops.gemm(h, w1, u, bias=b1, act=L.ACT_QUICKGELU)
fc2 = lambda: ops.gemm(u, w2, x, bias=b2, res=x)
for _ in range(3):
    fc1(); fc2()
torch.cuda.synchronize()
def timed(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(n):
            fn()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1e3)
    return sorted(ts)[2]
t1, t2 = timed(fc1), timed(fc2)
t12 = timed(lambda: (fc1(), fc2()))
print(f"back to back: fc1 {t1:.1f} us, fc2 {t2:.1f} us, sum {t1 + t2:.1f}; fc1 + fc2 interleaved {t12:.1f} us per pair")
