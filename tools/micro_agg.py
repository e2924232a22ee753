"""Run selected aggregation kernels on full config-3 shapes (for rocprofv3 --pmc runs)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L
which = sys.argv[1] if len(sys.argv) > 1 else "all"
S, HW, D = 1200, 576, 128
R = S * HW
dev = "cuda"
qkv = (torch.randn(R, 3 * D, device=dev) * 0.5).to(torch.bfloat16)
o = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
X = (torch.randn(R, D, device=dev)).to(torch.bfloat16)
w1 = (torch.randn(512, D, device=dev) / 11).to(torch.bfloat16); b1 = torch.zeros(512, device=dev)
w2 = (torch.randn(D, 512, device=dev) / 22).to(torch.bfloat16); b2 = torch.zeros(D, device=dev)
g, b = torch.ones(D, device=dev), torch.zeros(D, device=dev)
def attn():
    ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, n_seq=S * 4, seq_len=144, n_heads=4, head_dim=32,
                  scale=32 ** -0.5, mode=1, img_hw=(24, 24), window=12, shift=6)
def mlp():
    ops.rows_mlp(X, w1, b1, w2, X, ln=(g, b), b2=b2, act=L.ACT_GELU, res=X)
fns = {"attn": attn, "mlp": mlp}
sel = [fns[which]] if which in fns else list(fns.values())
for f in sel:
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5): f()
    torch.cuda.synchronize()
    print(f.__name__, (time.perf_counter() - t0) / 5 * 1e3, "ms")
