import os, sys
sys.path[:0] = [os.path.join(os.environ["GRAFT_REPO_ROOT"], "cat-seg_amd"), os.environ["GRAFT_REPO_ROOT"]]
import torch, torch.nn.functional as F
from cat_seg import ops
B, T, H, W, c1, co = 1, 1, 96, 96, 48, 32
g = torch.Generator().manual_seed(0)
x = (torch.rand(B * T, c1, H, W, generator=g) * 2 - 1)
w = (torch.rand(co, c1, 3, 3, generator=g) * 2 - 1) / 8
dt = torch.bfloat16
ref = F.conv2d(x.to(dt).double(), w.to(dt).double(), padding=1)[0]
a1 = x.permute(0, 2, 3, 1).contiguous().to("cuda", dt)
wk = w.permute(0, 2, 3, 1).reshape(co, -1).contiguous().to("cuda", dt)
out = torch.zeros(H * W, co, device="cuda", dtype=dt)
ops.conv3x3(a1, wk, out, S=1, H=H, W=W, c1=c1)
got = out.reshape(H, W, co).permute(2, 0, 1).double().cpu()
err = (got - ref).abs() > 2 ** -7 * ref.abs() + 1e-3
print("bad frac", err.double().mean().item())
print("bad per channel", err.reshape(co, -1).double().mean(1))
pix = err.any(0).reshape(-1).nonzero().reshape(-1)
print("bad pixels (first 40)", pix[:40].tolist())
print("bad pixel mod 128 hist", torch.bincount(pix % 128, minlength=128).tolist())
