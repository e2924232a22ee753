"""Time catseg_preprocess_im2col (normalise + bilinear resize of the padded 352² canvas to 336² +
14x14 patch im2col, bf16, K padded to 640) at the headline shape (bs 8) and print a checksum, so
that two libraries (CATSEG_HIP_LIB) can be compared bit for bit.
usage: python tools/micro_pre.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops

torch.manual_seed(0)
B, S, pad, res, patch, ld = 8, 336, 352, 336, 14, 640
G = res // patch
raw = torch.zeros(B, 3, pad, pad, device="cuda")
raw[:, :, :S, :S] = torch.rand(B, 3, S, S, device="cuda") * 255
sizes = torch.tensor([[S, S]] * B, dtype=torch.int32, device="cuda")
mean = torch.tensor([122.7709383, 116.7460125, 104.09373615], device="cuda")
std = torch.tensor([68.5005327, 66.6321579, 70.32316305], device="cuda")
for dt in (torch.bfloat16, torch.float32):
    out = torch.empty(B * G * G, ld, device="cuda", dtype=dt)
    run = lambda: ops.preprocess_im2col(raw, sizes, mean=mean, std=std, res=res, patch=patch, out=out)
    run(); torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    t = sorted(ts)[3]
    nb = raw.numel() * 4 + out.numel() * out.element_size()
    print(f"preprocess_im2col {dt}: {t:.1f} us  {nb / t / 1e6:.2f} TB/s  checksum "
          f"{out.double().sum().item():.6f} {out.double().abs().sum().item():.6f}", flush=True)
