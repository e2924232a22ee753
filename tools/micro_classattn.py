"""A/B of the class-attention kernels at the bench shape (B=8, HW=576, T=150 / 256), one process,
interleaved rounds; prints per-launch µs (median) and the max |diff| between the variants."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cat-seg_amd")]
from cat_seg import ops, _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    lib = L.load()
    for T, n_pad in ((150, 106), (256, 0)):
        B, HW, D = 8, 576, 128
        R = B * T * HW
        X = (torch.randn(R, D, device=dev) * 2).to(torch.bfloat16)
        g1, b1 = 1 + 0.2 * torch.randn(D, device=dev), 0.2 * torch.randn(D, device=dev)
        W = (torch.randn(3 * D, D, device=dev) / D ** 0.5).to(torch.bfloat16)
        bias = 0.1 * torch.randn(3 * D, device=dev)
        tg = (0.5 * torch.randn(T, 2 * D, device=dev)).to(torch.bfloat16)
        kp, vp = torch.randn(D, device=dev), torch.randn(D, device=dev)
        ys = {}
        variants = [int(v) for v in os.environ.get("CA_VARIANTS", "0").split(",")] + \
            [int(v) for v in os.environ.get("CA_DBG", "").split(",") if v]
        times = {v: [] for v in variants}
        for rnd in range(7):
            for v in variants:
                L.tune("classattn_variant", v)
                y = torch.empty_like(X)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.class_attention(X, (g1, b1), W, bias, tg, y, B=B, T=T, HW=HW, n_heads=4, head_dim=32,
                                    n_pad=n_pad, k_pad=kp, v_pad=vp)
                e1.record()
                torch.cuda.synchronize()
                if rnd > 0:
                    times[v].append(e0.elapsed_time(e1) * 1e3)
                ys[v] = y
        L.tune("classattn_variant", 0)
        d = (ys[variants[0]].float() - ys[variants[-1]].float()).abs()
        med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
        print(f"T={T}: max|diff| first/last variant {d.max().item():.3e} mean {d.mean().item():.3e}"
              + "".join(f"  v{v} {med[v]:.1f} us" for v in variants)
              + f"  checksum {ys[variants[0]].view(torch.int16).double().abs().sum().item():.0f}", flush=True)


if __name__ == "__main__":
    main()
