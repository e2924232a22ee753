"""Time catseg_upconv_addend (the Up blocks' guidance half + ConvT bias, conv_partial_vec_kernel<.., true>)
at the bs=8 L/14@336 shapes: Up1 (48², cin 32 -> cout 64) and Up2 (96², cin 16 -> cout 32)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

torch.manual_seed(0)
B = 8
for name, (Ho, cin, cout) in {"up1": (48, 32, 64), "up2": (96, 16, 32)}.items():
    g = torch.randn(B, Ho, Ho, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, 9 * cin, device="cuda") / 12
    tb = torch.randn(9, cout, device="cuda")
    outs = {}
    for v in (0, 1):                    # tuning knob partial_mfma: 0 = VALU kernel, 1 = MFMA kernel
        L.tune("partial_mfma", v)
        out = torch.empty(B * (Ho // 2) ** 2, 4 * cout, device="cuda")
        ops.upconv_addend(g, w, tb, out, B=B, H2=Ho, W2=Ho)
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                ops.upconv_addend(g, w, tb, out, B=B, H2=Ho, W2=Ho)
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 50 * 1e3)
        outs[v] = out
        print(f"{name} partial_mfma={v}: {sorted(ts)[3]:.1f} us", flush=True)
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"{name}: max |mfma - valu| {d:.2e} (max |out| {outs[0].abs().max().item():.2f})", flush=True)
    L.tune("partial_mfma", 1)
