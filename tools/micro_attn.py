"""Time the dense attention tilings (tuning knob attn_variant) on the ViT-L/14@336 shape
(8 images x 16 heads x 577 tokens, head_dim 64, bf16) and check them against variant 0.
usage: python tools/micro_attn.py [variants, default "0,200"]
variant 200: mode 2 (q pre-scaled by scale * log2(e); the engine's ViT path)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,200").split(",")]
B, Lq, H, d = 8, 577, 16, 64
lib = L.load()
torch.manual_seed(0)
qkv = (torch.randn(B * Lq, 3 * H * d, device="cuda") * 0.5).to(torch.bfloat16)
out = torch.empty(B * Lq, H * d, device="cuda", dtype=torch.bfloat16)
qkv2 = qkv.clone()
qkv2[:, :H * d] = (qkv[:, :H * d].float() * (d ** -0.5 * 1.4426950408889634)).to(torch.bfloat16)
mode = [0]
def run():
    x = qkv2 if mode[0] == 2 else qkv
    ops.attention(x[:, :H * d], x[:, H * d:2 * H * d], x[:, 2 * H * d:], out, n_seq=B, seq_len=Lq, n_heads=H,
                  head_dim=d, scale=d ** -0.5, mode=mode[0])
def setv(v):
    mode[0] = 2 if v >= 200 else 0
    L.tune("attn_variant", 0 if v >= 200 else v)

L.tune("attn_variant", 0); run(); ref = out.clone()
flops = 4 * B * H * Lq * Lq * d
res = {}
for rnd in range(5):
    for v in variants:
        setv(v)
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record(); torch.cuda.synchronize()
        res.setdefault(v, []).append(e0.elapsed_time(e1) / 20)
for v in variants:
    setv(v); run(); torch.cuda.synchronize()
    err = (out.float() - ref.float()).abs().max().item()
    t = sorted(res[v])[2]
    ck = out.view(torch.int16).double().abs().sum().item()
    print(f"variant {v}: {t * 1e3:7.1f} us  {flops / t / 1e9:6.1f} TF/s  max diff vs v0 {err:.2e}  checksum {ck:.0f}",
          flush=True)
setv(0)
