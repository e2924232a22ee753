"""Attention mode 2's folded q scaling against the unscaled CLIP weights (engine.py _block).

The bf16 engine multiplies the ViT q projection by head_dim^-0.5 * log2(e) in fp32 before the bf16
rounding (catseg_attention mode 2), so its stored q weights round differently from a bf16 cast of
the reference's unscaled weights.  One ResidualAttentionBlock (model_vpt.py:193-217) through the
engine with the folded q (mode 2) and with the unscaled q (mode 0) is compared with the same block in
float64 on the unscaled weights: the folding must cost no accuracy against that reference."""
import pytest
import torch

from cat_seg.arch import TINY
from cat_seg.engine import CatSegEngine
from cat_seg.weights import CLIP, synthesize_state_dict

pytestmark = pytest.mark.gpu


def block_fp64(x, sd, p, heads):
    """ResidualAttentionBlock.forward in float64 (model_vpt.py:193-217, QuickGELU MLP)."""
    g = {k[len(p):]: v.double() for k, v in sd.items() if k.startswith(p)}
    M, D = x.shape
    hd = D // heads

    def ln(t, w, b):
        return torch.nn.functional.layer_norm(t, (D,), w, b, 1e-5)

    h = ln(x, g["ln_1.weight"], g["ln_1.bias"])
    b = g["attn.in_proj_bias"]
    q = h @ g["attn.q_proj_weight"].t() + b[:D]
    k = h @ g["attn.k_proj_weight"].t() + b[D:2 * D]
    v = h @ g["attn.v_proj_weight"].t() + b[2 * D:]
    return q, k, v, g, ln, hd


@pytest.mark.parametrize("n_seq,L", [(2, 50), (3, 197)])
def test_folded_q_scale_costs_no_accuracy(n_seq, L):
    sd = synthesize_state_dict(TINY, seed=0)
    eng = CatSegEngine(TINY, sd, dtype=torch.bfloat16)
    assert eng.vit_l2s
    heads = TINY.vision_heads
    p = f"{CLIP}visual.transformer.resblocks.0."
    D = TINY.vision_width
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(n_seq * L, D, generator=gen, dtype=torch.float64)

    q, k, v, g, ln, hd = block_fp64(x, sd, p, heads)
    split = lambda t: t.reshape(n_seq, L, heads, hd).transpose(1, 2)
    a = torch.softmax(split(q) @ split(k).transpose(-1, -2) * hd ** -0.5, -1) @ split(v)
    y = x + a.transpose(1, 2).reshape(n_seq * L, D) @ g["attn.out_proj.weight"].t() + g["attn.out_proj.bias"]
    u = ln(y, g["ln_2.weight"], g["ln_2.bias"]) @ g["mlp.c_fc.weight"].t() + g["mlp.c_fc.bias"]
    u = u * torch.sigmoid(1.702 * u)
    ref = y + u @ g["mlp.c_proj.weight"].t() + g["mlp.c_proj.bias"]

    errs = {}
    for mode, heads_fold in (("mode2", heads), ("mode0", 0)):
        blk = eng._block(sd, p, heads=heads_fold)
        xd = x.float().cuda().contiguous()
        out = eng._resblocks(xd, [blk], n_seq, L, heads, False, l2s=heads_fold > 0)
        d = (out.double().cpu() - ref).abs()
        errs[mode] = (d.max().item(), d.mean().item())
    scale = ref.abs().max().item()
    print(f"n_seq {n_seq} L {L}: max|ref| {scale:.3f}; mode 2 (folded q) max / mean err "
          f"{errs['mode2'][0]:.3e} / {errs['mode2'][1]:.3e}, mode 0 (unscaled q) "
          f"{errs['mode0'][0]:.3e} / {errs['mode0'][1]:.3e}")
    # both within the bf16 engine's budget, and the folded form no worse than the unscaled one
    # beyond bf16 noise (mean error within 10 %, max within 25 %)
    for m in errs:
        assert errs[m][0] < 3e-2 * scale, (m, errs[m])
    assert errs["mode2"][1] <= 1.10 * errs["mode0"][1] + 1e-6, errs
    assert errs["mode2"][0] <= 1.25 * errs["mode0"][0] + 1e-6, errs
