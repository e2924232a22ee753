"""The aggregation head's backward on the device against torch autograd through
the pinned oracle (oracle/catseg_oracle.py, itself checked against the reference's own modules by
tests/test_oracle_golden.py) in float64 on the CPU.

Gate: every head parameter's gradient (Aggregator + the CATSeg ConvTranspose upsamplers) within
1e-4 of its largest reference magnitude (max |hip - ref| <= 1e-4 * max |ref|), fp32 HIP vs fp64 ref,
plus the loss itself within 1e-5 relative.  Geometries: TINY (the tests' narrow CLIP) with the
training config's POOLING [2,2] and class padding (T < pad_len), POOLING [1,1], no padding
(T == pad_len), and ViT-B/16's widths (C_o 512, hook width 768) with POOLING [2,2].
"""
import os

import pytest
import torch
import torch.nn.functional as F

from cat_seg import build_model, ops
from cat_seg.arch import TINY, VIT_B16
from cat_seg.training import head_train_forward
from cat_seg.weights import AGG, synthesize_state_dict
from oracle import catseg_oracle as O

from test_boundary_cpu import tiny_cfg

pytestmark = pytest.mark.gpu
torch.set_num_threads(min(16, os.cpu_count() or 1))

TOL = 1e-4


def ref_loss(logits, targets, ignore=255):
    """cat_seg_model.py:190-201 (interpolate to the target size, one-hot, BCE-with-logits mean)."""
    out = F.interpolate(logits, size=targets.shape[-2:], mode="bilinear", align_corners=False)
    T = out.shape[1]
    mask = targets != ignore
    out = out.permute(0, 2, 3, 1)
    tg = torch.zeros(out.shape, dtype=out.dtype)
    tg[mask] = F.one_hot(targets[mask].long(), num_classes=T).to(out.dtype)
    return F.binary_cross_entropy_with_logits(out, tg)


def ref_head(arch, sd, feats, hooks, text):
    """cat_seg_model.py:178-188 from the CLIP outputs: feats (B, 1+HW, C_o), hooks 2 x (L, B, W)
    sequence-first, text (T, C_o) -> logits (B, T, 4G, 4G) through the oracle's Aggregator."""
    B, g = feats.shape[0], arch.grid
    res3 = feats[:, 1:, :].reshape(B, g, g, -1).permute(0, 3, 1, 2)
    res4 = hooks[0][1:].permute(1, 2, 0).reshape(B, -1, g, g)
    res5 = hooks[1][1:].permute(1, 2, 0).reshape(B, -1, g, g)
    res4 = F.conv_transpose2d(res4, sd["upsample1.weight"], sd["upsample1.bias"], stride=2)
    res5 = F.conv_transpose2d(res5, sd["upsample2.weight"], sd["upsample2.bias"], stride=4)
    text_b = text.unsqueeze(1).unsqueeze(0).expand(B, -1, -1, -1)
    return O.aggregator(arch, sd, res3, text_b, [res3, res4, res5])


def head_keys(sd):
    return [k for k in sd if k.startswith(AGG) or k.startswith("upsample")]


def compare_grads(got, ref, keys, tol=TOL):
    worst = []
    for k in keys:
        r = ref[k].double()
        gk = got[k]
        assert gk is not None, f"{k}: no gradient"
        gk = gk.detach().double().cpu().reshape(r.shape)
        e = ((gk - r).abs().max() / (r.abs().max() + 1e-30)).item()
        worst.append((e, k))
    worst.sort(reverse=True)
    assert worst[0][0] <= tol, f"worst gradients (rel err, key): {worst[:5]}"
    return worst


CASES = {
    "tiny_pool2_pad": (TINY.replace(pooling_size=(2, 2)), 2, 20),
    "tiny_pool1_pad": (TINY, 2, 12),
    "tiny_pool2_nopad": (TINY.replace(pooling_size=(2, 2), pad_len=24), 1, 24),
    "vitb16_pool2_pad": (VIT_B16.replace(pooling_size=(2, 2)), 1, 16),
}


@pytest.mark.parametrize("case", list(CASES))
def test_head_backward_matches_oracle_autograd(case):
    arch, B, T = CASES[case]
    sd = synthesize_state_dict(arch, seed=0)
    keys = head_keys(sd)
    L_ = arch.grid ** 2 + 1
    gen = torch.Generator().manual_seed(5)
    feats = torch.randn(B, L_, arch.embed_dim, generator=gen, dtype=torch.float64)
    hooks = [torch.randn(B, L_, arch.vision_width, generator=gen, dtype=torch.float64) for _ in range(2)]
    text = F.normalize(torch.randn(T, arch.embed_dim, generator=gen, dtype=torch.float64), dim=-1)
    R = 4 * arch.grid
    targets = torch.randint(0, T, (B, R, R), generator=gen, dtype=torch.int32)
    targets[:, :3] = 255

    # reference: fp64 autograd through the oracle
    sd64 = {k: v.double().requires_grad_(k in keys) for k, v in sd.items()}
    ref_logits = ref_head(arch, sd64, feats, [h.permute(1, 0, 2) for h in hooks], text)
    rl = ref_loss(ref_logits, targets)
    rl.backward()
    ref_grads = {k: sd64[k].grad for k in keys}

    # HIP: fp32 on the device, autograd Functions backed by the training kernels
    P = {k: v.cuda().requires_grad_(k in keys) for k, v in sd.items()}
    logits = head_train_forward(arch, P, feats.reshape(B * L_, -1).float().cuda(),
                                [h.reshape(B * L_, -1).float().cuda() for h in hooks], text.float().cuda())
    assert logits.shape == (B, T, R, R) and logits.requires_grad
    assert (logits.detach().cpu().double() - ref_logits.detach()).abs().max().item() < 1e-4
    loss = ops.BCEOneHotLoss.apply(logits, targets.cuda(), 255)
    assert abs(loss.item() - rl.item()) <= 1e-5 * abs(rl.item())
    loss.backward()
    compare_grads({k: P[k].grad for k in keys}, ref_grads, keys)


def test_head_backward_is_deterministic():
    """Two backward passes of the same step give bit-identical gradients (no atomics)."""
    arch, B, T = CASES["tiny_pool2_pad"]
    sd = synthesize_state_dict(arch, seed=0)
    keys = head_keys(sd)
    L_ = arch.grid ** 2 + 1
    gen = torch.Generator().manual_seed(9)
    feats = torch.randn(B * L_, arch.embed_dim, generator=gen).cuda()
    hooks = [torch.randn(B * L_, arch.vision_width, generator=gen).cuda() for _ in range(2)]
    text = F.normalize(torch.randn(T, arch.embed_dim, generator=gen), dim=-1).cuda()
    targets = torch.randint(0, T, (B, 96, 96), generator=gen, dtype=torch.int32).cuda()
    runs = []
    for _ in range(2):
        P = {k: v.cuda().requires_grad_(k in keys) for k, v in sd.items()}
        ops.BCEOneHotLoss.apply(head_train_forward(arch, P, feats, hooks, text), targets, 255).backward()
        runs.append({k: P[k].grad.clone() for k in keys})
    for k in keys:
        assert torch.equal(runs[0][k], runs[1][k]), k


def test_catseg_train_step_backward_and_optimizer():
    """model.train(); model(batch)["loss_sem_seg"].backward() fills .grad of every Aggregator and
    upsampler parameter (vs the oracle from the same images, CLIP in fp64 included); torch.optim.AdamW
    steps the real nn.Parameters and the next eval forward runs on the updated weights."""
    cfg = tiny_cfg(**{"MODEL.SEM_SEG_HEAD.POOLING_SIZES": "[2,2]"})
    model = build_model(cfg).cuda()
    T = 9
    gen = torch.Generator().manual_seed(3)
    toks = torch.zeros(T, 16, dtype=torch.long)
    toks[:, 0] = 1
    toks[:, 1:4] = torch.randint(2, 400, (T, 3), generator=gen)
    toks[:, 4] = 511                                     # EOT = the argmax id
    model.sem_seg_head.predictor.set_class_tokens(toks)
    ims = [torch.randint(0, 256, (3, 384, 384), generator=gen).float() for _ in range(2)]
    sems = [torch.randint(0, T, (384, 384), generator=gen) for _ in range(2)]
    sems[0][:20] = 255
    model.train()
    loss = model([{"image": i, "sem_seg": s} for i, s in zip(ims, sems)])["loss_sem_seg"]
    assert loss.requires_grad
    loss.backward()
    named = dict(model.named_parameters())
    keys = head_keys(named)
    assert all(named[k].grad is not None for k in keys)
    assert all(named[k].grad is None for k in named if k.startswith("sem_seg_head.predictor.clip_model"))

    # reference from the same images, every stage in fp64 (CLIP frozen: no_grad)
    arch = model.arch
    sd64 = {k: v.detach().cpu().double() for k, v in named.items()}
    for k in keys:
        sd64[k].requires_grad_(True)
    with torch.no_grad():
        clip_ims, _ = O.preprocess(arch, ims)
        feats, hooks = O.encode_image_dense(arch, sd64, clip_ims.double())
        text = O.text_embeds(arch, sd64, toks)[:, 0]
    rl = ref_loss(ref_head(arch, sd64, feats, hooks, text), torch.stack(sems).int())
    assert abs(loss.item() - rl.item()) <= 1e-5 * abs(rl.item())
    rl.backward()
    compare_grads({k: named[k].grad for k in keys}, {k: sd64[k].grad for k in keys}, keys)

    # an optimizer step on the real parameters; eval then runs on the new weights
    before = model.engine.w.ce_b.clone()
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad and p.grad is not None], lr=1e-3)
    opt.step()
    model.eval()
    with torch.no_grad():
        out = model([{"image": ims[0]}])[0]["sem_seg"]
    assert not torch.equal(model.engine.w.ce_b, before)
    sd_new = {k: v.detach().cpu() for k, v in model.named_parameters()}
    ref = O.catseg_forward(arch, sd_new, [{"image": ims[0]}], O.text_embeds(arch, sd_new, toks))[0]["sem_seg"]
    assert (out.cpu() - ref).abs().max().item() < 1e-3
