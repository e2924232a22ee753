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


def _rel(a, r):
    return ((a.detach().double().cpu().reshape(r.shape) - r).abs().max() / (r.abs().max() + 1e-30)).item()


def compare_grads(got, ref, keys, tol=TOL, ref32=None, report=None):
    """Per parameter: max |got - ref| / max |ref| <= max(tol, 8 x the error of torch's own fp32
    autograd of the same reference graph, ref32) — a gradient whose reference value is a heavily
    cancelled sum is as sensitive to fp32 rounding in the reference's arithmetic as in ours.
    The Swin `attn.k.bias` gradients are zero in exact arithmetic (a key bias adds q . b_k to every
    score of a query row, which softmax cancels, model.py:86-114): they are checked against the
    k weight's gradient scale instead (|got| <= 1e-5 max |d k.weight|)."""
    rows = []
    for k in keys:
        if ref[k] is None:          # a parameter off the graph (padding tokens at T == pad_len; the dense
            # block's q / k projections, whose outputs the reference discards: zeros here)
            assert got[k] is None or not got[k].abs().max().item(), f"{k}: gradient where the reference has none"
            continue
        r = ref[k].double()
        gk = got[k]
        assert gk is not None, f"{k}: no gradient"
        if ".swin_block." in k and k.endswith("attn.k.bias"):
            wscale = ref[k[:-len("bias")] + "weight"].double().abs().max().item()
            a = gk.detach().double().abs().max().item()
            assert a <= 1e-5 * wscale, (k, a, wscale)
            continue
        e = _rel(gk, r)
        e32 = _rel(ref32[k], r) if ref32 is not None else 0.0
        rows.append((e, e32, k))
    rows.sort(reverse=True)
    if report is not None:
        report.extend(rows)
    bad = [x for x in rows if x[0] > max(tol, 8 * x[1])]
    assert not bad, f"gradients off (rel err hip, rel err torch-fp32, key): {bad[:5]}; worst {rows[:3]}"
    return rows


def _write_report(name, rows):
    d = os.environ.get("CATSEG_GRAD_REPORT")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"grad_{name}.txt"), "w") as f:
            f.write("rel_err_hip\trel_err_torch_fp32\tparameter\n")
            for e, e32, k in rows:
                f.write(f"{e:.3e}\t{e32:.3e}\t{k}\n")


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

    # reference: fp64 autograd through the oracle (and the same graph in torch fp32, the noise floor)
    ref_grads = {}
    for dt, store in ((torch.float64, ref_grads), (torch.float32, {})):
        sdr = {k: v.detach().clone().to(dt).requires_grad_(k in keys) for k, v in sd.items()}
        lg = ref_head(arch, sdr, feats.to(dt), [h.permute(1, 0, 2).to(dt) for h in hooks], text.to(dt))
        l_ = ref_loss(lg, targets)
        l_.backward()
        store.update({k: sdr[k].grad for k in keys})
        if dt == torch.float64:
            ref_logits, rl = lg, l_
        else:
            ref32 = store

    # HIP: fp32 on the device, autograd Functions backed by the training kernels
    P = {k: v.detach().cuda().requires_grad_(k in keys) for k, v in sd.items()}
    logits = head_train_forward(arch, P, feats.reshape(B * L_, -1).float().cuda(),
                                [h.reshape(B * L_, -1).float().cuda() for h in hooks], text.float().cuda())
    assert logits.shape == (B, T, R, R) and logits.requires_grad
    assert (logits.detach().cpu().double() - ref_logits.detach()).abs().max().item() < 1e-4
    loss = ops.BCEOneHotLoss.apply(logits, targets.cuda(), 255)
    assert abs(loss.item() - rl.item()) <= 1e-5 * abs(rl.item())
    loss.backward()
    rows = []
    try:
        compare_grads({k: P[k].grad for k in keys}, ref_grads, keys, ref32=ref32, report=rows)
    finally:
        _write_report(case, rows)


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
        P = {k: v.detach().cuda().requires_grad_(k in keys) for k, v in sd.items()}
        ops.BCEOneHotLoss.apply(head_train_forward(arch, P, feats, hooks, text), targets, 255).backward()
        runs.append({k: P[k].grad.clone() for k in keys})
    for k in keys:
        assert torch.equal(runs[0][k], runs[1][k]), k


def test_clip_encoders_backward_matches_oracle_autograd():
    """The CLIP image encoder (blocks, forward_dense, hooks, ln_post @ proj) and the causal text encoder
    (EOT gather, ln_final @ text_projection, L2 norm) as autograd Functions, every transformer-block
    parameter trained (CLIP_FINETUNE "full", cat_seg_model.py:70-71), vs fp64 autograd through the
    oracle (model_vpt.py:202-240,288-314,421-438) on a random linear loss of every output."""
    from cat_seg.engine import CatSegEngine
    from cat_seg.training import clip_image_train_forward, clip_text_train_forward
    from cat_seg.weights import CLIP
    arch = TINY
    sd = synthesize_state_dict(arch, seed=0)
    keys = [k for k in sd if k.startswith(CLIP) and "transformer.resblocks" in k]
    gen = torch.Generator().manual_seed(4)
    B, T = 2, 7
    ims = [torch.randint(0, 256, (3, 384, 384), generator=gen).float() for _ in range(B)]
    toks = torch.zeros(T, arch.context_length, dtype=torch.long)
    toks[:, 0] = 1
    for t in range(T):
        n = 3 + t % 4
        toks[t, 1:n] = torch.randint(2, 400, (n - 1,), generator=gen)
        toks[t, n] = arch.vocab_size - 1
    L_ = arch.grid ** 2 + 1
    rf = torch.randn(B, L_, arch.embed_dim, generator=gen, dtype=torch.float64)
    rh = [torch.randn(B, L_, arch.vision_width, generator=gen, dtype=torch.float64) for _ in range(2)]
    rt = torch.randn(T, arch.embed_dim, generator=gen, dtype=torch.float64)

    refs = {}
    for dt in (torch.float64, torch.float32):
        sdr = {k: v.detach().clone().to(dt).requires_grad_(k in keys) for k, v in sd.items()}
        clip_ims, _ = O.preprocess(arch, ims)
        feats, hooks = O.encode_image_dense(arch, sdr, clip_ims.to(dt))
        text = O.text_embeds(arch, sdr, toks)[:, 0]
        loss = (feats * rf.to(dt)).sum() + (text * rt.to(dt)).sum()
        for h, r in zip(hooks, rh):
            loss = loss + (h.permute(1, 0, 2) * r.to(dt)).sum()
        loss.backward()
        refs[dt] = {k: sdr[k].grad for k in keys}

    eng = CatSegEngine(arch, sd, dtype=torch.float32, device="cuda")
    P = {k: v.detach().cuda().requires_grad_(k in keys) for k, v in sd.items()}
    raw = torch.stack(ims).cuda()
    sizes = torch.tensor([[384, 384]] * B, dtype=torch.int32, device="cuda")
    feats, hooks = clip_image_train_forward(arch, P, eng, raw, sizes)
    text = clip_text_train_forward(arch, P, eng, toks)
    loss = (feats * rf.reshape(B * L_, -1).float().cuda()).sum() + (text * rt.float().cuda()).sum()
    for h, r in zip(hooks, rh):
        loss = loss + (h * r.reshape(B * L_, -1).float().cuda()).sum()
    loss.backward()
    rows = []
    try:
        compare_grads({k: P[k].grad for k in keys}, refs[torch.float64], keys, ref32=refs[torch.float32], report=rows)
    finally:
        _write_report("clip_encoders", rows)


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
    # CLIP_FINETUNE "attention": the head, the upsamplers and the CLIP q / v projections train
    keys = [k for k, p in named.items() if p.requires_grad]
    assert any("visual.transformer.resblocks.0.attn.q_proj_weight" in k for k in keys)
    assert any(k.endswith("clip_model.transformer.resblocks.0.attn.v_proj_weight") for k in keys)
    assert all(named[k].grad is not None for k in keys)
    assert all(named[k].grad is None for k in named if k not in keys)

    # reference from the same images, every stage in fp64 (CLIP q / v with grad), and torch fp32
    arch = model.arch
    refs = {}
    for dt in (torch.float64, torch.float32):
        sdr = {k: v.detach().cpu().clone().to(dt) for k, v in named.items()}
        for k in keys:
            sdr[k].requires_grad_(True)
        clip_ims, _ = O.preprocess(arch, ims)
        feats, hooks = O.encode_image_dense(arch, sdr, clip_ims.to(dt))
        text = O.text_embeds(arch, sdr, toks)[:, 0]
        rl = ref_loss(ref_head(arch, sdr, feats, hooks, text), torch.stack(sems).int())
        rl.backward()
        refs[dt] = ({k: sdr[k].grad for k in keys}, rl.item())
    rl64 = refs[torch.float64][1]
    assert abs(loss.item() - rl64) <= 1e-5 * abs(rl64)
    rows = []
    try:
        compare_grads({k: named[k].grad for k in keys}, refs[torch.float64][0], keys, ref32=refs[torch.float32][0],
                      report=rows)
    finally:
        _write_report("catseg_train_step", rows)

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


def test_catseg_train_step_matches_reference_gradients():
    """The whole training step pinned to the REFERENCE's own modules, not the oracle: the loss and every
    trainable parameter's gradient against tests/golden/train_tiny_pool2.npz, which
    tests/golden/make_golden.py ("train") produced by running the reference's model_vpt.CLIP and
    Aggregator (requires_grad per cat_seg_model.py:57-75, loss per :189-203, text per
    cat_seg_predictor.py:190-224) in float64 on the same inputs.  Per parameter, an evenly strided
    sample of the flattened gradient and its max magnitude are compared, gate max(1e-4, 8 x the same
    reference graph's own float32 error); the Swin k biases (zero in exact arithmetic) against the k
    weights' scale."""
    import numpy as np
    from conftest import ROOT
    g = np.load(os.path.join(ROOT, "tests", "golden", "train_tiny_pool2.npz"))
    cfg = tiny_cfg(**{"MODEL.SEM_SEG_HEAD.POOLING_SIZES": "[2,2]"})
    model = build_model(cfg).cuda()
    model.sem_seg_head.predictor.set_class_tokens(torch.from_numpy(g["tokens"]))
    ims = [torch.from_numpy(g["image0"]).float(), torch.from_numpy(g["image1"]).float()]
    tg = torch.from_numpy(g["targets"]).long()
    model.train()
    loss = model([{"image": ims[i], "sem_seg": tg[i]} for i in range(2)])["loss_sem_seg"]
    loss.backward()
    l64 = float(g["loss64"])
    assert abs(loss.item() - l64) <= 1e-5 * abs(l64), (loss.item(), l64)
    named = dict(model.named_parameters())
    names = [str(k) for k in g["names"]]
    assert {k for k, p in named.items() if p.requires_grad} == set(names) | {str(k) for k in g["none"]}
    rows = []
    try:
        for k in names:
            mx, e32 = (float(v) for v in g["m_" + k])
            got = named[k].grad.detach().double().cpu().reshape(-1)
            if ".swin_block." in k and k.endswith("attn.k.bias"):
                scale = float(g["m_" + k[:-len("bias")] + "weight"][0])
                assert got.abs().max().item() <= 1e-5 * scale, k
                continue
            if mx == 0.0:                 # the dense block's dead q / k projections
                assert got.abs().max().item() == 0.0, k
                continue
            idx = torch.from_numpy(g["i_" + k])
            err = max((got[idx] - torch.from_numpy(g["g_" + k])).abs().max().item() / mx,
                      abs(got.abs().max().item() - mx) / mx)
            rows.append((err, e32, k))
            assert err <= max(TOL, 8 * e32), f"{k}: {err:.3e} (reference fp32 {e32:.3e})"
    finally:
        _write_report("reference_modules_train_step", sorted(rows, reverse=True))


def test_hip_adamw_step_refreshes_the_eval_engine():
    """the HIP AdamW (cat_seg.optim, as build_optimizer returns it) writes the parameters
    through raw pointers; the eval forward after its step must run on the UPDATED weights (the engine is
    keyed on the parameters' version counters), checked against the oracle on the new state dict."""
    from cat_seg.optim import AdamW, build_optimizer
    cfg = tiny_cfg(**{"SOLVER.CLIP_GRADIENTS.ENABLED": "True", "SOLVER.CLIP_GRADIENTS.CLIP_TYPE": "full_model",
                      "SOLVER.CLIP_GRADIENTS.CLIP_VALUE": "0.01", "SOLVER.BASE_LR": "0.01"})
    model = build_model(cfg).cuda()
    T = 5
    gen = torch.Generator().manual_seed(11)
    toks = torch.zeros(T, 16, dtype=torch.long)
    toks[:, 0] = 1
    toks[:, 1:4] = torch.randint(2, 400, (T, 3), generator=gen)
    toks[:, 4] = 511
    model.sem_seg_head.predictor.set_class_tokens(toks)
    ims = [torch.randint(0, 256, (3, 384, 384), generator=gen).float()]
    sems = [torch.randint(0, T, (384, 384), generator=gen)]
    model.eval()
    with torch.no_grad():
        out0 = model([{"image": ims[0]}])[0]["sem_seg"].clone()
    opt = build_optimizer(cfg, model)
    assert isinstance(opt, AdamW)
    model.train()
    model([{"image": i, "sem_seg": s} for i, s in zip(ims, sems)])["loss_sem_seg"].backward()
    versions = [p._version for p in model.parameters()]
    opt.step()
    torch.cuda.synchronize()
    assert any(p._version != v for p, v in zip(model.parameters(), versions))
    model.eval()
    with torch.no_grad():
        out1 = model([{"image": ims[0]}])[0]["sem_seg"]
    assert not torch.equal(out1, out0)
    arch = model.arch
    sd_new = {k: v.detach().cpu() for k, v in model.named_parameters()}
    ref = O.catseg_forward(arch, sd_new, [{"image": ims[0]}], O.text_embeds(arch, sd_new, toks))[0]["sem_seg"]
    assert (out1.cpu() - ref).abs().max().item() < 1e-3
