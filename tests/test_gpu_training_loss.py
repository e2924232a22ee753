"""The training branch's loss (cat_seg_model.py:189-203) on the device: catseg_bce_onehot_loss vs
the reference's own arithmetic (F.interpolate bilinear align_corners=False to the target size,
one-hot targets with ignore rows left zero, F.binary_cross_entropy_with_logits mean) in fp64, and
CATSeg.forward in training mode; the loss's backward to the logits (catseg_bce_onehot_loss_backward)
vs torch autograd of the same arithmetic.  The network itself has no backward."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cat_seg import build_model, ops

from conftest import GOLDEN
from test_boundary_cpu import tiny_cfg

pytestmark = pytest.mark.gpu


def reference_loss(logits, targets, ignore):
    """cat_seg_model.py:190-201, restated on CPU float64."""
    out = F.interpolate(logits.double(), size=targets.shape[-2:], mode="bilinear", align_corners=False)
    T = out.shape[1]
    mask = targets != ignore
    out = out.permute(0, 2, 3, 1)
    tg = torch.zeros(out.shape, dtype=torch.float64)
    tg[mask] = F.one_hot(targets[mask].long(), num_classes=T).double()
    return F.binary_cross_entropy_with_logits(out, tg).item()


@pytest.mark.parametrize("B,T,h,w,H,W", [(2, 7, 24, 24, 96, 96), (3, 150, 24, 24, 50, 37), (1, 5, 96, 96, 384, 512)])
def test_bce_onehot_loss_matches_reference(B, T, h, w, H, W):
    g = torch.Generator().manual_seed(B * 100 + T)
    logits = torch.randn(B, T, h, w, generator=g) * 3
    targets = torch.randint(0, T, (B, H, W), generator=g, dtype=torch.int32)
    targets[torch.rand(B, H, W, generator=g) < 0.2] = 255                 # ignore_value pixels
    got = ops.bce_onehot_loss(logits.cuda(), targets.cuda(), 255).item()
    ref = reference_loss(logits, targets, 255)
    assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-6, (got, ref)
    # deterministic: fixed-order reduction
    assert ops.bce_onehot_loss(logits.cuda(), targets.cuda(), 255).item() == got


def test_catseg_training_forward_loss():
    """model.train(); model(batched_inputs with "sem_seg") -> {"loss_sem_seg"} equal to the
    reference loss of the same head logits (the eval path's logits, checked elsewhere against
    the reference goldens)."""
    gd = dict(np.load(os.path.join(GOLDEN, "e2e_tiny_pad.npz")))
    model = build_model(tiny_cfg(**{"MODEL.CATSEG_HIP.DTYPE": "f32"})).cuda()
    model.sem_seg_head.predictor.set_class_tokens(gd["tokens"])
    model.arch = model.arch.replace(pad_len=int(gd["pad_len"]))
    model._engine = None
    im = torch.from_numpy(gd["image0"])
    H, W = im.shape[-2:]
    T = len(gd["tokens"])
    g = torch.Generator().manual_seed(7)
    sem = torch.randint(0, T, (H, W), generator=g)
    sem[:4] = 255
    batch = [{"image": im, "sem_seg": sem}, {"image": im, "sem_seg": sem.flip(-1)}]
    model.train()
    losses = model(batch)
    assert set(losses) == {"loss_sem_seg"} and losses["loss_sem_seg"].dim() == 0
    assert losses["loss_sem_seg"].requires_grad      # the head's HIP backward (tests/test_gpu_train_head.py)
    model.eval()
    eng = model.engine
    model.sem_seg_head.predictor.get_text_embeds()      # the eval engine's class set (= the train tokens here)
    raw, sizes_dev, _ = model._batch(eng, [b["image"] for b in batch])
    with torch.no_grad():
        logits = eng.head_logits(raw, sizes_dev).cpu()
    ref = reference_loss(logits, torch.stack([b["sem_seg"] for b in batch]).int(), 255)
    got = losses["loss_sem_seg"].item()
    assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-6, (got, ref)


def test_train_eval_alternation_keeps_the_test_class_set():
    """eval -> train step -> eval with different train / test class lists (Trainer with EVAL_PERIOD):
    the second eval must run on the test classes again, bit for bit the first eval's output, and the
    training step must see the train classes (its loss equals the loss of the train-class logits)."""
    gd = dict(np.load(os.path.join(GOLDEN, "e2e_tiny_pad.npz")))
    model = build_model(tiny_cfg(**{"MODEL.CATSEG_HIP.DTYPE": "f32"})).cuda()
    test_tok, train_tok = gd["tokens"], gd["tokens"][::-1][:7].copy()      # 10 test classes, 7 train classes
    model.sem_seg_head.predictor.set_class_tokens(test_tok, mode="test")
    model.sem_seg_head.predictor.set_class_tokens(train_tok, mode="train")
    model.arch = model.arch.replace(pad_len=int(gd["pad_len"]))
    model._engine = None
    im = torch.from_numpy(gd["image0"])
    model.eval()
    first = model([{"image": im}])[0]["sem_seg"].clone()
    assert first.shape[0] == len(test_tok)
    sem = torch.randint(0, len(train_tok), im.shape[-2:], generator=torch.Generator().manual_seed(3))
    model.train()
    loss = model([{"image": im, "sem_seg": sem}])["loss_sem_seg"].item()
    # the train-class logits from the training step's own fp32 engine
    eng = model.train_engine
    eng.set_text(eng.encode_text(torch.as_tensor(train_tok)))
    raw, sizes_dev, _ = model._batch(eng, [im])
    with torch.no_grad():
        train_logits = eng.head_logits(raw, sizes_dev).cpu()
    assert train_logits.shape[1] == len(train_tok)
    ref = reference_loss(train_logits, sem[None].int(), 255)
    assert abs(loss - ref) <= 1e-5 * abs(ref) + 1e-6, (loss, ref)
    model.eval()
    second = model([{"image": im}])[0]["sem_seg"]
    assert second.shape == first.shape and torch.equal(second, first)


def reference_grad(logits, targets, ignore, scale=1.0):
    """autograd of cat_seg_model.py:190-201 (interpolate -> BCE mean) in float64 on the CPU."""
    x = logits.double().clone().requires_grad_(True)
    out = F.interpolate(x, size=targets.shape[-2:], mode="bilinear", align_corners=False)
    T = out.shape[1]
    mask = targets != ignore
    out = out.permute(0, 2, 3, 1)
    tg = torch.zeros(out.shape, dtype=torch.float64)
    tg[mask] = F.one_hot(targets[mask].long(), num_classes=T).double()
    (F.binary_cross_entropy_with_logits(out, tg) * scale).backward()
    return x.grad


@pytest.mark.parametrize("B,T,h,w,H,W", [(2, 7, 24, 24, 96, 96), (3, 150, 24, 24, 50, 37), (1, 5, 96, 96, 384, 512),
                                         (2, 3, 17, 29, 17, 29), (1, 4, 40, 30, 20, 45)])
def test_bce_onehot_loss_backward_matches_autograd(B, T, h, w, H, W):
    """catseg_bce_onehot_loss_backward vs torch autograd of the reference loss (fp64): upsampling by
    4, ragged factors, identity size and a mixed down/up resize; deterministic (gather form)."""
    g = torch.Generator().manual_seed(B * 1000 + T + h)
    logits = torch.randn(B, T, h, w, generator=g) * 3
    targets = torch.randint(0, T, (B, H, W), generator=g, dtype=torch.int32)
    targets[torch.rand(B, H, W, generator=g) < 0.2] = 255
    ref = reference_grad(logits, targets, 255)
    got = ops.bce_onehot_loss_backward(logits.cuda(), targets.cuda(), 255).cpu().double()
    assert got.shape == ref.shape
    tol = 2e-5 * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= tol, ((got - ref).abs().max().item(), tol)
    again = ops.bce_onehot_loss_backward(logits.cuda(), targets.cuda(), 255).cpu().double()
    assert torch.equal(again, got)
    # the rows pass's LDS class chunk (knob bce_classes) does not change any sum's order
    from cat_seg import _lib as L
    try:
        for c in (1, 5, 32):
            L.tune("bce_classes", c)
            assert torch.equal(ops.bce_onehot_loss_backward(logits.cuda(), targets.cuda(), 255).cpu().double(), got)
    finally:
        L.tune("bce_classes", 0)


@pytest.mark.parametrize("case", ["all_ignored", "one_class", "one_pixel_logits", "wide_targets"])
def test_bce_onehot_loss_backward_edges(case):
    """edge cases of the gather ranges and the one-hot: every target pixel ignored (all-zero rows),
    T = 1, a 1 x 1 logit map (every target reads the same logit), targets wider than one LDS chunk
    row (W = 2100: the automatic class chunk drops to 3)."""
    g = torch.Generator().manual_seed(5)
    B, T, h, w, H, W = {"all_ignored": (2, 6, 12, 12, 48, 48), "one_class": (2, 1, 24, 24, 96, 96),
                        "one_pixel_logits": (1, 4, 1, 1, 9, 13), "wide_targets": (1, 5, 8, 300, 16, 2100)}[case]
    logits = torch.randn(B, T, h, w, generator=g) * 3
    targets = torch.randint(0, T, (B, H, W), generator=g, dtype=torch.int32)
    if case == "all_ignored":
        targets[:] = 255
    ref = reference_grad(logits, targets, 255)
    got = ops.bce_onehot_loss_backward(logits.cuda(), targets.cuda(), 255).cpu().double()
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
    loss = ops.bce_onehot_loss(logits.cuda(), targets.cuda(), 255).item()
    assert abs(loss - reference_loss(logits, targets, 255)) <= 1e-5 * abs(loss) + 1e-6


def test_bce_onehot_loss_autograd_function():
    """BCEOneHotLoss.apply(...).backward() on the device: loss equals bce_onehot_loss and
    logits.grad equals the fp64 autograd gradient of the reference loss times the upstream scale."""
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(2, 9, 24, 24, generator=g) * 2
    targets = torch.randint(0, 9, (2, 96, 96), generator=g, dtype=torch.int32)
    targets[:, :5] = 255
    x = logits.cuda().requires_grad_(True)
    loss = ops.BCEOneHotLoss.apply(x, targets.cuda(), 255)
    assert loss.requires_grad
    (loss * 3.0).backward()
    assert abs(loss.item() - reference_loss(logits, targets, 255)) <= 1e-5 * abs(loss.item()) + 1e-6
    ref = reference_grad(logits, targets, 255, scale=3.0)
    got = x.grad.cpu().double()
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
