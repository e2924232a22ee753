"""Time the training loss and its backward at the reference's training shape (cat_seg_model.py:189-203;
configs: 384^2 crops, COCO-Stuff's 171 training classes, logits 96^2, 4 images per GPU):
catseg_bce_onehot_loss, catseg_bce_onehot_loss_backward, and torch's own GPU autograd of the same
arithmetic (F.interpolate + one-hot BCE, fp32) beside them; checks the gradients agree.
usage: python tools/micro_bce.py [B] [bce_classes values for the backward's LDS chunk, e.g. 0,4,8,16]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
import torch.nn.functional as F
from cat_seg import ops
from cat_seg import _lib as L

L.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
T, h, w, H, W = 171, 96, 96, 384, 384
g = torch.Generator(device="cuda").manual_seed(0)
logits = torch.randn(B, T, h, w, device="cuda", generator=g) * 3
targets = torch.randint(0, T, (B, H, W), device="cuda", generator=g, dtype=torch.int32)
targets[torch.rand(B, H, W, device="cuda", generator=g) < 0.1] = 255


def torch_fwd_bwd():
    x = logits.clone().requires_grad_(True)
    out = F.interpolate(x, size=(H, W), mode="bilinear", align_corners=False).permute(0, 2, 3, 1)
    mask = targets != 255
    tg = torch.zeros(out.shape, device="cuda")
    tg[mask] = F.one_hot(targets[mask].long(), num_classes=T).float()
    F.binary_cross_entropy_with_logits(out, tg).backward()
    return x.grad


fns = {"loss": lambda: ops.bce_onehot_loss(logits, targets, 255),
       "loss_backward": lambda: ops.bce_onehot_loss_backward(logits, targets, 255),
       "torch_autograd_fwd_bwd": torch_fwd_bwd}
chunks = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else []
for c in chunks:
    fns[f"loss_backward_classes{c}"] = (lambda c=c: (L.tune("bce_classes", c),
                                                     ops.bce_onehot_loss_backward(logits, targets, 255))[1])
res = {}
for name, f in fns.items():
    f()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 5 * 1e3)
    res[name] = round(best, 1)
L.tune("bce_classes", 0)
ref = torch_fwd_bwd()
got = ops.bce_onehot_loss_backward(logits, targets, 255)
err = (got - ref).abs().max().item() / ref.abs().max().item()
alg = (logits.numel() * 4 * 2 + targets.numel() * 4)          # logits in, grad out, targets in
print(json.dumps({"B": B, "T": T, "logits": [h, w], "targets": [H, W], "us": res,
                  "backward_alg_GBps": round(alg / res["loss_backward"] / 1e3, 1),
                  "grad_rel_err_vs_torch": err}))
