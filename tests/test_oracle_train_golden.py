"""The oracle's training graph against the REFERENCE's own modules (CPU, no GPU).

tests/golden/train_tiny_pool2.npz holds the loss and the gradients of every trainable parameter of
the reference's model_vpt.CLIP + Aggregator training step in float64 (tests/golden/make_golden.py
"train": TINY geometry, POOLING [2,2], T=9 < pad_len, CLIP_FINETUNE "attention").  Here the same step
runs through oracle/catseg_oracle.py under float64 torch autograd -- the graph the GPU gradient tests
(tests/test_gpu_train_*.py) use as their reference -- and must reproduce the reference modules'
gradients to float64 rounding, so the GPU tests' oracle is pinned for the backward as
tests/test_oracle_golden.py pins it for the forward.
"""
import os

import numpy as np
import torch

from cat_seg.arch import TINY
from cat_seg.weights import synthesize_state_dict
from oracle import catseg_oracle as O

from conftest import ROOT
from test_gpu_train_head import ref_head, ref_loss


def test_oracle_training_gradients_match_reference_modules():
    g = np.load(os.path.join(ROOT, "tests", "golden", "train_tiny_pool2.npz"))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    arch = TINY.replace(pooling_size=(2, 2))
    names = [str(k) for k in g["names"]]
    sd = {k: v.double() for k, v in synthesize_state_dict(arch, seed=0).items()}
    for k in names:
        sd[k].requires_grad_(True)
    ims = [torch.from_numpy(g["image0"]).float(), torch.from_numpy(g["image1"]).float()]
    clip_ims, _ = O.preprocess(arch, ims)
    feats, hooks = O.encode_image_dense(arch, sd, clip_ims.double())
    text = O.text_embeds(arch, sd, torch.from_numpy(g["tokens"]))[:, 0]
    loss = ref_loss(ref_head(arch, sd, feats, hooks, text), torch.from_numpy(g["targets"]).long())
    loss.backward()
    l64 = float(g["loss64"])
    assert abs(loss.item() - l64) <= 1e-10 * abs(l64), (loss.item(), l64)
    worst = (0.0, "")
    for k in names:
        mx = float(g["m_" + k][0])
        if sd[k].grad is None:        # off the oracle's graph (the dense block's dead q / k): zero there
            assert mx == 0.0, k
            continue
        got = sd[k].grad.detach().reshape(-1)
        if mx == 0.0:
            assert got.abs().max().item() == 0.0, k
            continue
        idx = torch.from_numpy(g["i_" + k])
        err = (got[idx] - torch.from_numpy(g["g_" + k])).abs().max().item() / mx
        if ".swin_block." in k and k.endswith("attn.k.bias"):
            # zero in exact arithmetic: compare against the k weight's gradient scale
            err = (got[idx] - torch.from_numpy(g["g_" + k])).abs().max().item() / float(
                g["m_" + k[:-len("bias")] + "weight"][0])
        worst = max(worst, (err, k))
    assert worst[0] <= 1e-9, worst
