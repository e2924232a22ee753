"""Pin the CPU oracle (oracle/catseg_oracle.py) to the golden vectors produced by the
reference's own modules (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import catseg_oracle as O
from cat_seg.arch import TINY, VIT_B16
from cat_seg.weights import synthesize_state_dict

from conftest import GOLDEN

CASES = {
    "e2e_tiny_pad": TINY,
    "e2e_tiny_topk_pool": TINY.replace(pooling_size=(2, 2)),
    "e2e_tiny_eval": TINY,
    "e2e_tiny_topk": TINY,
    "e2e_b16_voc20": VIT_B16.replace(pooling_size=(2, 2)),
    # ATTENTION_TYPE "full" (FullAttention, model.py:289-320)
    "e2e_tiny_full_pad": TINY.replace(attention_type="full", pooling_size=(2, 2)),
    "e2e_tiny_full_eval": TINY.replace(attention_type="full"),
    # visual prompt tuning (model_vpt.py:243-265): 3 prompts in each of the 4 vision blocks
    "e2e_tiny_vpt": TINY.replace(prompt_depth=4, prompt_length=3),
}


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_matches_reference_golden(name):
    if name == "e2e_b16_voc20" and os.environ.get("CATSEG_FAST_TESTS"):
        pytest.skip("fast mode")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = load(name)
    arch = CASES[name].replace(pad_len=int(g["pad_len"]))
    sd = synthesize_state_dict(arch, seed=0)
    tokens = torch.from_numpy(g["tokens"]).long()
    text = O.text_embeds(arch, sd, tokens)
    np.testing.assert_allclose(text.numpy(), g["text"], atol=2e-6, rtol=0)
    imgs = [torch.from_numpy(g[k]).float() for k in sorted(k for k in g if k.startswith("image"))]
    clip_images, sizes = O.preprocess(arch, imgs)
    logits = O.head_logits(arch, sd, clip_images, torch.from_numpy(g["text"]))
    sub = int(g["sub"])
    got = logits[:, :, ::sub, ::sub] if sub > 1 else logits
    np.testing.assert_allclose(got.numpy(), g["logits"], atol=2e-5, rtol=0)
    assert abs(logits.double().sum().item() - float(g["logits_sum"])) < 1e-2
    out = O.catseg_forward(arch, sd, [{"image": i} for i in imgs], torch.from_numpy(g["text"]))
    np.testing.assert_allclose(out[0]["sem_seg"][:, ::8, ::8].numpy(), g["sem_seg0_sub"], atol=1e-5, rtol=0)


def test_oracle_sliding_matches_reference_golden():
    """TEST.SLIDING_WINDOW branch (cat_seg_model.py:156-176,204-218): per-crop top-k, Fold/count,
    global average, non-default height/width."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = load("e2e_tiny_sliding")
    arch = TINY.replace(pad_len=int(g["pad_len"]))
    sd = synthesize_state_dict(arch, seed=0)
    text = O.text_embeds(arch, sd, torch.from_numpy(g["tokens"]).long())
    np.testing.assert_allclose(text.numpy(), g["text"], atol=2e-6, rtol=0)
    inp = [{"image": torch.from_numpy(g["image0"]), "height": int(g["height"]), "width": int(g["width"])}]
    out = O.catseg_forward_sliding(arch, sd, inp, torch.from_numpy(g["text"]))[0]["sem_seg"]
    sub = int(g["sub"])
    assert out.shape == (g["text"].shape[0], int(g["height"]), int(g["width"]))
    np.testing.assert_allclose(out[:, ::sub, ::sub].numpy(), g["sem_seg_sub"], atol=1e-5, rtol=0)
    assert abs(out.double().sum().item() - float(g["sem_seg_sum"])) < 1e-2


@pytest.mark.parametrize("name", ["e2e_l14_ade150", "e2e_l14_ade847"])
def test_oracle_matches_reference_golden_l14(name):
    """ViT-L/14@336 (the benchmarked geometry) with real class prompts: the oracle's logits, the
    top-k key (per-class max correlation) and, for ade847, the top-256 selection itself."""
    from cat_seg.arch import VIT_L14_336
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = load(name)
    arch = VIT_L14_336
    sd = synthesize_state_dict(arch, seed=0)
    text = torch.from_numpy(g["text"])
    if name == "e2e_l14_ade150":      # text encoder at L/14 width (the ade847 one is the same code)
        t = O.text_embeds(arch, sd, torch.from_numpy(g["tokens"]).long())
        np.testing.assert_allclose(t.numpy(), g["text"], atol=2e-6, rtol=0)
    imgs = [torch.from_numpy(g[k]).float() for k in sorted(k for k in g if k.startswith("image"))]
    clip_images, _ = O.preprocess(arch, imgs)
    with torch.no_grad():
        cmax = O.class_corr_max(arch, sd, clip_images, text)
        logits = O.head_logits(arch, sd, clip_images, text)
    np.testing.assert_allclose(cmax.numpy(), g["corr_max"], atol=2e-6, rtol=0)
    sub = int(g["sub"])
    np.testing.assert_allclose(logits[:, :, ::sub, ::sub].numpy(), g["logits"], atol=2e-5, rtol=0)
    assert abs(logits.double().sum().item() - float(g["logits_sum"])) < 2e-2
