"""Generate the golden vectors under tests/golden/ from the REFERENCE's own modules.

Run in the build container only (the reference tree is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it imports from /root/reference (read-only, by file path):
  * cat_seg/third_party/model_vpt.py       -> CLIP (visual dense encoder + text encoder)
  * cat_seg/modeling/transformer/model.py  -> Aggregator (needs `timm.layers`, absent here:
    a stub module provides Mlp/DropPath/to_2tuple with timm 0.8 eval semantics —
    fc1 -> act -> fc2, DropPath identity at eval)
  * cat_seg/third_party/simple_tokenizer.py + clip.tokenize semantics (needs `ftfy`, absent:
    stubbed as identity; exact for the ASCII class lists)
The detectron2 glue (ImageList pad, sem_seg_postprocess, CATSeg.forward eval branches,
cat_seg_model.py:147-229) cannot be imported (detectron2 is not installed) and is
restated inline below, independently of oracle/catseg_oracle.py.

Weights come from the build's deterministic synthesizer (cat_seg.weights), loaded into
the reference modules with strict=True so every key name is checked.
Outputs: small .npz fixtures (inputs + expected outputs).
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "cat-seg_amd"))

from cat_seg.arch import TINY, VIT_B16  # noqa: E402
from cat_seg.weights import synthesize_state_dict, CLIP as CLIP_P, AGG as AGG_P  # noqa: E402


def _stub_timm():
    class Mlp(nn.Module):
        def __init__(self, in_features, hidden_features=None, out_features=None,
                     act_layer=nn.GELU, drop=0.0, **_):
            super().__init__()
            out_features = out_features or in_features
            hidden_features = hidden_features or in_features
            self.fc1 = nn.Linear(in_features, hidden_features)
            self.act = act_layer()
            self.fc2 = nn.Linear(hidden_features, out_features)

        def forward(self, x):
            return self.fc2(self.act(self.fc1(x)))

    class DropPath(nn.Module):
        def __init__(self, p=0.0):
            super().__init__()

        def forward(self, x):
            return x

    layers = types.ModuleType("timm.layers")
    layers.Mlp = Mlp
    layers.DropPath = DropPath
    layers.to_2tuple = lambda x: tuple(x) if isinstance(x, (tuple, list)) else (x, x)
    layers.to_ntuple = lambda n: (lambda x: tuple([x] * n))
    layers.trunc_normal_ = lambda t, **k: t
    layers.PatchEmbed = None
    layers._assert = lambda c, m="": None
    timm = types.ModuleType("timm")
    timm.layers = layers
    sys.modules["timm"] = timm
    sys.modules["timm.layers"] = layers
    ftfy = types.ModuleType("ftfy")
    ftfy.fix_text = lambda s: s
    sys.modules["ftfy"] = ftfy


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_stub_timm()
model_vpt = _load("ref_model_vpt", f"{REF}/cat_seg/third_party/model_vpt.py")
agg_mod = _load("ref_agg_model", f"{REF}/cat_seg/modeling/transformer/model.py")
tok_mod = _load("ref_simple_tokenizer", f"{REF}/cat_seg/third_party/simple_tokenizer.py")


# ---------------------------------------------------------------- tokens
def tokenize(tok, texts, context_length=77):
    # clip.tokenize semantics (cat_seg/third_party/clip.py:200-214)
    sot, eot = tok.encoder["<|startoftext|>"], tok.encoder["<|endoftext|>"]
    out = np.zeros((len(texts), context_length), dtype=np.int64)
    for i, t in enumerate(texts):
        ids = [sot] + tok.encode(t) + [eot]
        assert len(ids) <= context_length
        out[i, : len(ids)] = ids
    return out


def class_prompts(names):
    # cat_seg_predictor.py:196-201: first alias before ", ", single template (:84-85)
    return ["A photo of a {} in the scene".format(n.split(", ")[0] if ", " in n else n) for n in names]


# ---------------------------------------------------------------- reference model build
def build_reference(arch, sd, pad_len=256):
    clip = model_vpt.CLIP(
        arch.embed_dim, arch.vision_pretrain_res, arch.vision_layers, arch.vision_width,
        arch.vision_patch, arch.context_length, arch.vocab_size, arch.text_width,
        arch.text_heads, arch.text_layers, prompt_depth=arch.prompt_depth, prompt_length=arch.prompt_length)
    clip_sd = {k[len(CLIP_P):]: v for k, v in sd.items() if k.startswith(CLIP_P)}
    clip.load_state_dict(clip_sd, strict=True)
    agg = agg_mod.Aggregator(
        text_guidance_dim=arch.embed_dim, text_guidance_proj_dim=arch.text_guidance_proj_dim,
        appearance_guidance_dim=arch.embed_dim,
        appearance_guidance_proj_dim=arch.appearance_guidance_proj_dim,
        decoder_dims=list(arch.decoder_dims), decoder_guidance_dims=list(arch.decoder_guidance_dims),
        decoder_guidance_proj_dims=list(arch.decoder_guidance_proj_dims),
        num_layers=arch.num_layers, nheads=arch.nheads, hidden_dim=arch.hidden_dim,
        pooling_size=list(arch.pooling_size), feature_resolution=list(arch.feature_resolution),
        window_size=arch.window_size, attention_type=arch.attention_type, prompt_channel=1, pad_len=pad_len)
    agg_sd = {k[len(AGG_P):]: v for k, v in sd.items() if k.startswith(AGG_P)}
    missing, unexpected = agg.load_state_dict(agg_sd, strict=False)
    # the only non-parameter entries are the SW-MSA mask buffers (model.py:183)
    assert all(k.endswith("attn_mask") for k in missing), missing
    assert not unexpected, unexpected
    up1 = nn.ConvTranspose2d(arch.vision_width, arch.decoder_guidance_dims[0], 2, 2)
    up2 = nn.ConvTranspose2d(arch.vision_width, arch.decoder_guidance_dims[1], 4, 4)
    up1.load_state_dict({"weight": sd["upsample1.weight"], "bias": sd["upsample1.bias"]})
    up2.load_state_dict({"weight": sd["upsample2.weight"], "bias": sd["upsample2.bias"]})
    for m in (clip, agg, up1, up2):
        m.eval()
    return clip.float(), agg, up1, up2


def ref_text(clip, tokens):
    # cat_seg_predictor.py:214-219
    with torch.no_grad():
        e = clip.encode_text(torch.from_numpy(tokens))
        e = e / e.norm(dim=-1, keepdim=True)
    return e.unsqueeze(1)


def ref_head(arch, clip, agg, up1, up2, clip_images, text):
    """cat_seg_model.py:155,178-188 with the reference CLIP/Aggregator modules."""
    layers = []
    hs = [clip.visual.transformer.resblocks[l].register_forward_hook(lambda m, i, o: layers.append(o))
          for l in arch.hook_layers]
    with torch.no_grad():
        feats = clip.encode_image(clip_images, dense=True)
        g = arch.grid
        img = feats[:, 1:, :]
        B = img.shape[0]
        res3 = img.reshape(B, g, g, -1).permute(0, 3, 1, 2)
        res4 = layers[0][1:].permute(1, 2, 0).reshape(B, -1, g, g)
        res5 = layers[1][1:].permute(1, 2, 0).reshape(B, -1, g, g)
        vis = [res3, up1(res4), up2(res5)]
        out = agg(res3, text.repeat(B, 1, 1, 1), vis)
    for h in hs:
        h.remove()
    return out


def glue_preprocess(arch, images):
    """cat_seg_model.py:149-154 + detectron2 ImageList.from_tensors (pad /32, value 0)."""
    mean = torch.tensor(arch.clip_pixel_mean).view(-1, 1, 1)
    std = torch.tensor(arch.clip_pixel_std).view(-1, 1, 1)
    norm = [(im - mean) / std for im in images]
    H = max(x.shape[1] for x in norm)
    W = max(x.shape[2] for x in norm)
    d = arch.size_divisibility
    H, W = -(-H // d) * d, -(-W // d) * d
    pad = torch.zeros(len(norm), 3, H, W)
    for i, x in enumerate(norm):
        pad[i, :, : x.shape[1], : x.shape[2]] = x
    R = arch.clip_resolution
    return F.interpolate(pad, size=(R, R), mode="bilinear", align_corners=False)


def glue_post(logits0, size, h, w):
    """sigmoid + detectron2 sem_seg_postprocess (cat_seg_model.py:222-227)."""
    r = logits0.sigmoid()[:, : size[0], : size[1]].unsqueeze(0)
    return F.interpolate(r, size=(h, w), mode="bilinear", align_corners=False)[0]


def rand_images(seed, shapes):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, 256, (3, h, w), generator=g, dtype=torch.uint8) for h, w in shapes]


def rand_tokens(seed, T, ctx, vocab):
    g = np.random.default_rng(seed)
    toks = np.zeros((T, ctx), dtype=np.int64)
    for t in range(T):
        n = int(g.integers(3, ctx - 1))
        toks[t, 0] = vocab - 2
        toks[t, 1:n] = g.integers(1, vocab - 2, n - 1)
        toks[t, n] = vocab - 1                           # EOT = highest id (argmax)
    return toks


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


def e2e_case(name, arch, T, shapes, seed, pad_len=256, tokens=None, sub=1):
    sd = synthesize_state_dict(arch, seed=0)
    clip, agg, up1, up2 = build_reference(arch, sd, pad_len=pad_len)
    if tokens is None:
        tokens = rand_tokens(seed, T, arch.context_length, arch.vocab_size)
    text = ref_text(clip, tokens)
    imgs = rand_images(seed, shapes)
    clip_images = glue_preprocess(arch, [i.float() for i in imgs])
    logits = ref_head(arch, clip, agg, up1, up2, clip_images, text)
    out0 = glue_post(logits[0], shapes[0], shapes[0][0], shapes[0][1])
    kw = dict(tokens=tokens, text=text, logits=logits[:, :, ::sub, ::sub] if sub > 1 else logits,
              logits_sum=logits.double().sum(), logits_abs_sum=logits.double().abs().sum(),
              sem_seg0_sub=out0[:, ::8, ::8], sem_seg0_sum=out0.double().sum(),
              pad_len=pad_len, sub=sub)
    for i, im in enumerate(imgs):
        kw[f"image{i}"] = im
    save(name, **kw)


def glue_sliding(arch, clip, agg, up1, up2, image, text, height, width):
    """TEST.SLIDING_WINDOW eval branch (cat_seg_model.py:156-176,204-218), restated with the
    same torch ops (nn.Unfold / nn.Fold, bilinear align_corners=False) around ref_head."""
    kernel, overlap, out_res = 384, 0.333, [640, 640]
    stride = int(kernel * (1 - overlap))
    unfold = nn.Unfold(kernel_size=kernel, stride=stride)
    fold = nn.Fold(out_res, kernel_size=kernel, stride=stride)
    img = image.float()
    x = F.interpolate(img.unsqueeze(0), size=out_res, mode="bilinear", align_corners=False).squeeze()
    L = unfold(x).shape[-1]
    x = unfold(x).reshape(3, kernel, kernel, L).permute(3, 0, 1, 2)          # "(C H W) L -> L C H W"
    g = F.interpolate(img.unsqueeze(0), size=(kernel, kernel), mode="bilinear", align_corners=False)
    x = torch.cat((x, g), dim=0)
    mean = torch.tensor(arch.clip_pixel_mean).view(-1, 1, 1)
    std = torch.tensor(arch.clip_pixel_std).view(-1, 1, 1)
    R = arch.clip_resolution
    clip_images = F.interpolate((x - mean) / std, size=(R, R), mode="bilinear", align_corners=False)
    out = ref_head(arch, clip, agg, up1, up2, clip_images, text)
    out = F.interpolate(out, size=kernel, mode="bilinear", align_corners=False).sigmoid()
    glob = F.interpolate(out[-1:], size=out_res, mode="bilinear", align_corners=False)
    out = out[:-1]
    out = fold(out.flatten(1).T) / fold(unfold(torch.ones([1] + out_res)))
    out = (out + glob) / 2.0
    r = out[0][:, : out_res[0], : out_res[1]].unsqueeze(0)                 # sem_seg_postprocess
    return F.interpolate(r, size=(height, width), mode="bilinear", align_corners=False)[0]


def sliding_case(name, arch, T, shape, seed, pad_len, height, width, sub=4):
    sd = synthesize_state_dict(arch, seed=0)
    clip, agg, up1, up2 = build_reference(arch, sd, pad_len=pad_len)
    tokens = rand_tokens(seed, T, arch.context_length, arch.vocab_size)
    text = ref_text(clip, tokens)
    img = rand_images(seed, [shape])[0]
    with torch.no_grad():
        out = glue_sliding(arch, clip, agg, up1, up2, img, text, height, width)
    save(name, tokens=tokens, text=text, image0=img, height=height, width=width, pad_len=pad_len, sub=sub,
         sem_seg_sub=out[:, ::sub, ::sub], sem_seg_sum=out.double().sum())


def ref_corr_max(arch, clip, agg, clip_images, text):
    """Per-image, per-class max of the fp32 cost volume over (P, H, W) — the top-k key of
    model.py:694-697 — from the reference CLIP + Aggregator.correlation (model.py:648-652)."""
    with torch.no_grad():
        feats = clip.encode_image(clip_images, dense=True)
        g = arch.grid
        B = feats.shape[0]
        img = feats[:, 1:, :].reshape(B, g, g, -1).permute(0, 3, 1, 2)
        corr = agg.correlation(img, text.repeat(B, 1, 1, 1))          # (B, P, T, H, W)
        return corr.permute(0, 2, 1, 3, 4).flatten(2).max(dim=-1)[0]   # (B, T)


def l14_case(name, T_name, shapes, seed, sub=4):
    """ViT-L/14@336 (the benchmarked geometry: patch 14, K=588 im2col, hooks 7/15, no pos-embed
    resize, 1024-wide ViT) with the real class prompts of `T_name`."""
    from cat_seg.arch import VIT_L14_336
    arch = VIT_L14_336
    sd = synthesize_state_dict(arch, seed=0)
    clip, agg, up1, up2 = build_reference(arch, sd)
    tokens = np.load(os.path.join(HERE, "class_tokens.npz"))[T_name].astype(np.int64)
    text = ref_text(clip, tokens)
    imgs = rand_images(seed, shapes)
    clip_images = glue_preprocess(arch, [i.float() for i in imgs])
    logits = ref_head(arch, clip, agg, up1, up2, clip_images, text)
    cmax = ref_corr_max(arch, clip, agg, clip_images, text)
    out0 = glue_post(logits[0], shapes[0], shapes[0][0], shapes[0][1])
    kw = dict(tokens=tokens.astype(np.int32), text=text, logits=logits[:, :, ::sub, ::sub], corr_max=cmax,
              logits_sum=logits.double().sum(), logits_abs_sum=logits.double().abs().sum(),
              sem_seg0_sub=out0[:, ::8, ::8], pad_len=256, sub=sub)
    for i, im in enumerate(imgs):
        kw[f"image{i}"] = im
    save(name, **kw)


CLASS_LISTS = ("voc20", "voc20b", "pc59", "pc459", "ade150", "ade847", "coco")


def class_data():
    """Class-name token ids of the reference's class lists (datasets/*.json), made with the
    reference tokenizer: the golden fixture, plus the package data the predictor reads
    (cat_seg/data: class_tokens.npz, class_lists.json = sha1 of the names -> list key,
    class_names.json = the names, for dataset metadata)."""
    import hashlib
    tok = tok_mod.SimpleTokenizer()
    toks, names_all, table = {}, {}, {}
    for ds in CLASS_LISTS:
        names = json.load(open(f"{REF}/datasets/{ds}.json"))
        toks[ds] = tokenize(tok, class_prompts(names)).astype(np.int32)
        names_all[ds] = names
        table[hashlib.sha1("\n".join(names).encode()).hexdigest()] = ds
    save("class_tokens", **toks)
    pkg = os.path.join(ROOT, "cat-seg_amd", "cat_seg", "data")
    np.savez_compressed(os.path.join(pkg, "class_tokens.npz"), **toks)
    with open(os.path.join(pkg, "class_lists.json"), "w") as f:
        json.dump(table, f, indent=0)
    with open(os.path.join(pkg, "class_names.json"), "w") as f:
        json.dump(names_all, f)
    return toks


def train_case(name, arch, T, seed=3, n_sub=256):
    """The training step (cat_seg_model.py:57-75 requires_grad for CLIP_FINETUNE 'attention', :136-146 +
    :178-203 forward and one-hot BCE loss, cat_seg_predictor.py:150-160,190-224 text embeddings with
    grad) through the reference's own modules in float64, backward, and the gradient of every trainable
    parameter.  A gradient is stored as an evenly strided sample of at most n_sub entries of the
    flattened tensor (the build's parameters have the reference's shapes) plus max |g|, with the
    relative error of the same reference graph run in float32 (the gate's scale); inputs are the GPU
    test's (tests/test_gpu_train_head.py::test_catseg_train_step_matches_reference_gradients)."""
    sd = synthesize_state_dict(arch, seed=0)
    gen = torch.Generator().manual_seed(seed)
    toks = torch.zeros(T, arch.context_length, dtype=torch.long)
    toks[:, 0] = 1
    toks[:, 1:4] = torch.randint(2, 400, (T, 3), generator=gen)
    toks[:, 4] = 511                                   # EOT = the argmax id
    ims = [torch.randint(0, 256, (3, 384, 384), generator=gen).float() for _ in range(2)]
    sems = [torch.randint(0, T, (384, 384), generator=gen) for _ in range(2)]
    sems[0][:20] = 255
    targets = torch.stack(sems)
    grads, losses = {}, {}
    # model_vpt.py:156-162's LayerNorm casts its input to float32 (an fp16 guard): the identity for the
    # float32 run; for the float64 run it is bypassed so the graph stays float64 end to end
    ln_forward = model_vpt.LayerNorm.forward
    for dt in (torch.float64, torch.float32):
        model_vpt.LayerNorm.forward = nn.LayerNorm.forward if dt == torch.float64 else ln_forward
        clip, agg, up1, up2 = build_reference(arch, sd, pad_len=arch.pad_len)
        clip, agg, up1, up2 = clip.to(dt), agg.to(dt), up1.to(dt), up2.to(dt)
        for n, p in clip.named_parameters():         # cat_seg_model.py:57-75, CLIP_FINETUNE "attention"
            rg = False
            if "transformer" in n:
                rg = ("q_proj" in n or "v_proj" in n) if "attn" in n else ("position" in n)
            p.requires_grad_(rg)
        for m in (clip, agg, up1, up2):
            m.train()
        text = clip.encode_text(toks)
        text = (text / text.norm(dim=-1, keepdim=True)).unsqueeze(1)
        layers = []
        hs = [clip.visual.transformer.resblocks[l].register_forward_hook(lambda m, i, o: layers.append(o))
              for l in arch.hook_layers]
        clip_images = glue_preprocess(arch, ims).to(dt)
        feats = clip.encode_image(clip_images, dense=True)
        for h in hs:
            h.remove()
        g = arch.grid
        B = feats.shape[0]
        res3 = feats[:, 1:, :].reshape(B, g, g, -1).permute(0, 3, 1, 2)
        res4 = up1(layers[0][1:].permute(1, 2, 0).reshape(B, -1, g, g))
        res5 = up2(layers[1][1:].permute(1, 2, 0).reshape(B, -1, g, g))
        out = agg(res3, text.repeat(B, 1, 1, 1), [res3, res4, res5])
        out = F.interpolate(out, size=targets.shape[-2:], mode="bilinear", align_corners=False)
        mask = targets != 255
        out = out.permute(0, 2, 3, 1)
        tg = torch.zeros(out.shape, dtype=dt)
        tg[mask] = F.one_hot(targets[mask], num_classes=out.shape[-1]).to(dt)
        loss = F.binary_cross_entropy_with_logits(out, tg)
        loss.backward()
        losses[dt] = loss.item()
        named = {CLIP_P + n: p for n, p in clip.named_parameters()}
        named.update({AGG_P + n: p for n, p in agg.named_parameters()})
        named.update({"upsample1." + n: p for n, p in up1.named_parameters()})
        named.update({"upsample2." + n: p for n, p in up2.named_parameters()})
        grads[dt] = {k: (None if p.grad is None else p.grad.detach().double().reshape(-1))
                     for k, p in named.items() if p.requires_grad}
    model_vpt.LayerNorm.forward = ln_forward
    kw = dict(tokens=toks, targets=targets.to(torch.int16), loss64=losses[torch.float64],
              loss32=losses[torch.float32], image0=ims[0].to(torch.uint8), image1=ims[1].to(torch.uint8))
    names, none = [], []
    for k, g64 in grads[torch.float64].items():
        if g64 is None:
            none.append(k)
            continue
        n = g64.numel()
        step = max(1, n // n_sub)
        idx = torch.arange(0, n, step)[:n_sub]
        g32 = grads[torch.float32][k]
        mx = g64.abs().max().item()
        names.append(k)
        kw["g_" + k] = g64[idx].numpy()
        kw["i_" + k] = idx.numpy().astype(np.int64)
        kw["m_" + k] = np.array([mx, (g32 - g64).abs().max().item() / (mx + 1e-300)])
    kw["names"] = np.array(names)
    kw["none"] = np.array(none)
    save(name, **kw)


def prompt_ensemble_probe():
    """PROMPT_ENSEMBLE_TYPE "imagenet" / "imagenet_select" (cat_seg_predictor.py:80-83): the eval text
    path stacks each class's P template token rows to (T, P, 77) (:196-208; squeeze(1) only drops
    P = 1) and hands that to CLIP.encode_text (:214), whose NLD -> LND permute (model_vpt.py:428) is
    3-d.  Runs the reference's own encode_text on such a tensor and records what it raises."""
    import json
    arch = TINY
    sd = synthesize_state_dict(arch, seed=0)
    clip, _, _, _ = build_reference(arch, sd)
    T, P = 3, 80                                      # IMAGENET_TEMPLATES has 80 templates
    toks = np.stack([rand_tokens(9 + t, P, arch.context_length, arch.vocab_size) for t in range(T)])
    tokens = torch.from_numpy(toks).squeeze(1)        # cat_seg_predictor.py:208
    rec = {"tokens_shape": list(tokens.shape), "raised": None, "error": None}
    try:
        with torch.no_grad():
            out = clip.encode_text(tokens)
        rec["output_shape"] = list(out.shape)
    except Exception as e:  # noqa: BLE001 - the failure is the result
        rec["raised"], rec["error"] = type(e).__name__, str(e)
    path = os.path.join(HERE, "prompt_ensemble_probe.json")
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
    print("wrote", path, rec)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "train":
        torch.set_num_threads(8)
        # the training step at TINY geometry, the training config's POOLING [2,2], T=9 < pad_len (padding
        # tokens train), CLIP q / v of both encoders
        train_case("train_tiny_pool2", TINY.replace(pooling_size=(2, 2)), 9)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "classes":
        class_data()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "l14":
        torch.set_num_threads(8)
        # config 3 geometry, real ade150 prompts, two images (one ragged: ImageList pad 352 -> 336)
        l14_case("e2e_l14_ade150", "ade150", [(336, 336), (300, 336)], seed=21)
        # config 4 class count: ade847 prompts -> top-256 + -100 scatter, one image
        l14_case("e2e_l14_ade847", "ade847", [(336, 336)], seed=22, sub=6)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "ensemble":
        prompt_ensemble_probe()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "vpt":
        torch.set_num_threads(8)
        # visual prompt tuning (model_vpt.py:243-265): 3 prompt tokens in every one of TINY's 4 vision
        # blocks (PROMPT_DEPTH = the layer count), T=10 < pad_len=16, two ragged images
        vpt = TINY.replace(prompt_depth=4, prompt_length=3)
        e2e_case("e2e_tiny_vpt", vpt, 10, [(300, 352), (320, 256)], seed=9, pad_len=16)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "full":
        torch.set_num_threads(8)
        # ATTENTION_TYPE "full" (FullAttention, model.py:289-320): T=10 < pad_len=16 with pooling
        # (2,2) (pad keys + pooled class attention), and T=20 with the eval pooling (1,1) padded to
        # the default pad_len 256, B=2
        full = TINY.replace(attention_type="full")
        e2e_case("e2e_tiny_full_pad", full.replace(pooling_size=(2, 2)), 10, [(300, 352)], seed=7, pad_len=16)
        e2e_case("e2e_tiny_full_eval", full, 20, [(384, 384), (352, 384)], seed=8)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sliding":
        torch.set_num_threads(8)
        # TEST.SLIDING_WINDOW: tiny arch, T=20 > pad_len=16 (per-crop top-k), ragged 440x360 image,
        # output resized to 480x400 (non-default height/width)
        sliding_case("e2e_tiny_sliding", TINY, 20, (440, 360), seed=6, pad_len=16, height=480, width=400)
        return
    torch.manual_seed(0)
    torch.set_num_threads(8)
    toks = class_data()
    # 1) tiny arch, T=10 < pad_len=16 (learned padding path), two ragged images (ImageList pad)
    e2e_case("e2e_tiny_pad", TINY, 10, [(300, 352), (320, 256)], seed=1, pad_len=16)
    # 2) tiny arch, T=24 > pad_len=16 (top-k + scatter -100), pooling (2,2)
    e2e_case("e2e_tiny_topk_pool", TINY.replace(pooling_size=(2, 2)), 24, [(384, 384)], seed=2, pad_len=16)
    # 2b) tiny arch, T=24 > pad_len=16 (top-k + scatter -100), eval pooling (1,1), B=2
    e2e_case("e2e_tiny_topk", TINY, 24, [(384, 384), (352, 384)], seed=5, pad_len=16)
    # 3) tiny arch, default pad_len 256, T=20, pooling (1,1) (the eval protocol), B=2
    e2e_case("e2e_tiny_eval", TINY, 20, [(384, 384), (384, 384)], seed=3)
    # 4) config 1: ViT-B/16@384 (pos-embed bicubic resize), voc20 tokens, bs=1, POOLING (2,2)
    e2e_case("e2e_b16_voc20", VIT_B16.replace(pooling_size=(2, 2)), 20, [(384, 384)], seed=4,
             tokens=toks["voc20"].astype(np.int64), sub=2)


if __name__ == "__main__":
    main()
