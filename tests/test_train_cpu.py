"""CPU tests of the training surface (no GPU calls): the training C ABI (include/catseg_hip_train.h)
is exported and bound, its host-side validation rejects bad arguments before any launch, and the
model's weights are real nn.Parameters in the reference's module tree, so the reference's
`Trainer.build_optimizer` (train_net.py:174-258) groups them as it would the reference model."""
import copy
import itertools
import os
import re

import torch

from cat_seg import build_model
from cat_seg import _lib as L
from cat_seg.params import apply_clip_finetune

from conftest import ROOT
from test_boundary_cpu import tiny_cfg


def test_train_header_symbols_are_exported_and_bound():
    hdr = open(os.path.join(ROOT, "include", "catseg_hip_train.h")).read()
    declared = set(re.findall(r"\b(catseg_[a-z0-9_]+)\s*\(", hdr))
    assert {"catseg_gemm_ex", "catseg_window_attention_backward", "catseg_linear_attention_backward",
            "catseg_conv2d_wgrad", "catseg_layernorm_backward", "catseg_groupnorm_relu_backward"} <= declared
    lib = L.load()
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared <= set(L.EXPORTED)


def test_train_entry_points_validate_on_the_host():
    lib = L.load()
    a = L.GemmExArgs()
    assert lib.catseg_gemm_ex(a, None) == -1                                   # null operands
    a.A = a.B = a.C = 16
    a.M, a.N, a.K = 8, 8, 8
    a.a_sm, a.a_sk, a.b_sk, a.b_sn = 3, 5, 7, 9                                 # no unit stride
    assert lib.catseg_gemm_ex(a, None) == -1
    assert "unit stride" in lib.catseg_last_error().decode()
    w = L.WinAttnBwdArgs()
    assert lib.catseg_window_attention_backward(w, None) == -1
    c = L.Conv2dArgs()
    assert lib.catseg_conv2d_nhwc(c, None) == -1
    la = L.LinAttnBwdArgs()
    assert lib.catseg_linear_attention_backward(la, None) == -1
    # workspace queries are pure host arithmetic
    assert lib.catseg_gemm_ex_workspace(384, 128, 400000) > 0
    assert lib.catseg_gemm_ex_workspace(400000, 128, 384) == 0
    assert lib.catseg_colsum_workspace(5000, 128) == 79 * 128 * 4            # 79 chunks of 64 rows


REF_NORM_TYPES = (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d, torch.nn.BatchNorm3d, torch.nn.SyncBatchNorm,
                  torch.nn.GroupNorm, torch.nn.InstanceNorm1d, torch.nn.InstanceNorm2d, torch.nn.InstanceNorm3d,
                  torch.nn.LayerNorm, torch.nn.LocalResponseNorm)


def build_optimizer_groups(model, base_lr=2e-4, wd=1e-4, wd_norm=0.0, wd_embed=0.0, clip_mult=0.01):
    """train_net.py:174-226 restated (the per-parameter hyper-parameter rules)."""
    groups, memo = [], set()
    for module_name, module in model.named_modules():
        for pname, value in module.named_parameters(recurse=False):
            if not value.requires_grad or value in memo:
                continue
            memo.add(value)
            hp = {"lr": base_lr, "weight_decay": wd}
            if "backbone" in module_name:
                hp["lr"] *= 0.01
            if "clip_model" in module_name:
                hp["lr"] *= clip_mult
            if "relative_position_bias_table" in pname or "absolute_pos_embed" in pname:
                hp["weight_decay"] = 0.0
            if isinstance(module, REF_NORM_TYPES):
                hp["weight_decay"] = wd_norm
            if isinstance(module, torch.nn.Embedding):
                hp["weight_decay"] = wd_embed
            groups.append({"name": f"{module_name}.{pname}", "params": [value], **hp})
    return groups


def test_parameters_are_a_reference_module_tree():
    m = build_model(tiny_cfg())
    names = dict(m.named_parameters())
    assert list(names) == list(m.state_dict())
    mods = dict(m.named_modules())
    agg = "sem_seg_head.predictor.transformer."
    assert isinstance(mods[agg + "layers.0.swin_block.block_1.norm1"], torch.nn.LayerNorm)
    assert isinstance(mods[agg + "layers.0.swin_block.guidance_norm"], torch.nn.LayerNorm)
    assert isinstance(mods[agg + "decoder1.conv.double_conv.1"], torch.nn.GroupNorm)
    assert mods[agg + "decoder1.conv.double_conv.1"].num_groups == 4
    assert isinstance(mods[agg + "decoder2.up"], torch.nn.ConvTranspose2d)
    assert isinstance(mods[agg + "conv1"], torch.nn.Conv2d) and isinstance(mods[agg + "head"], torch.nn.Conv2d)
    assert isinstance(mods[agg + "decoder_guidance_projection.1.0"], torch.nn.Conv2d)
    assert isinstance(mods[agg + "text_guidance_projection.0"], torch.nn.Linear)
    assert isinstance(mods[agg + "layers.1.attention.MLP.2"], torch.nn.Linear)
    assert isinstance(mods["upsample2"], torch.nn.ConvTranspose2d) and mods["upsample2"].stride == (4, 4)
    assert isinstance(mods["sem_seg_head.predictor.clip_model.token_embedding"], torch.nn.Embedding)
    assert isinstance(mods["sem_seg_head.predictor.clip_model.visual.ln_post"], torch.nn.LayerNorm)
    assert all(p.device.type == "cpu" for p in m.parameters())
    # the nn.Parameters are the weights: a checkpoint load writes into them
    sd = {k: v.clone() * 0 + 0.5 for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert torch.equal(names[agg + "head.bias"].detach(), torch.full((1,), 0.5))


def test_clip_finetune_requires_grad_like_the_reference():
    """cat_seg_model.py:57-75: 'attention' trains the q/v projections inside the CLIP transformers
    (and positional parameters there); everything else of CLIP is frozen; the head always trains."""
    m = build_model(tiny_cfg())
    tr = {n for n, p in m.named_parameters() if p.requires_grad}
    clip = [n for n, _ in m.named_parameters() if "clip_model" in n]
    assert {n for n in clip if n in tr} == {n for n in clip if "transformer" in n and
                                            ("q_proj" in n or "v_proj" in n)}
    assert all(n in tr for n, _ in m.named_parameters() if "clip_model" not in n)
    apply_clip_finetune(m.sem_seg_head.predictor.clip_model, "full")
    assert all(p.requires_grad for n, p in m.named_parameters() if "clip_model" in n and "transformer" in n)
    assert not m.sem_seg_head.predictor.clip_model.visual.proj.requires_grad
    apply_clip_finetune(m.sem_seg_head.predictor.clip_model, "none")
    assert not any(p.requires_grad for n, p in m.named_parameters() if "clip_model" in n)


def test_build_optimizer_groups_and_adamw_chunk_table():
    """cat_seg.optim.build_optimizer gives the same per-parameter groups as the restated reference rules;
    the fused AdamW's chunk table covers every element once (host code)."""
    from cat_seg.optim import AdamW, build_optimizer, chunk_table
    cfg = tiny_cfg(**{"SOLVER.CLIP_GRADIENTS.ENABLED": "True", "SOLVER.CLIP_GRADIENTS.CLIP_TYPE": "full_model",
                      "SOLVER.CLIP_GRADIENTS.CLIP_VALUE": "0.01", "SOLVER.BASE_LR": "0.0002"})
    m = build_model(cfg)
    opt = build_optimizer(cfg, m)
    assert isinstance(opt, AdamW) and opt.max_grad_norm == 0.01
    ref = build_optimizer_groups(m, base_lr=2e-4, wd=cfg.SOLVER.WEIGHT_DECAY, wd_norm=cfg.SOLVER.WEIGHT_DECAY_NORM,
                                 wd_embed=cfg.SOLVER.WEIGHT_DECAY_EMBED, clip_mult=cfg.SOLVER.CLIP_MULTIPLIER)
    assert len(opt.param_groups) == len(ref)
    for a, b in zip(opt.param_groups, ref):
        assert a["params"][0] is b["params"][0] and a["lr"] == b["lr"] and a["weight_decay"] == b["weight_decay"]
    t = chunk_table([4096, 1, 8193])
    assert t.tolist() == [0, 1 << 40, (2 << 40), (2 << 40) | 1, (2 << 40) | 2]


def test_reference_build_optimizer_rules_apply():
    m = build_model(tiny_cfg())
    groups = build_optimizer_groups(m)
    by = {g["name"]: g for g in groups}
    agg = "sem_seg_head.predictor.transformer."
    assert by[agg + "layers.0.swin_block.block_1.norm1.weight"]["weight_decay"] == 0.0
    assert by[agg + "decoder1.conv.double_conv.4.bias"]["weight_decay"] == 0.0
    assert by[agg + "layers.0.swin_block.block_1.attn.q.weight"]["weight_decay"] == 1e-4
    q = "sem_seg_head.predictor.clip_model.visual.transformer.resblocks.0.attn.q_proj_weight"
    assert by[q]["lr"] == 2e-4 * 0.01
    assert by["upsample1.weight"]["lr"] == 2e-4
    # torch's AdamW accepts the groups, with the reference's full-model gradient clipping wrapper
    opt = torch.optim.AdamW([{k: v for k, v in g.items() if k != "name"} for g in groups], 2e-4)
    for p in itertools.chain(*[g["params"] for g in opt.param_groups]):
        p.grad = torch.ones_like(p)
    torch.nn.utils.clip_grad_norm_(itertools.chain(*[g["params"] for g in opt.param_groups]), 0.01)
    before = copy.deepcopy(dict(m.named_parameters())[agg + "head.bias"].detach())
    opt.step()
    assert not torch.equal(dict(m.named_parameters())[agg + "head.bias"].detach(), before)


def test_sgd_full_model_clipping_and_position_table_decay():
    """SOLVER.OPTIMIZER SGD gets the reference's FullModelGradientClippingOptimizer too
    (train_net.py:228-256): its step equals clip_grad_norm_ over every parameter + torch SGD; and a
    parameter named relative_position_bias_table / absolute_pos_embed gets weight decay 0
    (train_net.py:216-221)."""
    from cat_seg.optim import FullModelClipSGD, build_optimizer
    cfg = tiny_cfg(**{"SOLVER.OPTIMIZER": "SGD", "SOLVER.CLIP_GRADIENTS.ENABLED": "True",
                      "SOLVER.CLIP_GRADIENTS.CLIP_TYPE": "full_model", "SOLVER.CLIP_GRADIENTS.CLIP_VALUE": "0.01"})
    m = build_model(cfg)
    m.sem_seg_head.predictor.transformer.register_parameter("absolute_pos_embed", torch.nn.Parameter(torch.ones(4)))
    opt = build_optimizer(cfg, m)
    assert isinstance(opt, FullModelClipSGD) and opt.max_grad_norm == 0.01
    pos = [g for g in opt.param_groups if g["params"][0].shape == (4,) and bool((g["params"][0] == 1).all())]
    assert len(pos) == 1 and pos[0]["weight_decay"] == 0.0
    m2 = copy.deepcopy(m)
    params = [p for g in opt.param_groups for p in g["params"]]
    torch.manual_seed(0)
    for p in params:
        p.grad = torch.randn_like(p)
    name_of = {id(p): n for n, p in m.named_parameters()}
    p2 = dict(m2.named_parameters())
    ref_params = [p2[name_of[id(p)]] for p in params]
    for p, q in zip(params, ref_params):
        q.grad = p.grad.clone()
    ref = torch.optim.SGD([{"params": [q], "lr": g["lr"], "weight_decay": g["weight_decay"]}
                           for q, g in zip(ref_params, opt.param_groups)], cfg.SOLVER.BASE_LR, momentum=cfg.SOLVER.MOMENTUM)
    torch.nn.utils.clip_grad_norm_(ref_params, 0.01)
    ref.step()
    opt.step()
    for p, q in zip(params, ref_params):
        assert torch.equal(p.detach(), q.detach())


def test_custom_ops_are_registered_with_meta_kernels():
    """torch.ops.catseg.* exist and their fake kernels give the output shape / dtype on meta tensors
    (no GPU: the dispatcher routes meta inputs to the registered fake implementation)."""
    from cat_seg import custom_ops  # noqa: F401
    C = torch.ops.catseg
    A = torch.empty(300, 256, device="meta", dtype=torch.bfloat16)
    W = torch.empty(128, 256, device="meta", dtype=torch.bfloat16)
    out = C.gemm(A, W, None, 0, None, 0)
    assert out.shape == (300, 128) and out.dtype == torch.float32 and out.device.type == "meta"
    ln = C.layernorm(torch.empty(7, 64, device="meta"), torch.empty(64, device="meta"),
                     torch.empty(64, device="meta"), 1e-5, 1)
    assert ln.dtype == torch.bfloat16 and ln.shape == (7, 64)
    pp = C.postprocess(torch.empty(2, 5, 96, 96, device="meta"), 336, 300, 96, 96)
    assert pp.shape == (2, 5, 336, 300)
    att = C.attention(torch.empty(154, 384, device="meta"), 2, 77, 2, True, 0, 0, 0, 0, 0)
    assert att.shape == (154, 128)
    mm = C.mm(torch.empty(10, 20, device="meta"), torch.empty(10, 30, device="meta"), True, False)
    assert mm.shape == (20, 30)
