"""The torch.library custom ops over the C ABI (cat_seg/custom_ops.py): opcheck (schema,
fake / meta kernel, autograd registration, AOT dispatch) on the device, a fullgraph torch.compile of a
chain of them, and the registered backward of catseg::linear against torch autograd."""
import pytest
import torch
import torch.nn.functional as F

from cat_seg import _lib as L
from cat_seg import custom_ops  # noqa: F401  (registers torch.ops.catseg.*)

pytestmark = pytest.mark.gpu
C = torch.ops.catseg


def _g(*s, seed=0, dt=torch.float32):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn(*s, generator=gen).to(dt).cuda()


def test_opcheck_gemm_layernorm_postprocess_attention():
    A, W = _g(300, 256, dt=torch.bfloat16), _g(128, 256, seed=1, dt=torch.bfloat16)
    torch.library.opcheck(C.gemm, (A, W, _g(128, seed=2), L.ACT_QUICKGELU, _g(300, 128, seed=3), 0))
    torch.library.opcheck(C.gemm, (A, W, None, L.ACT_NONE, None, 1))
    torch.library.opcheck(C.layernorm, (_g(77, 1024), 1 + _g(1024, seed=4) * 0.1, _g(1024, seed=5) * 0.1, 1e-5, 1))
    torch.library.opcheck(C.postprocess, (_g(2, 5, 96, 96), 336, 336, 96, 96))
    torch.library.opcheck(C.attention, (_g(2 * 77, 3 * 128), 2, 77, 2, True, 0, 0, 0, 0, 0))
    torch.library.opcheck(C.attention, (_g(2 * 576, 3 * 128), 2 * 4, 144, 4, False, 1, 24, 24, 12, 6))


def test_opcheck_class_attention():
    B, T, HW, D = 2, 20, 36, 128
    x = _g(B * T * HW, D, dt=torch.bfloat16)
    args = (x, 1 + _g(D, seed=1) * 0.1, _g(D, seed=2) * 0.1, _g(3 * D, D, seed=3, dt=torch.bfloat16) * 0.1,
            _g(3 * D, seed=4) * 0.1, _g(T, 2 * D, seed=5, dt=torch.bfloat16) * 0.1, B, T, HW, 256 - T,
            _g(D, seed=6), _g(D, seed=7))
    torch.library.opcheck(C.class_attention, args)


def test_linear_custom_op_backward_and_opcheck():
    x = _g(333, 128).requires_grad_(True)
    w = (_g(64, 128, seed=1) * 0.1).requires_grad_(True)
    b = _g(64, seed=2).requires_grad_(True)
    torch.library.opcheck(C.linear, (x, w, b, L.ACT_RELU))
    y = C.linear(x, w, b, L.ACT_RELU)
    dy = _g(333, 64, seed=3)
    y.backward(dy)
    xr, wr, br = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    F.relu(F.linear(xr, wr, br)).backward(dy.double())
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (got.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_compile_fullgraph_through_custom_ops():
    """A LayerNorm -> GEMM (+QuickGELU) -> GEMM (+residual) block written with the registered ops traces as
    one graph (fullgraph=True: no graph breaks) and matches the eager call."""
    x = _g(64, 256)
    g, bt = 1 + _g(256, seed=1) * 0.1, _g(256, seed=2) * 0.1
    w1, b1 = _g(512, 256, seed=3, dt=torch.bfloat16) * 0.05, _g(512, seed=4) * 0.1
    w2, b2 = _g(256, 512, seed=5, dt=torch.bfloat16) * 0.05, _g(256, seed=6) * 0.1

    def block(x):
        h = C.layernorm(x, g, bt, 1e-5, 1)
        u = C.gemm(h, w1, b1, L.ACT_QUICKGELU, None, 1)
        return C.gemm(u, w2, b2, L.ACT_NONE, x, 0)

    eager = block(x)
    compiled = torch.compile(block, fullgraph=True, backend="aot_eager")(x)
    assert torch.equal(compiled, eager)


def test_compile_catseg_forward_fullgraph():
    """torch.compile(CATSeg, fullgraph=True) traces the eval forward with no graph break: the canvas
    staging as torch ops, the network as catseg::head_logits, the resize as catseg::postprocess; the
    compiled forward returns the eager forward's probabilities bit for bit (same kernels)."""
    import os
    import numpy as np
    from cat_seg import build_model
    from conftest import ROOT
    from test_boundary_cpu import tiny_cfg
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "e2e_tiny_eval.npz")))
    model = build_model(tiny_cfg()).cuda().eval()
    model.sem_seg_head.predictor.set_class_tokens(g["tokens"])
    im = torch.from_numpy(g["image0"])
    inputs = [{"image": im, "height": 200, "width": 300}, {"image": im[:, :40, :48]}]
    eager = model(inputs)
    torch._dynamo.reset()
    compiled = torch.compile(model, fullgraph=True, backend="aot_eager")
    got = compiled(inputs)
    assert len(got) == len(eager) == 2
    for a, b in zip(eager, got):
        assert a["sem_seg"].shape == b["sem_seg"].shape
        assert torch.equal(a["sem_seg"], b["sem_seg"])
    # the traced graph holds the two registered operators, not the engine's ctypes calls
    from torch._dynamo.testing import CompileCounterWithBackend
    cnt = CompileCounterWithBackend("aot_eager")
    torch._dynamo.reset()
    torch.compile(model, fullgraph=True, backend=cnt)(inputs)
    assert cnt.frame_count == 1
