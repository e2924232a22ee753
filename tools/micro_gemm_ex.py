"""Time the training GEMMs (catseg_gemm_ex, fp32 MFMA) and the forward fp32 GEMM on the shapes of the
training step (B/16@384: R = 4 x 171 x 576 rows of 128 channels) and check them against torch.

usage: python tools/micro_gemm_ex.py [terms, default "0"]   (tuning knob gemm_ex_terms: 0 = exact-f32
MFMA, 6 / 3 = split-bf16 MFMA; each gemm_ex line is repeated per value)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch  # noqa: E402

from cat_seg import ops  # noqa: E402
from cat_seg import train_ops as TO  # noqa: E402
from cat_seg import _lib as L  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
R = int(os.environ.get("MGX_R", 4 * 171 * 576))
TERMS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0").split(",")]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(ts)[2]


def report(name, M, N, K, t, err):
    print(f"{name:34s} M={M:7d} N={N:5d} K={K:7d}: {t:8.1f} us {2 * M * N * K / t / 1e6:7.1f} TF/s  "
          f"rel err {err:.2e}", flush=True)


def rel(a, b):
    return ((a.double() - b).abs().max() / b.abs().max()).item()


for Kin, Nout in ((128, 512), (512, 128), (128, 128), (128, 384)):
    X = torch.randn(R, Kin, device=dev)
    W = torch.randn(Nout, Kin, device=dev) / Kin ** 0.5
    dY = torch.randn(R, Nout, device=dev)
    # forward: Y = X . W^T (catseg_gemm fp32)
    Y = torch.empty(R, Nout, device=dev)
    t = timeit(lambda: ops.gemm(X, W, Y))
    report(f"fwd  X.W^T   ({Kin}->{Nout})", R, Nout, Kin, t, rel(Y, X.double() @ W.double().t()))
    dX = torch.empty(R, Kin, device=dev)
    dW = torch.empty(Nout, Kin, device=dev)
    for tv in TERMS:
        L.tune("gemm_ex_terms", tv)
        # dX = dY . W (gemm_ex: A k-contiguous, B n-contiguous)
        t = timeit(lambda: TO.mm(dY, W, out=dX))
        report(f"dX   dY.W    ({Kin}->{Nout}) t{tv}", R, Kin, Nout, t, rel(dX, dY.double() @ W.double()))
        # dW = dY^T . X (A m-contiguous, K = R: split-K)
        t = timeit(lambda: TO.mm(dY.t(), X, out=dW))
        report(f"dW   dY^T.X  ({Kin}->{Nout}) t{tv}", Nout, Kin, R, t, rel(dW, dY.double().t() @ X.double()))
    L.tune("gemm_ex_terms", 0)
    del X, W, dY, Y, dX, dW
    torch.cuda.empty_cache()
