"""Time the bf16 GEMM tile variants on the ViT-L/14@336 (B=8) shapes and check them.

usage: python tools/micro_gemm.py [variants, default "-1,0,1,2,3,4,5,6,7,8"]
Each variant is checked against torch (fp32 accumulate of the same bf16 operands) and
timed over interleaved rounds in one process (median of per-round means).
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg import _lib as L

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,5").split(",")]
# variants >= 1000: automatic tile, tile order grouped by (v - 1000) m-tiles (tuning knob gemm_group);
# >= 2000: variant v - 2000 with the prefetching lean epilogue (tuning knob epi_prefetch)
M = 8 * 577
shapes = {"qkv": (3072, 1024, L.ACT_NONE, False), "proj": (1024, 1024, L.ACT_NONE, True),
          "fc1": (4096, 1024, L.ACT_QUICKGELU, False), "fc2": (1024, 4096, L.ACT_NONE, True),
          "fc2h": (1024, 2048, L.ACT_NONE, True),   # half of fc2's K (split-K probe: run at 2 M for 2 halves)
          "sq4k": (4096, 4096, L.ACT_NONE, False), "sq8k": (8192, 8192, L.ACT_NONE, False)}
# MG_SHAPES=qkv,fc1,sq4k selects shapes (sq4k: M = N = K = 4096, the guide's reference size)
sel = os.environ.get("MG_SHAPES", "qkv,proj,fc1,fc2").split(",")
shapes = {k: v for k, v in shapes.items() if k in sel}
dev = "cuda"
torch.manual_seed(0)
lib = L.load()
res = {}
for name, (N, K, act, has_res) in shapes.items():
    M = {"sq4k": 4096, "sq8k": 8192}.get(name, int(os.environ.get("MG_M", 8 * 577)))   # MG_M=2308: config 4's 4 images
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    bias = torch.rand(N, device=dev) - 0.5
    # the residual-stream GEMMs (out-proj, fc2) write the fp32 stream, as in the engine
    R = (torch.rand(M, N, device=dev) - 0.5) if has_res else None
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if has_res else torch.bfloat16)
    ref = A.float() @ W.float().t() + bias
    if act == L.ACT_QUICKGELU:
        ref = ref * torch.sigmoid(1.702 * ref)
    if R is not None:
        ref = ref + R.float()
    def run():
        ops.gemm(A, W, out, bias=bias, act=act, res=R)
    def setv(v):
        # 5000 + x: variant 2000 + x with the wide kernels' fp32-staged epilogue (tuning knob wide_epi 0)
        L.tune("wide_epi", 0 if v >= 5000 else 1)
        v = v - 3000 if v >= 5000 else v
        pf = v >= 2000                 # 2000 + v: variant v with the prefetching lean epilogue (epi_prefetch 1,
                                       # the library default); v < 2000 runs with epi_prefetch 0;
                                       # 3000 + g = 2000 + (1000 + g): the automatic tile, prefetching
                                       # epilogue, tile-order group g
        v = v - 2000 if pf else v
        L.tune("epi_prefetch", 1 if pf else 0)
        L.tune("gemm_variant", 0 if v >= 1000 else v)
        L.tune("gemm_group", v - 1000 if v >= 1000 else 0)
    for v in variants:
        setv(v)
        out.zero_()
        run(); torch.cuda.synchronize()
        err = (out.float() - ref).abs().max().item()
        res[(name, v)] = {"err": err, "t": []}
    flops = 2 * M * N * K
    for rnd in range(7):
        for v in variants:
            setv(v)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record(); torch.cuda.synchronize()
            res[(name, v)]["t"].append(e0.elapsed_time(e1) / 20)
    # hipBLASLt (torch.mm, bf16 out, no fused epilogue) as the library reference point
    Ab, Wt = A, W.t()
    torch.mm(Ab, Wt); torch.cuda.synchronize()
    tl = []
    for rnd in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.mm(Ab, Wt)
        e1.record(); torch.cuda.synchronize()
        tl.append(e0.elapsed_time(e1) / 20)
    t = sorted(tl)[3]
    print(f"{name:5s} N={N:5d} K={K:5d} torch.mm   : {t * 1e3:8.1f} us  {flops / t / 1e9:7.1f} TF/s  (hipBLASLt)")
    for v in variants:
        t = sorted(res[(name, v)]["t"])[3]
        print(f"{name:5s} N={N:5d} K={K:5d} variant {v:2d}: {t * 1e3:8.1f} us  {flops / t / 1e9:7.1f} TF/s  "
              f"({flops / t / 1e9 / 2500:.3f} of 2.5 PF)  max_err {res[(name, v)]['err']:.3e}", flush=True)
L.tune("gemm_variant", 0)
L.tune("gemm_group", 0)
