"""Same-process A/B: the headline batch (L/14@336, T=150, bs=8, bf16) as ONE stream of bs=8
kernels vs the batch split into S sub-batches on S concurrent streams inside one hipGraph
(each sub-batch's kernels are single-round launches; concurrent sub-batches fill each other's
prologue / epilogue / tail gaps).  Prints ms/step and whether the logits are bit-identical
(the kernels choose tiles from per-image shapes, so they must be).
usage: python tools/ab_streams.py [splits ...]   (default: 2 4)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import numpy as np
import torch
from cat_seg.arch import VIT_L14_336
from cat_seg.engine import CatSegEngine
from cat_seg.weights import synthesize_state_dict

# S > 0: S sub-batches on S streams in lockstep; S < 0: |S| sub-batches, sub-batch i's encoder
# starts when sub-batch i-1's encoder has finished (its head overlaps the next encoder)
splits = [int(s) for s in sys.argv[1:]] or [2, 4, -2, -4]
arch = VIT_L14_336
B, T, R = 8, 150, arch.clip_resolution
eng = CatSegEngine(arch, synthesize_state_dict(arch, 0), dtype=torch.bfloat16)
tok = np.load(os.path.join(ROOT, "tests", "golden", "class_tokens.npz"))["ade150"][:T]
with torch.no_grad():
    eng.set_text(eng.encode_text(torch.from_numpy(tok.astype(np.int32))))
gen = torch.Generator().manual_seed(1234)
raw = torch.zeros(B, 3, 352, 352)
raw[:, :, :R, :R] = torch.rand(B, 3, R, R, generator=gen) * 255
raw = raw.cuda()
sizes = torch.tensor([[R, R]] * B, dtype=torch.int32, device="cuda")
main = torch.cuda.Stream()
side = [torch.cuda.Stream() for _ in range(max(abs(s) for s in splits))]


def staggered(S):
    b = B // S
    outs, prev = [None] * S, None
    for i in range(1, S):
        side[i].wait_stream(main)         # fork before any work is queued on main
    for i in range(S):
        st = main if i == 0 else side[i]
        with torch.cuda.stream(st):
            if prev is not None:
                st.wait_event(prev)
            f, hk = eng.encode_image(raw[i * b:(i + 1) * b], sizes[i * b:(i + 1) * b])
            prev = torch.cuda.Event()
            prev.record(st)
            outs[i] = eng.aggregate(f, *eng.guidance(f, hk))
    for i in range(1, S):
        main.wait_stream(side[i])
    return outs


def step(S):
    if S == 1:
        return eng.head_logits(raw, sizes)
    if S < 0:
        return staggered(-S)
    b = B // S
    outs = [None] * S
    for i in range(1, S):
        side[i].wait_stream(main)
        with torch.cuda.stream(side[i]):
            outs[i] = eng.head_logits(raw[i * b:(i + 1) * b], sizes[i * b:(i + 1) * b])
    outs[0] = eng.head_logits(raw[:b], sizes[:b])
    for i in range(1, S):
        main.wait_stream(side[i])
    return outs


graphs, res = {}, {}
for S in [1] + splits:
    with torch.no_grad(), torch.cuda.stream(main):
        step(S)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main):
            res[S] = step(S)
    graphs[S] = g
ts = {S: [] for S in graphs}
for rnd in range(6):
    for S, g in graphs.items():
        g.replay(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        ts[S].append((time.perf_counter() - t0) / 10 * 1e3)
ref = res[1]
for S in graphs:
    t = sorted(ts[S])[len(ts[S]) // 2]
    same = True if S == 1 else torch.equal(torch.cat(res[S], 0), ref)
    print(f"streams {S}: {t:7.3f} ms/step  {B / t * 1e3:7.1f} img/s  bit-identical to one stream: {same}", flush=True)
