"""Same-process A/B of CatSegEngine switches on the headline step (L/14@336, T=150, bs=8, bf16):
one engine, one hipGraph per configuration, interleaved timing rounds (cdna_hip_programming.md
§5.4 rule 24).  usage: python tools/ab_engine.py side_stream fused_swin_mlp fold_upconv ..."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import numpy as np
import torch
from cat_seg.arch import VIT_L14_336
from cat_seg.engine import CatSegEngine
from cat_seg.weights import synthesize_state_dict

flags = sys.argv[1:] or ["side_stream"]
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
configs = [("baseline", {})] + [(f"-{f}", {f: False}) for f in flags]
stream = torch.cuda.Stream()
graphs, outs = {}, {}
for name, over in configs:
    saved = {k: getattr(eng, k) for k in over}
    for k, v in over.items():
        setattr(eng, k, v)
    with torch.no_grad(), torch.cuda.stream(stream):
        eng.head_logits(raw, sizes)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            outs[name] = eng.head_logits(raw, sizes)
    graphs[name] = g
    for k, v in saved.items():
        setattr(eng, k, v)
ts = {n: [] for n, _ in configs}
for rnd in range(6):
    for name, _ in configs:
        graphs[name].replay(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            graphs[name].replay()
        torch.cuda.synchronize()
        ts[name].append((time.perf_counter() - t0) / 10 * 1e3)
ref = outs["baseline"]
for name, _ in configs:
    t = sorted(ts[name])[len(ts[name]) // 2]
    same = torch.equal(outs[name], ref)
    print(f"{name:20s} {t:7.3f} ms/step  {B / t * 1e3:7.1f} img/s  bit-identical to baseline: {same}", flush=True)
