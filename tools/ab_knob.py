"""Same-process A/B of a tuning knob (catseg_tuning_set) on the headline step (L/14@336, T=150, bs=8, bf16):
one engine, one hipGraph per knob value (the value is read at launch, so at capture), rounds
interleaved; prints ms/step per value and whether the logits equal the first value's bit for bit.
usage: python tools/ab_knob.py mlp_variant 0 1
       python tools/ab_knob.py wide_store,ln_store,attn_store 2,1,1 0,0,0   (several knobs set together)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import numpy as np
import torch
from cat_seg import _lib as L
from cat_seg.arch import VIT_L14_336
from cat_seg.engine import CatSegEngine
from cat_seg.weights import synthesize_state_dict

knob, values = sys.argv[1], sys.argv[2:]
knobs = knob.split(",")
L.load()
def setter(v):
    vs = [int(x) for x in v.split(",")]
    assert len(vs) == len(knobs), (knobs, v)
    for k, x in zip(knobs, vs):
        L.tune(k, x)
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
stream = torch.cuda.Stream()
graphs, outs = {}, {}
for v in values:
    setter(v)
    with torch.no_grad(), torch.cuda.stream(stream):
        eng.head_logits(raw, sizes)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            outs[v] = eng.head_logits(raw, sizes)
    graphs[v] = g
setter(values[0])
ts = {v: [] for v in values}
for rnd in range(7):
    for v in values:
        graphs[v].replay(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            graphs[v].replay()
        torch.cuda.synchronize()
        ts[v].append((time.perf_counter() - t0) / 10 * 1e3)
ref = outs[values[0]]
for v in values:
    t = sorted(ts[v])[len(ts[v]) // 2]
    d = (outs[v] - ref).abs().max().item()
    print(f"{knob}({v}): {t:7.3f} ms/step  {B / t * 1e3:7.1f} img/s  max|logit diff| vs {values[0]}: {d:.3e}", flush=True)
