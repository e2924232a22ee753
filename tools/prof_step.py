"""Per-launch breakdown of one CAT-Seg forward (HIP events around every wrapped launch).
Usage: python tools/prof_step.py [--batch 8] [--classes 150] [--dtype bf16]"""
import argparse, os, sys, collections
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
from cat_seg import ops
from cat_seg.arch import VIT_L14_336
from cat_seg.engine import CatSegEngine
from cat_seg.weights import synthesize_state_dict

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--classes", type=int, default=150)
ap.add_argument("--dtype", default="bf16")
a = ap.parse_args()
dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
arch = VIT_L14_336
eng = CatSegEngine(arch, synthesize_state_dict(arch, 0), dtype=dt)
text = torch.nn.functional.normalize(torch.randn(a.classes, arch.embed_dim), dim=-1).cuda()
eng.set_text(text)
B, R = a.batch, 336
raw = (torch.rand(B, 3, 352, 352) * 255).cuda()
sizes = torch.tensor([[R, R]] * B, dtype=torch.int32).cuda()
eng.head_logits(raw, sizes); torch.cuda.synchronize()

LAST = [""]
real_call = ops.L.call
def call(name, *args):
    g = args[0]
    if name == "catseg_gemm":
        LAST[0] = f"gemm M{g.M} N{g.N} K{g.K}"
    elif name == "catseg_conv3x3":
        LAST[0] = f"conv S{g.S} {g.H}x{g.W} c{g.c1}+{g.c2}->{g.c_out}{' gn' if g.gn_mean else ''}"
    elif name == "catseg_attention":
        LAST[0] = f"attn mode{g.mode} L{g.seq_len} H{g.n_heads} d{g.head_dim} n{g.n_seq}"
    elif name == "catseg_layernorm":
        LAST[0] = f"layernorm rows{args[9]} cols{args[10]}"
    elif name == "catseg_rows_gemm":
        LAST[0] = f"rows_gemm M{args[2]} N{args[7]}{' ln' if args[3] else ''}"
    elif name == "catseg_rows_mlp":
        LAST[0] = f"rows_mlp M{args[2]} hidden{args[8]}"
    else:
        LAST[0] = name
    return real_call(name, *args)
ops.L.call = call
orig_exit = ops._rec.__exit__
def _exit(self, *exc):
    r = orig_exit(self, *exc)
    if ops.PROFILE:
        ops.PROFILE[-1]["shape"] = LAST[0]
    return r
ops._rec.__exit__ = _exit
ops.PROFILE = []
torch.cuda.synchronize()
import time
t0 = time.perf_counter()
eng.head_logits(raw, sizes); torch.cuda.synchronize()
wall = (time.perf_counter() - t0) * 1e3
recs = ops.PROFILE; ops.PROFILE = None
agg = collections.OrderedDict()
for r in recs:
    ms = r["start"].elapsed_time(r["end"])
    e = agg.setdefault(r.get("shape", r["kernel"]), [0, 0.0, 0, 0])
    e[0] += 1; e[1] += ms; e[2] += r["flops"]; e[3] += r["bytes"]
tot = sum(v[1] for v in agg.values())
print(f"total wrapped {tot:.3f} ms   (instrumented eager wall {wall:.1f} ms)")
for s, (n, ms, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    tf = fl / (ms / 1e3) / 1e12 if fl else 0
    gbs = by / (ms / 1e3) / 1e9 if by else 0
    print(f"{s:55s} x{n:3d} {ms:8.3f} ms {100*ms/tot:5.1f}% {tf:7.1f} TF/s {gbs:7.0f} GB/s")
