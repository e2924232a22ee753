"""Config-5 accuracy sweep: which ViT GEMMs in fp8 (sliding 640², L/14, T=459) vs the oracle."""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "cat-seg_amd"), os.path.join(os.path.dirname(__file__), "..")]
import torch
from cat_seg.arch import VIT_L14_336
from cat_seg.engine import CatSegEngine
from cat_seg.weights import synthesize_state_dict
from oracle import catseg_oracle as O

arch = VIT_L14_336
sd = synthesize_state_dict(arch, seed=0)
T = 459
gen = torch.Generator().manual_seed(5)
text = torch.nn.functional.normalize(torch.randn(T, arch.embed_dim, generator=gen), dim=-1)
img = torch.randint(0, 256, (3, 480, 640), generator=gen).float()
torch.set_num_threads(16)
t0 = time.time()
ref = O.catseg_forward_sliding(arch, sd, [{"image": img, "height": 480, "width": 640}], text.unsqueeze(1))[0]["sem_seg"]
print("oracle", time.time() - t0, flush=True)
raw = torch.zeros(1, 3, 480, 640); raw[0] = img
raw = raw.cuda(); sizes = torch.tensor([[480, 640]], dtype=torch.int32).cuda()
for sel in ((), ("wqkv",), ("wo",), ("wfc",), ("wpr",), ("wqkv", "wfc"), ("wqkv", "wo", "wfc"), True):
    eng = CatSegEngine(arch, sd, dtype=torch.bfloat16, vit_fp8=sel)
    eng.set_text(text.cuda())
    got = eng.forward_sliding(raw, sizes, [(480, 640)])[0].cpu()
    e = (got - ref).abs()
    # per-class view: classes whose whole map differs (top-k swaps) vs the rest
    cls = e.mean(dim=(1, 2))
    print(f"{sel}: mean {e.mean().item():.4e} max {e.max().item():.3f}  classes>0.05: {(cls > 0.05).sum().item()}"
          f"  mean over the rest {cls[cls <= 0.05].mean().item():.4e}", flush=True)
    del eng
