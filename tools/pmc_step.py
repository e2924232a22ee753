"""One CAT-Seg forward (L/14@336, T=150, bs=8, bf16) for rocprofv3 --pmc passes.

Runs the step once to warm up, then launches a fill kernel as a delimiter
(at::native FillFunctor<float>) and runs the step once more; tools/pmc_traffic.py keeps
only the dispatches after the last delimiter, so setup launches (weight prep, class cache)
never enter the per-launch averages.  Eager launches (no hipGraph) so every dispatch is
counted on its own.
Usage (GPU box): rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d DIR -- python3 tools/pmc_step.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch  # noqa: E402
from cat_seg import ops  # noqa: E402
from cat_seg.arch import VIT_L14_336  # noqa: E402
from cat_seg.engine import CatSegEngine  # noqa: E402
from cat_seg.weights import synthesize_state_dict  # noqa: E402

B, T = 8, 150
arch = VIT_L14_336
R = arch.clip_resolution
with torch.no_grad():
    eng = CatSegEngine(arch, synthesize_state_dict(arch, 0), dtype=torch.bfloat16)
    gen = torch.Generator().manual_seed(0)
    eng.set_text(torch.nn.functional.normalize(torch.randn(T, arch.embed_dim, generator=gen), dim=-1).cuda())
    raw = torch.zeros(B, 3, 352, 352)
    raw[:, :, :R, :R] = torch.rand(B, 3, R, R, generator=gen) * 255
    raw = raw.cuda()
    sizes = torch.tensor([[R, R]] * B, dtype=torch.int32).cuda()
    out = torch.empty(B, T, R, R, device="cuda")
    marker = torch.empty(1024, device="cuda")

    def step():
        lg = eng.head_logits(raw, sizes)
        ops.postprocess(lg, out, crop=(min(lg.shape[-2], R), min(lg.shape[-1], R)))

    step()
    torch.cuda.synchronize()
    marker.fill_(1.0)
    step()
    torch.cuda.synchronize()
print("pmc_step done")
