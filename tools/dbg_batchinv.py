"""Locate batch-size dependence: run each stage of the engine at bs=big and on a slice, compare bitwise."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cat-seg_amd")]
from cat_seg.arch import VIT_L14_336  # noqa: E402
from cat_seg.engine import CatSegEngine  # noqa: E402
from cat_seg.weights import synthesize_state_dict  # noqa: E402
from cat_seg import ops  # noqa: E402


def cmp(name, a, b):
    a, b = a.float(), b.float()
    d = (a - b).abs().max().item()
    print(f"{name:28s} equal={torch.equal(a, b)} maxdiff={d:.3e}", flush=True)


def main():
    big = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    arch = VIT_L14_336
    g = np.load(os.path.join(ROOT, "tests/golden/e2e_l14_ade150.npz"))
    eng = CatSegEngine(arch, synthesize_state_dict(arch, seed=0), dtype=torch.bfloat16)
    eng.set_text(torch.from_numpy(g["text"]).cuda())
    gen = torch.Generator().manual_seed(35)
    raw = (torch.rand(big, 3, 352, 352, generator=gen) * 255).cuda()
    sizes = torch.tensor([[336, 336]] * big, dtype=torch.int32).cuda()
    Lt = arch.grid ** 2 + 1
    HW = arch.grid ** 2
    with torch.no_grad():
        fB, hB = eng.encode_image(raw, sizes)
        f1, h1 = eng.encode_image(raw[:1].contiguous(), sizes[:1].contiguous())
        cmp("feats", fB[:Lt], f1)
        cmp("hook0", hB[0][:Lt], h1[0])
        cmp("hook1", hB[1][:Lt], h1[1])
        gB = eng.guidance(fB, hB)
        g1 = eng.guidance(f1, h1)
        cmp("res3", gB[0][:HW], g1[0])
        cmp("res4", gB[1][:4 * HW], g1[1])
        cmp("res5", gB[2][:16 * HW], g1[2])
        # aggregate on identical inputs (image 0 of the big batch alone vs inside the batch)
        lB = eng.aggregate(fB, *gB)
        l1 = eng.aggregate(fB[:Lt].contiguous(), gB[0][:HW].contiguous(), gB[1][:4 * HW].contiguous(),
                           gB[2][:16 * HW].contiguous())
        cmp("aggregate(same inputs)", lB[:1], l1)


if __name__ == "__main__":
    main()
