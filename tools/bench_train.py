"""Training-step throughput of the MI355X path (not the headline metric).

One step = the reference Trainer's iteration (train_net.py:298-311 via detectron2 SimpleTrainer):
CATSeg training forward (fp32 CLIP with CLIP_FINETUNE "attention", the aggregation head) -> BCE loss
-> backward through the HIP kernels -> AdamW with full-model clipping (train_net.py:228-253),
on the reference training config (configs/vitb_384.yaml: ViT-B/16 @384, COCO-Stuff's 171 classes,
POOLING [2,2], IMS_PER_BATCH 4, BASE_LR 2e-4, CLIP_GRADIENTS full_model 0.01), synthetic images and
labels, random-init weights.  Prints one JSON line; --profile adds the per-kernel HIP-event times of one
step (ops.PROFILE).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]

from cat_seg import add_cat_seg_config, build_model, get_cfg, ops  # noqa: E402
from cat_seg.optim import build_optimizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clip", default="ViT-B/16", choices=["ViT-B/16", "ViT-L/14@336px"])
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--classes", type=int, default=171)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--finetune", default="attention", choices=["attention", "none", "full"])
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--image", type=int, default=384,
                    help="training crop (the reference's INPUT.CROP.SIZE (384, 384) for B/16 and L/14; the "
                         "CLIP encoder sees it resized to its resolution, cat_seg_model.py:136-146)")
    a = ap.parse_args()

    cfg = get_cfg()
    add_cat_seg_config(cfg)
    cfg.merge_from_file(os.path.join(ROOT, "cat-seg_amd", "configs", "vitb_384.yaml"))
    cfg.merge_from_list(["MODEL.SEM_SEG_HEAD.CLIP_PRETRAINED", a.clip, "MODEL.SEM_SEG_HEAD.POOLING_SIZES", "[2,2]",
                         "MODEL.SEM_SEG_HEAD.CLIP_FINETUNE", a.finetune, "MODEL.CATSEG_HIP.DTYPE", "f32",
                         "SOLVER.BASE_LR", "0.0002", "SOLVER.CLIP_GRADIENTS.ENABLED", "True",
                         "SOLVER.CLIP_GRADIENTS.CLIP_TYPE", "full_model", "SOLVER.CLIP_GRADIENTS.CLIP_VALUE", "0.01"])
    if a.clip != "ViT-B/16":
        cfg.merge_from_list(["MODEL.SEM_SEG_HEAD.TEXT_GUIDANCE_DIM", "768",
                             "MODEL.SEM_SEG_HEAD.APPEARANCE_GUIDANCE_DIM", "768"])
    model = build_model(cfg).cuda().train()
    toks = np.load(os.path.join(ROOT, "tests", "golden", "class_tokens.npz"))["ade847"][:a.classes]
    model.sem_seg_head.predictor.set_class_tokens(torch.from_numpy(toks.astype(np.int64)))
    opt = build_optimizer(cfg, model)
    S = a.image
    gen = torch.Generator().manual_seed(0)
    batch = [{"image": torch.randint(0, 256, (3, S, S), generator=gen, dtype=torch.uint8),
              "sem_seg": torch.randint(0, a.classes, (S, S), generator=gen)} for _ in range(a.batch)]
    for b in batch:
        b["sem_seg"][:8] = 255

    def step():
        opt.zero_grad(set_to_none=True)
        loss = model(batch)["loss_sem_seg"]
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    out = {"metric": "training images/sec (forward + backward + AdamW step)", "value": a.batch / dt,
           "unit": "images/sec", "ms_per_step": dt * 1e3, "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
           "dtype": "f32", "data": "synthetic images / labels, random-init weights",
           "loss": float(loss.detach()), "grad_norm": float(opt.last_grad_norm[0]),
           "peak_mem_gb": torch.cuda.max_memory_allocated() / 2 ** 30,
           "config": {"clip": a.clip, "resolution": S, "clip_resolution": model.clip_resolution[0], "classes": a.classes, "batch": a.batch, "pooling": [2, 2],
                      "clip_finetune": a.finetune, "optimizer": "AdamW (HIP) + full-model clip 0.01"}}
    if a.profile:
        ops.PROFILE = []
        step()
        torch.cuda.synchronize()
        fam, shp = {}, {}
        for r in ops.PROFILE:
            ms = r["start"].elapsed_time(r["end"])
            f = fam.setdefault(r["kernel"], [0.0, 0, 0.0])
            f[0] += ms
            f[1] += 1
            f[2] += r["flops"]
            if r.get("shape") is not None:
                g = shp.setdefault((r["kernel"],) + tuple(r["shape"]), [0.0, 0, 0.0])
                g[0] += ms
                g[1] += 1
                g[2] += r["flops"]
        ops.PROFILE = None
        # the GEMM launches by shape (M, N, K[, A / B contiguous dimension]): where the GEMM time goes
        out["gemm_shapes"] = [{"kernel": k[0], "shape": list(k[1:]), "ms": round(v[0], 3), "launches": v[1],
                               "tflops": round(v[2] / (v[0] * 1e9), 1) if v[0] > 0 else None}
                              for k, v in sorted(shp.items(), key=lambda kv: -kv[1][0])[:40]]
        tot = sum(v[0] for v in fam.values())
        out["kernels_ms"] = {k: {"ms": round(v[0], 3), "launches": v[1],
                                 "tflops": round(v[2] / (v[0] * 1e9), 1) if v[0] > 0 and v[2] else None}
                             for k, v in sorted(fam.items(), key=lambda kv: -kv[1][0])}
        out["kernels_total_ms"] = round(tot, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
