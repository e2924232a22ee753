"""Where the boundary leg's time goes (bench.py boundary_pass vs the engine leg): per-call host time of
CATSeg.forward, and the step time with host uint8 images, device uint8 images and device fp32 images."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cat-seg_amd"), ROOT]
import torch
import bench
from cat_seg import add_cat_seg_config, build_model, get_cfg

B, S, T = 8, 336, 150
c = get_cfg()
add_cat_seg_config(c)
c.merge_from_file(os.path.join(ROOT, "cat-seg_amd", "configs", "vitl_336.yaml"))
c.merge_from_list(["MODEL.SEM_SEG_HEAD.POOLING_SIZES", "[1,1]", "MODEL.CATSEG_HIP.DTYPE", "bf16"])
model = build_model(c).cuda().eval()
model.sem_seg_head.predictor.set_class_tokens(bench.class_tokens("ade150", T))
gen = torch.Generator().manual_seed(4321)
host = [{"image": (torch.rand(3, S, S, generator=gen) * 255).to(torch.uint8)} for _ in range(B)]
dev8 = [{"image": x["image"].cuda()} for x in host]
devf = [{"image": x["image"].float().cuda()} for x in host]


def run(batch, steps=20, label=""):
    with torch.no_grad():
        for _ in range(3):
            out = model(batch)
        torch.cuda.synchronize()
        host_ms = []
        t0 = time.perf_counter()
        for _ in range(steps):
            a = time.perf_counter()
            out = model(batch)
            host_ms.append((time.perf_counter() - a) * 1e3)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
    host_ms.sort()
    print(f"{label:28s} {el:7.3f} ms/step  host per call median {host_ms[len(host_ms) // 2]:.3f} ms "
          f"max {host_ms[-1]:.3f}", flush=True)


for rnd in range(2):
    run(host, label="host uint8")
    run(dev8, label="device uint8")
    run(devf, label="device fp32")
eng = model.engine
with torch.no_grad():
    t = time.perf_counter(); [model.engine for _ in range(100)]; print("engine property", (time.perf_counter() - t) * 10, "ms")


# variant: the H2D copy on the compute stream itself (no copy stream, no cross-stream events)
def stage_same_stream(self, eng, images, canvas):
    dt = images[0].dtype
    key = ("same", tuple(canvas.shape), dt)
    st = self._stage.get(key)
    if st is None:
        st = {"slots": [{"host": torch.zeros(canvas.shape, dtype=dt, pin_memory=True),
                         "dev": torch.zeros(canvas.shape, dtype=dt, device=canvas.device), "ev": None}
                        for _ in range(2)], "next": 0}
        self._stage[key] = st
    slot = st["slots"][st["next"]]
    st["next"] ^= 1
    if slot["ev"] is not None:
        slot["ev"].synchronize()
    for k, im in enumerate(images):
        slot["host"][k, :, : im.shape[-2], : im.shape[-1]].copy_(im)
    slot["dev"].copy_(slot["host"], non_blocking=True)
    canvas.copy_(slot["dev"])
    slot["ev"] = torch.cuda.Event()
    slot["ev"].record()


import types
orig = model._stage_canvas
model._stage_canvas = types.MethodType(stage_same_stream, model)
for rnd in range(2):
    run(host, label="host uint8, same-stream copy")
    model._stage_canvas = orig
    run(host, label="host uint8, copy stream")
    model._stage_canvas = types.MethodType(stage_same_stream, model)
