"""Benchmark: CAT-Seg dense inference, images/sec @ ViT-L/14 336², 150 classes, bs=8 per GPU.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = the full eval forward of one batch of 8 synthetic images already resident in
HBM: CLIP-normalize / pad / resize -> CLIP ViT-L/14 dense encoder -> cost volume ->
2 aggregation layers -> guided upsampler -> sigmoid logits bilinearly upsampled to
336² (cat_seg_model.py:147-229).  Class embeddings of the 150 ade150 prompts are
encoded once on the GPU before timing (the predictor's eval cache,
cat_seg_predictor.py:191-192).  With N > 1 each rank runs its own 8 images and the
(8, 150, 96, 96) logits are all-gathered over RCCL (weak scaling).

Prints ONE JSON line (rank 0) with the metric, a roofline object for the dominant
kernel (HIP-event timed per launch on the launch stream, algorithmic FLOPs from the
launch shapes) and the CPU baseline (the oracle, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cat-seg_amd"))
sys.path.insert(0, ROOT)

from cat_seg import ops  # noqa: E402
from cat_seg.distributed import gather_logits  # noqa: E402
from cat_seg.arch import VIT_L14_336  # noqa: E402
from cat_seg.engine import CatSegEngine  # noqa: E402
from cat_seg.weights import synthesize_state_dict  # noqa: E402

GF_PER_IMAGE = 875.7          # reference eval forward FLOPs, L/14@336, T=150
GF_PER_IMAGE_CFG4 = 1128.0    # L/14@336, T=847 (top-256)
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_FP8_TFLOPS = 5000.0      # MI355X dense fp8 MFMA (block-scaled K=128 form)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--classes", type=int, default=150)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one hipGraph per step")
    ap.add_argument("--cpu-images", type=int, default=4, help="oracle sample size for cpu_baseline (0 = skip)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--config", type=int, default=3, choices=[3, 4, 5],
                    help="3 = the headline (L/14@336, T=150, bf16); 4 = ade847 (top-256) at 4 images/GPU "
                         "(SURVEY §8 config 4: bs=32 over 8 GPUs); 5 = sliding-window 640², pc459 classes, "
                         "fp8 ViT GEMMs (SURVEY §8 config 5)")
    ap.add_argument("--vit-fp8", action="store_true",
                    help="config 5's e4m3 CLIP image-encoder GEMMs (not the headline: the headline is bf16)")
    return ap.parse_args()


def class_tokens(T):
    g = np.load(os.path.join(ROOT, "tests", "golden", "class_tokens.npz"))
    tok = g["ade150"] if T <= 150 else g["pc459"] if T <= 459 else g["ade847"]
    return torch.from_numpy(tok[:T].astype(np.int32))


def _spawned_rank(local, args_list, world, port):
    """One rank of a self-launched N-GPU run (python bench.py --gpus N without torchrun)."""
    os.environ.update(RANK=str(local), LOCAL_RANK=str(local), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + args_list
    main()


def launch_ranks(n):
    """--gpus N with no WORLD_SIZE in the environment: start N rank processes (spawned
    interpreters, one per GPU) before this process touches the GPU, and exit with their status
    (detectron2 `launch` for the reference, train_net.py:314-324)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_spawned_rank, args=(sys.argv[1:], n, port), nprocs=n, join=True, start_method="spawn")


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: the ranks must match the GPUs asked for")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"RCCL group has {dist.get_world_size()} ranks, expected {args.gpus}")
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    arch = VIT_L14_336
    cfg5 = args.config == 5
    cfg4 = args.config == 4
    if cfg4:      # the class-attention stress config: T = 847 -> top-256, 4 images per GPU
        if args.classes == 150:
            args.classes = 847
        if args.batch == 8:
            args.batch = 4
    gf_per_image = GF_PER_IMAGE_CFG4 if cfg4 else GF_PER_IMAGE
    if cfg5:
        if world > 1:
            raise SystemExit("--config 5 is a single-GPU measurement (the scaling runs use the headline config)")
        args.vit_fp8 = True
        if args.classes == 150:
            args.classes = 459
    B, T = args.batch, args.classes
    R = arch.clip_resolution

    sd = synthesize_state_dict(arch, seed=0)
    eng = CatSegEngine(arch, sd, dtype=dtype, device=dev, vit_fp8=args.vit_fp8)
    with torch.no_grad():
        text = eng.encode_text(class_tokens(T))
        eng.set_text(text)
    gen = torch.Generator().manual_seed(1234 + rank)
    S = 640 if cfg5 else R          # config 5: 640² images through the sliding-window branch
    pad = (S + 31) // 32 * 32
    raw = torch.zeros(B, 3, pad, pad)
    raw[:, :, :S, :S] = torch.rand(B, 3, S, S, generator=gen) * 255
    raw = raw.to(dev)
    sizes = torch.tensor([[S, S]] * B, dtype=torch.int32, device=dev)
    out = None if cfg5 else torch.empty(B, T, R, R, device=dev)
    gsize = eng.SLIDE_OUT if cfg5 else 4 * arch.grid
    gathered = torch.empty(world * B, T, gsize, gsize, device=dev) if world > 1 else None

    def step():
        if cfg5:      # crops + head + Fold merge -> 640² probabilities at the image size (sem_seg_postprocess)
            return eng.forward_sliding(raw, sizes, [(S, S)] * B)[0]
        logits = eng.head_logits(raw, sizes)
        ops.postprocess(logits, out, crop=(min(logits.shape[-2], R), min(logits.shape[-1], R)))
        return logits

    stream = torch.cuda.Stream(device=dev)
    graph = None
    torch.cuda.synchronize()
    with torch.no_grad():
        if not args.no_graph:
            with torch.cuda.stream(stream):
                step()            # allocate / warm the caching allocator outside capture
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                g_logits = step()

        def run():
            if graph is not None:
                graph.replay()
                lg = g_logits
            else:
                with torch.cuda.stream(stream):
                    lg = step()
            if world > 1:
                with torch.cuda.stream(stream):
                    gather_logits(lg, world * B, out=gathered)     # RCCL all-gather over xGMI
            return lg

        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lg_last = run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    images = world * B * args.steps
    value = images / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # the all-gather is a pure copy: every rank's slice of the gathered logits must equal its
    # own logits bit for bit (the multi-GPU parity gate of BASELINE.md), checked after timing
    gather_ok = None
    if world > 1:
        local_lg = g_logits if graph is not None else lg_last
        mine = gathered[rank * B:(rank + 1) * B]
        flag = torch.tensor([1 if torch.equal(mine, local_lg) else 0], device=dev, dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather_ok = bool(flag.item())

    roofline, kernels = None, None
    if rank == 0 and not args.no_roofline:
        roofline, kernels = roofline_pass(step, stream, dtype)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_images > 0:
        cpu = (cpu_baseline_sliding(arch, sd, text.cpu()) if cfg5 else
               cpu_baseline(arch, sd, text.cpu(), min(args.cpu_images, 2) if cfg4 else args.cpu_images))
    if rank == 0:
        path_tflops = gf_per_image * value / 1e3
        line = {
            "metric": ("images/sec @ ViT-L/14 sliding-window 640² (5 crops/image), 459 classes, fp8 ViT GEMMs "
                       "(SURVEY §8 config 5; not the headline)" if cfg5 else
                       "images/sec @ ViT-L/14 336², 847 classes (top-256), 4 images/GPU "
                       "(SURVEY §8 config 4; not the headline)" if cfg4 else
                       "images/sec @ ViT-L/14 336², 150 classes, bs=8; 1/2/4/8-GPU scaling"),
            "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "ranks": world,
            "gather_bit_identical": gather_ok,
            "dtype": args.dtype + ("+fp8e4m3 ViT GEMMs" if args.vit_fp8 else ""),
            "data": "synthetic (seeded rand*255 images, deterministic synthetic weights, "
                    f"{'pc459' if cfg5 else 'ade847' if cfg4 else 'ade150'} prompt tokens)",
            "config": {"workload": (f"CATSeg eval forward, TEST.SLIDING_WINDOW: {B} images/GPU of 640², "
                                    f"{5 * B} crops through ViT-L/14@336, T={T} (top-256 per crop), "
                                    "Fold/avg merge to 640² probabilities" if cfg5 else
                                    f"CATSeg eval forward ViT-L/14@336, T={T} classes, bs={B}/GPU, "
                                    "POOLING [1,1], sigmoid upsampled to 336x336"),
                       "global_batch": world * B, "classes": T, "resolution": R,
                       "parallelism": f"batch-shard x{world} + RCCL all-gather of logits" if world > 1 else "1 GPU",
                       "hipgraph": graph is not None},
            "roofline": roofline,
            "path_roofline": None if cfg5 else {"bound": "mfma", "achieved": round(path_tflops, 2),
                              "peak": PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS,
                              "unit": "TFLOP/s", "gf_per_image": gf_per_image,
                              "frac": round(path_tflops / (PEAK_BF16_TFLOPS if dtype == torch.bfloat16
                                                           else PEAK_F32_TFLOPS), 4)},
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(family):
    """HBM bytes per launch of `family` from the newest committed PMC summary
    (profiles/<round>/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per the gfx950 note)."""
    import glob
    # profiles/<round>/[<version>/]pmc_traffic.json: the lexicographically last is the newest
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_traffic.json"), recursive=True))
    if not files:
        return None, None
    fam = json.load(open(files[-1]))["families"].get(family)
    if fam is None:
        return None, None
    return fam["traffic_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def roofline_pass(step, stream, dtype):
    """One eager pass with HIP events around every wrapped launch (on the launch stream)."""
    ops.PROFILE = []
    with torch.no_grad(), torch.cuda.stream(stream):
        step()
    torch.cuda.synchronize()
    recs, ops.PROFILE = ops.PROFILE, None
    agg = {}
    for r in recs:
        ms = r["start"].elapsed_time(r["end"])
        a = agg.setdefault(r["kernel"], {"launches": 0, "ms": 0.0, "flops": 0, "ref_flops": 0, "bytes": 0})
        a["launches"] += 1
        a["ms"] += ms
        a["flops"] += r["flops"]
        a["ref_flops"] += r.get("ref_flops", r["flops"])
        a["bytes"] += r["bytes"]
    top = max(agg, key=lambda k: agg[k]["ms"])
    a = agg[top]
    avg_s = a["ms"] / a["launches"] / 1e3
    traffic, tsrc = pmc_traffic(top)
    if a["flops"] > 0:
        achieved = a["flops"] / a["launches"] / avg_s / 1e12
        peak = (PEAK_FP8_TFLOPS if top == "gemm_fp8" else
                PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS)
        roof = {"bound": "mfma", "kernel": top, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "launches": a["launches"], "avg_launch_us": round(avg_s * 1e6, 2),
                "flops_per_launch": a["flops"] // a["launches"],
                "algorithmic_bytes_per_launch": a["bytes"] // a["launches"], "traffic_source": tsrc}
    else:
        achieved = a["bytes"] / a["launches"] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": top, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                "launches": a["launches"], "avg_launch_us": round(avg_s * 1e6, 2), "traffic_source": tsrc}
    # tflops: executed work / time; ref_tflops: the reference's count for the module / time
    # (differs where the build skips padding rows, per-class guidance halves or ConvT maps)
    kern = {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                "tflops": round(v["flops"] / (v["ms"] / 1e3) / 1e12, 2) if v["flops"] else None,
                **({"ref_tflops": round(v["ref_flops"] / (v["ms"] / 1e3) / 1e12, 2)}
                   if v["ref_flops"] != v["flops"] else {})}
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["ms"])}
    return roof, kern


def host_cores() -> int:
    """Cores this process may use: the affinity mask, capped by OMP_NUM_THREADS when the host
    sets it (the GPU box gives each job a 16-thread share of a larger machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def _timed_runs(fn, runs):
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return ts


def cpu_baseline_sliding(arch, sd, text, runs=3):
    """The oracle's sliding-window branch on one 640² image (config 5's CPU baseline):
    1 warm-up, median of `runs` timed runs."""
    from oracle import catseg_oracle as O

    cores = host_cores()
    torch.set_num_threads(cores)
    gen = torch.Generator().manual_seed(99)
    inp = [{"image": torch.rand(3, 640, 640, generator=gen) * 255}]
    O.catseg_forward_sliding(arch, sd, inp, text.unsqueeze(1))        # warm-up
    ts = _timed_runs(lambda: O.catseg_forward_sliding(arch, sd, inp, text.unsqueeze(1)), runs)
    med = float(np.median(ts))
    return {"value": round(1 / med, 4), "unit": "images/s", "cores": cores, "kind": "port", "runs": runs,
            "spread": [round(min(ts), 2), round(max(ts), 2)],
            "sample": f"1 image of the same workload (640² sliding, 5 crops, L/14@336, T={text.shape[0]}, fp32) "
                      f"through oracle/catseg_oracle.py on {cores} host threads: 1 warm-up, median of {runs} runs "
                      f"({med:.1f} s)"}


def cpu_baseline(arch, sd, text, n_images, runs=3):
    """The oracle (CPU fp32 restatement of the reference path) on a bounded sample of the same
    workload: a batch of `n_images`, 1 warm-up, the median of `runs` timed runs."""
    from oracle import catseg_oracle as O

    cores = host_cores()
    torch.set_num_threads(cores)
    gen = torch.Generator().manual_seed(99)
    R = arch.clip_resolution
    inputs = [{"image": torch.rand(3, R, R, generator=gen) * 255} for _ in range(n_images)]
    O.catseg_forward(arch, sd, inputs[:1], text.unsqueeze(1))     # warm-up
    ts = _timed_runs(lambda: O.catseg_forward(arch, sd, inputs, text.unsqueeze(1), all_images=True), runs)
    med = float(np.median(ts))
    return {"value": round(n_images / med, 4), "unit": "images/s", "cores": cores, "kind": "port", "runs": runs,
            "spread": [round(n_images / max(ts), 4), round(n_images / min(ts), 4)],
            "sample": f"batches of {n_images} images of the same workload (L/14@336, T={text.shape[0]}, fp32) through "
                      f"oracle/catseg_oracle.py on {cores} host threads: 1 warm-up, median of {runs} timed runs "
                      f"({med:.1f} s per batch)"}


if __name__ == "__main__":
    main()
