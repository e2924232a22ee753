"""Benchmark: CAT-Seg dense inference, images/sec @ ViT-L/14 336², 150 classes, bs=8 per GPU.

  python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = the full eval forward of one batch of synthetic images already resident in HBM:
CLIP-normalize / pad / resize -> CLIP ViT dense encoder -> cost volume -> 2 aggregation
layers -> guided upsampler -> sigmoid logits bilinearly upsampled to the CLIP resolution
(cat_seg_model.py:147-229).  Class embeddings of the dataset's prompts are encoded once on
the GPU before timing (the predictor's eval cache, cat_seg_predictor.py:191-192).  With
N > 1 each rank runs its own batch and the (B, T, 96, 96) logits are all-gathered over RCCL
(weak scaling); after timing, rank 0 re-runs every rank's seeded batch and checks that the
gathered logits equal its own, bit for bit (the multi-GPU parity gate).

Configs: 3 = the headline (L/14@336, T=150, bs=8, bf16); 2 = B/16@384, T=150,
bs=4, fp32 (exact-f32 MFMA); 4 = L/14@336, ade847 -> top-256, 4 images/GPU; 5 = sliding-window
640², pc459, fp8 ViT GEMMs.

Prints ONE JSON line (rank 0) with the metric, a roofline object for the dominant kernel
(HIP-event timed per launch on the launch stream, algorithmic FLOPs from the launch shapes)
and the CPU baseline (the oracle, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cat-seg_amd"))
sys.path.insert(0, ROOT)

from cat_seg import ops  # noqa: E402
from cat_seg import _lib as L  # noqa: E402
from cat_seg.distributed import gather_logits, gather_logits_async, init_distributed  # noqa: E402
from cat_seg.arch import VIT_B16, VIT_L14_336  # noqa: E402
from cat_seg.engine import CatSegEngine  # noqa: E402
from cat_seg.weights import synthesize_state_dict  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3       # exact-f32 MFMA = the f32 vector rate
PEAK_FP8_TFLOPS = 5000.0      # MI355X dense fp8 MFMA (block-scaled K=128 form)
PEAK_HBM_GBS = 8000.0

# reference eval-forward FLOPs per image (torch FlopCounter, text excluded)
CONFIGS = {
    2: dict(arch=VIT_B16, T=150, B=4, dtype="f32", gf=602.3, tokens="ade150",
            metric="images/sec @ ViT-B/16 384², 150 classes, bs=4, fp32 (SURVEY §8 config 2; not the headline)"),
    3: dict(arch=VIT_L14_336, T=150, B=8, dtype="bf16", gf=875.7, tokens="ade150",
            metric="images/sec @ ViT-L/14 336², 150 classes, bs=8; 1/2/4/8-GPU scaling"),
    4: dict(arch=VIT_L14_336, T=847, B=4, dtype="bf16", gf=1128.0, tokens="ade847",
            metric="images/sec @ ViT-L/14 336², 847 classes (top-256), 4 images/GPU "
                   "(SURVEY §8 config 4; not the headline)"),
    5: dict(arch=VIT_L14_336, T=459, B=8, dtype="bf16", gf=5638.1, tokens="pc459", fp8=True,
            metric="images/sec @ ViT-L/14 sliding-window 640² (5 crops/image), 459 classes, fp8 ViT GEMMs "
                   "(SURVEY §8 config 5; not the headline)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (0 = the config's)")
    ap.add_argument("--classes", type=int, default=0, help="class count (0 = the config's)")
    ap.add_argument("--dtype", default="", choices=["", "bf16", "f32"], help="engine dtype ('' = the config's)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one hipGraph per step")
    ap.add_argument("--cpu-images", type=int, default=-1,
                    help="oracle sample size for cpu_baseline (-1 = the benched batch, 0 = skip)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-boundary", action="store_true",
                    help="skip the drop-in boundary leg (CATSeg.forward(list[dict]) on host uint8 images)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend for N > 1: nccl (= RCCL) when every rank has its own GPU, "
                         "gloo (logits staged through the host) to rehearse N ranks on fewer GPUs")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds before a rendezvous or collective that has not completed fails the run (N > 1)")
    ap.add_argument("--vit-fp8", action="store_true",
                    help="e4m3 CLIP image-encoder GEMMs (config 5's setting) on another config")
    ap.add_argument("--attention-type", default="linear", choices=["linear", "full"],
                    help="MODEL.SEM_SEG_HEAD.ATTENTION_TYPE of the class aggregation (model.py:331-334)")
    ap.add_argument("--prompt-length", type=int, default=0,
                    help="visual prompt tuning: PROMPT_LENGTH tokens in every vision block (PROMPT_DEPTH = layers)")
    return ap.parse_args()


def class_tokens(name, T):
    g = np.load(os.path.join(ROOT, "tests", "golden", "class_tokens.npz"))
    return torch.from_numpy(g[name][:T].astype(np.int32))


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


def synthetic_batch(rank, B, S, dev):
    """Rank r's seeded images: rand*255 on an S² canvas padded to /32, valid size S x S."""
    gen = torch.Generator().manual_seed(1234 + rank)
    pad = (S + 31) // 32 * 32
    raw = torch.zeros(B, 3, pad, pad)
    raw[:, :, :S, :S] = torch.rand(B, 3, S, S, generator=gen) * 255
    return raw.to(dev)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: the ranks must match the GPUs asked for")
    n_dev = torch.cuda.device_count()
    if n_dev == 0:
        raise SystemExit("bench.py needs a visible MI355X")
    dev = torch.device("cuda", local % n_dev)
    torch.cuda.set_device(dev)
    backend = args.backend
    if world > 1:
        if backend == "auto":
            backend = "nccl" if n_dev >= world else "gloo"
        # bounded: a missing rank or a stuck collective exits non-zero after --dist-timeout seconds
        init_distributed(backend, timeout_s=args.dist_timeout, device=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, expected {args.gpus}")
    cfg = CONFIGS[args.config]
    cfg5 = args.config == 5
    arch = cfg["arch"]
    # the optional heads (not the reference configs' settings): a variant of the config, named in the line
    variant = []
    if args.attention_type != "linear":
        arch = arch.replace(attention_type=args.attention_type)
        variant.append(f"ATTENTION_TYPE {args.attention_type}")
    if args.prompt_length:
        arch = arch.replace(prompt_depth=arch.vision_layers, prompt_length=args.prompt_length)
        variant.append(f"visual prompts {args.prompt_length} x {arch.vision_layers} layers")
    B = args.batch or cfg["B"]
    T = args.classes or cfg["T"]
    dname = args.dtype or cfg["dtype"]
    dtype = torch.bfloat16 if dname == "bf16" else torch.float32
    vit_fp8 = bool(cfg.get("fp8")) or args.vit_fp8
    R = arch.clip_resolution

    sd = synthesize_state_dict(arch, seed=0)
    eng = CatSegEngine(arch, sd, dtype=dtype, device=dev, vit_fp8=vit_fp8)
    with torch.no_grad():
        text = eng.encode_text(class_tokens(cfg["tokens"], T))
        eng.set_text(text)
    S = 640 if cfg5 else R          # config 5: 640² images through the sliding-window branch
    raw = synthetic_batch(rank, B, S, dev)
    sizes = torch.tensor([[S, S]] * B, dtype=torch.int32, device=dev)
    out = None if cfg5 else torch.empty(B, T, R, R, device=dev)
    gsize = 4 * arch.grid
    rows = 5 * B if cfg5 else B          # gathered logit planes per rank (config 5: 4 tiles + global per image)

    def step():
        if cfg5:
            # crops + head + Fold merge -> 640² probabilities at the image size (sem_seg_postprocess is the
            # identity at 640²); the crops' logits (5 per image, 96²) are what N > 1 all-gathers
            _, crop_logits = eng.sliding_logits(raw, sizes, return_crops=True)
            return crop_logits
        logits = eng.head_logits(raw, sizes)
        ops.postprocess(logits, out, crop=(min(logits.shape[-2], R), min(logits.shape[-1], R)))
        return logits

    # One compute stream carries the whole step (input copies, graph replays, eager launches).  With
    # N > 1 the forward is captured twice (two graphs, each with its own logits buffer) and step i
    # replays graph i % 2; over RCCL the logits all-gather of step i runs on the collective's own
    # stream, after that replay and overlapped with step i+1's forward, and the replay of step i+2
    # waits for gather i (which reads the buffer it rewrites).  gloo stages through the host and
    # gathers synchronously after each step (same buffer ring, no overlap).
    stream = torch.cuda.Stream(device=dev)
    overlap = world > 1 and backend == "nccl"
    nbuf = 2 if world > 1 else 1
    graphs, g_logits = [], []
    gathered = ([torch.empty(world * rows, T, gsize, gsize, device=dev) for _ in range(nbuf)]
                if world > 1 else None)
    works = [None] * nbuf
    torch.cuda.synchronize()
    with torch.no_grad(), torch.cuda.stream(stream):
        if not args.no_graph:
            step()                # allocate / warm the caching allocator outside capture
            torch.cuda.synchronize()
            for _ in range(nbuf):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    g_logits.append(step())
                graphs.append(g)

        def forward_once(i=0):
            """Step i's forward on `stream` (the current stream inside run / the parity gate)."""
            if graphs:
                graphs[i % nbuf].replay()
                return g_logits[i % nbuf]
            return step()

        def run(i):
            k = i % nbuf
            if works[k] is not None:
                works[k].wait()                    # gather i-2 has read the buffer this replay rewrites
                works[k] = None
            lg = forward_once(i)
            if world > 1:
                works[k] = gather_logits_async(lg, gathered[k])   # RCCL all-gather over xGMI
            return lg

        for i in range(args.warmup):
            run(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            run(args.warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        last = (args.warmup + args.steps - 1) % nbuf
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64)
            t = t.to(dev) if backend == "nccl" else t
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = t.item()
        # multi-GPU parity gate: rank 0 recomputes every rank's seeded batch on its own GPU and
        # compares with that rank's slice of the last step's gathered logits, bit for bit
        gather_ok = None
        if world > 1:
            ok = True
            if rank == 0:
                ref = gathered[last].clone()
                for r in range(world):
                    raw.copy_(synthetic_batch(r, B, S, dev))
                    lg = forward_once(last)
                    torch.cuda.synchronize()
                    ok = ok and torch.equal(ref[r * rows:(r + 1) * rows], lg)
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            flag = flag.to(dev) if backend == "nccl" else flag
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            gather_ok = bool(flag.item())
            raw.copy_(synthetic_batch(rank, B, S, dev))
            torch.cuda.synchronize()
    images = world * B * args.steps
    value = images / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    boundary = None
    if rank == 0 and world == 1 and not cfg5 and not args.no_boundary and args.config == 3 and not variant:
        boundary = boundary_pass(cfg, B, S, T, args.steps, args.warmup, value)
    roofline, kernels = None, None
    if rank == 0 and not args.no_roofline:
        roofline, kernels = roofline_pass(step, stream, dtype, vit_fp8, args.config)
    cpu = None
    n_cpu = B if args.cpu_images < 0 else args.cpu_images
    if rank == 0 and world == 1 and n_cpu > 0:
        cpu = (cpu_baseline_sliding(arch, sd, text.cpu()) if cfg5 else
               cpu_baseline(arch, sd, text.cpu(), n_cpu))
    if rank == 0:
        path_peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
        path_tflops = cfg["gf"] * value / 1e3
        line = {
            "metric": cfg["metric"],
            "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "ranks": world,
            "backend": backend if world > 1 else None,
            "gather_matches_1gpu": gather_ok,
            "dtype": dname + ("+fp8e4m3 ViT GEMMs" if vit_fp8 else ""),
            "data": "synthetic (seeded rand*255 images, deterministic synthetic weights, "
                    f"{cfg['tokens']} prompt tokens)",
            "config": {"workload": (f"CATSeg eval forward, TEST.SLIDING_WINDOW: {B} images/GPU of 640², "
                                    f"{5 * B} crops through ViT-L/14@336, T={T} (top-256 per crop), "
                                    "Fold/avg merge to 640² probabilities" if cfg5 else
                                    f"CATSeg eval forward {arch.name}, T={T} classes, bs={B}/GPU, "
                                    f"POOLING [1,1], sigmoid upsampled to {R}x{R}"
                                    + "".join(f", {v}" for v in variant)),
                       "bench_config": args.config,
                       "global_batch": world * B, "classes": T, "resolution": R,
                       "parallelism": f"batch-shard x{world} + {backend} all-gather of logits" if world > 1 else "1 GPU",
                       "hipgraph": bool(graphs),
                       "gather_overlap": overlap if world > 1 else None},
            "roofline": roofline,
            "boundary": boundary,
            # the whole path's fraction of the dtype's dense peak; None with fp8 ViT GEMMs (a mix of
            # fp8 and bf16 work has no single roof)
            "path_roofline": None if vit_fp8 or variant else {
                "bound": "mfma", "achieved": round(path_tflops, 2), "peak": path_peak,
                "unit": "TFLOP/s", "gf_per_image": cfg["gf"], "frac": round(path_tflops / path_peak, 4)},
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def boundary_pass(cfg, B, S, T, steps, warmup, engine_value):
    """The reference's call shape (cat_seg_model.py:147-229, detectron2's inference loop): build_model(cfg)
    -> CATSeg.forward(list[{"image": uint8 (3, S, S) HOST tensor}]) -> list[{"sem_seg": (T, S, S)}], timed
    over three rounds of the engine leg's step count (the median round is reported).  Each call stages
    the host images through the model's reused pinned canvas (one H2D copy of the uint8 bytes and the
    fp32 conversion on the compute stream), replays the forward's hipGraph and returns every image's
    probabilities as fresh device tensors."""
    from cat_seg import add_cat_seg_config, build_model, get_cfg
    c = get_cfg()
    add_cat_seg_config(c)
    c.merge_from_file(os.path.join(ROOT, "cat-seg_amd", "configs", "vitl_336.yaml"))
    c.merge_from_list(["MODEL.SEM_SEG_HEAD.POOLING_SIZES", "[1,1]", "MODEL.CATSEG_HIP.DTYPE", "bf16"])
    model = build_model(c).cuda().eval()
    model.sem_seg_head.predictor.set_class_tokens(class_tokens(cfg["tokens"], T))
    gen = torch.Generator().manual_seed(4321)
    batch = [{"image": (torch.rand(3, S, S, generator=gen) * 255).to(torch.uint8)} for _ in range(B)]
    rounds = []
    with torch.no_grad():
        for _ in range(max(warmup, 3)):        # the first call captures the graph, allocates the slots
            out = model(batch)
        torch.cuda.synchronize()
        for _ in range(3):                     # three timed rounds of `steps` calls: the median round
            t0 = time.perf_counter()
            for _ in range(steps):
                out = model(batch)
            torch.cuda.synchronize()
            rounds.append(time.perf_counter() - t0)
    assert len(out) == B and tuple(out[0]["sem_seg"].shape) == (T, S, S)
    el = sorted(rounds)[1]
    v = B * steps / el
    res = {"value": round(v, 3), "unit": "images/s", "ms_per_step": round(el / steps * 1e3, 3),
           "ms_per_step_rounds": [round(r / steps * 1e3, 3) for r in rounds],
           "vs_engine": round(v / engine_value, 4),
           "call": "build_model(cfg) -> CATSeg.forward(list[{'image': uint8 (3,336,336) host tensor}]) -> "
                   f"{B} x {{'sem_seg': fp32 ({T},336,336) device tensor}}",
           "staging": "reused pinned uint8 canvas (two slots), one H2D copy and the fp32 conversion on the compute stream, hipGraph replay"}
    del model
    torch.cuda.empty_cache()
    return res


def lib_sha16() -> str:
    """Identity of the kernel build this process runs: sha256 of libcatseg_hip.so, 16 hex."""
    with open(L.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _version_key(path):
    """profiles/r03/v12/pmc_traffic.json -> (3, 12): numeric, so v10 sorts after v9."""
    nums = [int(n) for part in os.path.relpath(path, ROOT).split(os.sep) for n in re.findall(r"\d+", part)]
    return tuple(nums)


def pmc_traffic(family, bench_config=3):
    """HBM bytes per launch of `family` from a committed PMC summary (profiles/**/pmc_traffic.json,
    written by tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes;
    FETCH_SIZE doubled per the gfx950 note).  Only summaries taken on the same bench configuration
    count (tools/pmc_step.py runs the headline, config 3: a config-4 GEMM at M = 2308 moves other
    bytes than the headline's at M = 4616).  Prefers the newest summary recorded for this exact
    kernel build (lib_sha16 of the loaded libcatseg_hip.so), else the newest by round / version
    number.  Returns (bytes, source, same_build)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_traffic.json"), recursive=True),
                   key=_version_key)
    if not files:
        return None, None, False
    sha = lib_sha16()
    docs = [(f, json.load(open(f))) for f in files]
    docs = [(f, d) for f, d in docs if d.get("bench_config", 3) == bench_config]
    if not docs:
        return None, None, False
    same = [(f, d) for f, d in docs if d.get("lib_sha16") == sha]
    f, d = (same or docs)[-1]
    fam = d["families"].get(family)
    if fam is None:
        return None, os.path.relpath(f, ROOT), bool(same)
    return fam["traffic_bytes_per_launch"], os.path.relpath(f, ROOT), bool(same)


def _queued_profile(step, stream):
    """The eager step with HIP events around every wrapped launch, timed from a full queue.

    Events around an eager launch also measure the host's time to enqueue it (Python + ctypes,
    10-30 us) whenever the GPU runs ahead of the host -- a 10 us kernel can read 25 us.  So a first
    pass measures the host's enqueue time of the whole step, and the recorded pass is enqueued behind
    a spin kernel (torch.cuda._sleep) that holds the stream for about twice that long: the launches
    then run back to back exactly as in the replayed graph, and every event pair brackets GPU time
    only; one unrecorded step runs first, so the recorded one starts from full clocks and warm caches.
    Returns (records, timing note, gap fraction: idle share of the recorded span)."""
    ops.PROFILE = []
    with torch.no_grad(), torch.cuda.stream(stream):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        host_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    recs, ops.PROFILE = ops.PROFILE, None
    note = "eager, host-paced"
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            torch.cuda._sleep(2_000_000)
            e1.record(stream)
        torch.cuda.synchronize()
        cyc_per_ms = 2_000_000 / max(e0.elapsed_time(e1), 1e-3)
        # behind the spin: one unrecorded step (the GPU leaves the idle-ish spin at full clocks and warm
        # caches, as in a run of back-to-back steps), then the recorded one
        spin_ms = 4e3 * host_s + 20.0
        with torch.no_grad(), torch.cuda.stream(stream):
            torch.cuda._sleep(int(cyc_per_ms * spin_ms))
            step()
            ops.PROFILE = []
            step()
        torch.cuda.synchronize()
        recs, ops.PROFILE = ops.PROFILE, None
        note = (f"queued behind a {spin_ms:.0f} ms spin kernel and one unrecorded step "
                f"(host enqueue {host_s * 1e3:.0f} ms per step)")
    busy = sum(r["start"].elapsed_time(r["end"]) for r in recs)
    span = recs[0]["start"].elapsed_time(recs[-1]["end"]) if recs else 0.0
    return recs, note, (round(1.0 - busy / span, 4) if span > 0 else None)


def roofline_pass(step, stream, dtype, vit_fp8=False, bench_config=3):
    """One eager pass with HIP events around every wrapped launch (on the launch stream), enqueued
    behind a spin kernel so that the events bracket GPU time only (_queued_profile)."""
    recs, timing, gap = _queued_profile(step, stream)
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
    traffic, tsrc, tsame = pmc_traffic(top, bench_config)
    common = {"launches": a["launches"], "avg_launch_us": round(avg_s * 1e6, 2), "traffic": traffic,
              "traffic_source": tsrc, "traffic_same_build": tsame, "lib_sha16": lib_sha16(),
              "timing": timing, "idle_frac_of_span": gap}
    if a["flops"] > 0:
        achieved = a["flops"] / a["launches"] / avg_s / 1e12
        peak = (PEAK_FP8_TFLOPS if top == "gemm_fp8" else
                PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS)
        roof = {"bound": "mfma", "kernel": top, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), **common,
                "flops_per_launch": a["flops"] // a["launches"],
                "algorithmic_bytes_per_launch": a["bytes"] // a["launches"]}
    else:
        achieved = a["bytes"] / a["launches"] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": top, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), **common}
    # tflops: executed work / time; ref_tflops: the reference's count for the module / time
    # (differs where the build skips padding rows, per-class guidance halves or ConvT maps).
    # Per family the floor: floor_ms = max(executed flops / the dtype's dense MFMA peak, algorithmic
    # bytes / 8 TB/s) and floor_frac = floor_ms / ms (1.0 = at the roof); traffic_mb_per_launch from the
    # newest same-config PMC summary (tools/pmc_traffic.py) where one exists for the family.
    kern = {}
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
        e = {"launches": v["launches"], "ms": round(v["ms"], 3)}
        if v["flops"]:
            e["tflops"] = round(v["flops"] / (v["ms"] / 1e3) / 1e12, 2)
            if v["ref_flops"] != v["flops"]:
                e["ref_tflops"] = round(v["ref_flops"] / (v["ms"] / 1e3) / 1e12, 2)
        if v["bytes"]:
            e["gbs"] = round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1)
        peak = (PEAK_FP8_TFLOPS if k == "gemm_fp8" else PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else
                PEAK_F32_TFLOPS)
        floor_s = max(v["flops"] / (peak * 1e12), v["bytes"] / (PEAK_HBM_GBS * 1e9))
        e["gflop"] = round(v["flops"] / 1e9, 3)
        e["algorithmic_mb"] = round(v["bytes"] / 1e6, 3)
        e["floor_ms"] = round(floor_s * 1e3, 4)
        e["floor_frac"] = round(floor_s * 1e3 / v["ms"], 4) if v["ms"] > 0 else None
        e["floor_bound"] = "mfma" if v["flops"] / (peak * 1e12) >= v["bytes"] / (PEAK_HBM_GBS * 1e9) else "hbm"
        t, _, _ = pmc_traffic(k, bench_config)
        if t:
            e["traffic_mb_per_launch"] = round(t / 1e6, 3)
        kern[k] = e
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


def _cpu_line(n_images, ts, cores, runs, sample):
    """images/s of the median run; spread = [slowest, fastest] run in images/s."""
    med = float(np.median(ts))
    return {"value": round(n_images / med, 4), "unit": "images/s", "cores": cores, "kind": "port", "runs": runs,
            "spread_images_per_s": [round(n_images / max(ts), 4), round(n_images / min(ts), 4)],
            "seconds_per_run": round(med, 2), "sample": sample}


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
    return _cpu_line(1, ts, cores, runs,
                     f"1 image of the same workload (640² sliding, 5 crops, L/14@336, T={text.shape[0]}, fp32) "
                     f"through oracle/catseg_oracle.py on {cores} host threads: 1 warm-up, median of {runs} runs")


def cpu_baseline(arch, sd, text, n_images, runs=3):
    """The oracle (CPU fp32 restatement of the reference path) on a bounded sample of the same
    workload: one batch of `n_images` (the benched per-GPU batch), 1 warm-up image, the median
    of `runs` timed runs."""
    from oracle import catseg_oracle as O

    cores = host_cores()
    torch.set_num_threads(cores)
    gen = torch.Generator().manual_seed(99)
    R = arch.clip_resolution
    inputs = [{"image": torch.rand(3, R, R, generator=gen) * 255} for _ in range(n_images)]
    O.catseg_forward(arch, sd, inputs[:1], text.unsqueeze(1))     # warm-up
    ts = _timed_runs(lambda: O.catseg_forward(arch, sd, inputs, text.unsqueeze(1), all_images=True), runs)
    return _cpu_line(n_images, ts, cores, runs,
                     f"batches of {n_images} images of the same workload ({arch.name}, T={text.shape[0]}, fp32) "
                     f"through oracle/catseg_oracle.py on {cores} host threads: 1 warm-up, median of {runs} "
                     f"timed runs")


if __name__ == "__main__":
    main()
