"""Batch-sharded inference across the GPUs of one node.

Images are independent, so the only exchange is one all-gather of the per-image
logits.  This restates, for the MI355X path, what the reference gets from detectron2's
eval loop: `InferenceSampler` hands every rank a contiguous slice of the dataset
(detectron2 `data/samplers/distributed_sampler.py`, used via `build_detection_test_loader`
in `train_net.py:124-149`), each rank runs `model(inputs)` on its slice, and results are
combined with `comm.all_gather` (`plain_train_net.py:136-146`, over gloo there).

Here the gather moves the pre-upsample logits (B, T, 96, 96) fp32 — 5.5 MB per image at
T=150 — with one `all_gather_into_tensor` on the process group's backend: RCCL over
xGMI on the GPU box (backend "nccl" is RCCL on ROCm), gloo in the CPU tests.  The
gathered tensor is a pure copy of every rank's logits (bit-identical to running the
same shard alone).  Ragged shards (global batch not divisible by the world size) are
padded to the largest shard for the collective and trimmed afterwards.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_sizes(n: int, world: int) -> List[int]:
    """InferenceSampler's split: the first n % world ranks take one extra item."""
    base, left = divmod(n, world)
    return [base + int(r < left) for r in range(world)]


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """[begin, end) of rank's contiguous slice of n items."""
    sizes = shard_sizes(n, world)
    begin = sum(sizes[:rank])
    return begin, begin + sizes[rank]


DEFAULT_TIMEOUT_S = 300.0


def init_distributed(backend: str, timeout_s: float = DEFAULT_TIMEOUT_S, device=None) -> None:
    """torch.distributed.init_process_group from the launcher's environment (RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT) with a BOUNDED timeout, so that a missing rank or a stuck first
    collective ends the process with an error instead of hanging for the default 10 minutes (30 for
    gloo): the rendezvous raises after `timeout_s`, and on RCCL the watchdog aborts a collective
    that has not completed within it (TORCH_NCCL_ASYNC_ERROR_HANDLING, on unless the caller
    disabled it)."""
    import datetime
    kw = {"timeout": datetime.timedelta(seconds=float(timeout_s))}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)


def _world(group) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def gather_logits(local: torch.Tensor, n_total: int, group=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """All-gather per-rank logits (b_r, ...) into (n_total, ...) on every rank, rank order.

    One collective of max(b_r) rows per rank; `out` may be preallocated (hipGraph-friendly
    callers reuse it).  With world size 1 this is the identity."""
    rank, world = _world(group)
    if world == 1:
        return local
    sizes = shard_sizes(n_total, world)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank}: local batch {local.shape[0]} != shard size {sizes[rank]}")
    bmax = max(sizes)
    rest = tuple(local.shape[1:])
    if local.shape[0] != bmax:      # ragged: pad this rank's block to the common size
        padded = local.new_zeros((bmax,) + rest)
        padded[:local.shape[0]] = local
        local = padded
    even = all(s == bmax for s in sizes)
    buf = out if (even and out is not None) else local.new_empty((world * bmax,) + rest)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device all-gather: stage through the host (rehearsing N ranks on fewer GPUs)
        hbuf = torch.empty(buf.shape, dtype=buf.dtype)
        dist.all_gather_into_tensor(hbuf, local.cpu().contiguous(), group=group)
        buf.copy_(hbuf)
    else:
        dist.all_gather_into_tensor(buf, local.contiguous(), group=group)
    if even:
        return buf
    if out is None:
        out = local.new_empty((n_total,) + rest)
    o = 0
    for r, s in enumerate(sizes):
        out[o:o + s] = buf[r * bmax:r * bmax + s]
        o += s
    return out


def gather_logits_async(local: torch.Tensor, out: torch.Tensor, group=None):
    """Start the all-gather of equal-size per-rank logits into `out` (world * b rows, rank order)
    and return its work handle, or None when it completed synchronously.

    On a device backend (RCCL) the collective runs on its own stream: it starts after the work
    already queued on the caller's current stream (which produces `local`), and `work.wait()` makes
    the caller's current stream wait for it (before anything rewrites `local` or reads `out`).
    gloo has no device all-gather: the host-staged gather_logits runs synchronously instead."""
    rank, world = _world(group)
    if out.shape[0] != world * local.shape[0] or out.shape[1:] != local.shape[1:]:
        raise ValueError(f"gather_logits_async: out {tuple(out.shape)} is not world={world} x {tuple(local.shape)}")
    if world == 1:
        out.copy_(local)
        return None
    if local.is_cuda and dist.get_backend(group) == "gloo":
        gather_logits(local, out.shape[0], group=group, out=out)
        return None
    return dist.all_gather_into_tensor(out, local.contiguous(), group=group, async_op=True)


def allreduce_gradients(params, group=None, bucket_mb: float = 64.0) -> int:
    """Data-parallel gradient averaging of the training step (what DistributedDataParallel does for
    train_net.py's `Trainer`, train_net.py:309-311 / detectron2 create_ddp_model): the `.grad` of every
    parameter that has one, flattened into fp32 buckets of <= bucket_mb, one all_reduce(SUM) per bucket
    (RCCL over xGMI on the GPU box; gloo stages device buckets through the host), divided by the world
    size and copied back.  Every rank must reduce the SAME buckets even when ranks produced gradients
    for different parameters (an unused branch on one rank): one small all_reduce(MAX) of the per-
    parameter "has a gradient" flags comes first; a parameter with a gradient on ANY rank is reduced
    everywhere (zeros where this rank has none, as DDP's unused-parameter path), one with a gradient on
    no rank keeps `.grad = None`.  Buckets are filled in parameter order.  Returns the number of
    collectives issued (0 at world size 1)."""
    rank, world = _world(group)
    if world == 1:
        return 0
    ps = [p for p in params if p.requires_grad]
    if not ps:
        return 0
    dev = ps[0].device
    staged = dev.type == "cuda" and dist.get_backend(group) == "gloo"
    has = torch.tensor([p.grad is not None for p in ps], dtype=torch.int32, device="cpu" if staged else dev)
    dist.all_reduce(has, op=dist.ReduceOp.MAX, group=group)
    used = has.tolist()
    for p, u in zip(ps, used):
        if u and p.grad is None:
            p.grad = torch.zeros_like(p)
    grads = [p.grad for p, u in zip(ps, used) if u]
    if not grads:
        return 1
    limit = max(1, int(bucket_mb * (1 << 20)) // 4)
    buckets, cur, n = [], [], 0
    for g in grads:
        if cur and n + g.numel() > limit:
            buckets.append(cur)
            cur, n = [], 0
        cur.append(g)
        n += g.numel()
    buckets.append(cur)
    for b in buckets:
        flat = torch.cat([g.reshape(-1).float() for g in b])
        if flat.is_cuda and dist.get_backend(group) == "gloo":
            h = flat.cpu()
            dist.all_reduce(h, group=group)
            flat.copy_(h)
        else:
            dist.all_reduce(flat, group=group)
        flat.div_(world)
        o = 0
        for g in b:
            g.copy_(flat[o:o + g.numel()].view_as(g))
            o += g.numel()
    return 1 + len(buckets)


def create_ddp_model(model: torch.nn.Module, **kwargs) -> torch.nn.Module:
    """detectron2 create_ddp_model as train_net.py's Trainer uses it: torch DistributedDataParallel around
    the model when the world size is > 1 (gradients all-reduced in buckets during backward), else the
    model itself.  The CAT-Seg parameters are plain nn.Parameters whose gradients come from the HIP
    autograd Functions, so DDP's gradient hooks see them like any module's."""
    _, world = _world(None)
    if world == 1:
        return model
    from torch.nn.parallel import DistributedDataParallel
    dev = next(model.parameters()).device
    if dev.type == "cuda":
        kwargs.setdefault("device_ids", [dev.index if dev.index is not None else torch.cuda.current_device()])
    kwargs.setdefault("broadcast_buffers", False)
    return DistributedDataParallel(model, **kwargs)


def run_sharded(forward: Callable[[Sequence], torch.Tensor], items: Sequence, group=None) -> torch.Tensor:
    """Run `forward` on this rank's slice of `items` and all-gather the results.

    `forward(slice) -> Tensor (len(slice), ...)`; every rank returns the full (len(items), ...)."""
    rank, world = _world(group)
    b, e = shard_range(len(items), rank, world)
    local = forward(items[b:e])
    return gather_logits(local, len(items), group=group)
