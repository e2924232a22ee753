"""Batch-sharded inference over world_size 2 with the gloo backend on CPU.

Each rank computes the logits of its InferenceSampler slice (the oracle stands in for the
per-rank forward: these tests check the shard/gather host logic, not the kernels) and
`cat_seg.distributed` all-gathers them; the result must be a bit-exact copy of the
per-shard logits, in rank order, on every rank — even and ragged global batches.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cat_seg import distributed as D


def test_shard_sizes_match_inference_sampler():
    # detectron2 InferenceSampler._get_local_indices: first n % world ranks get one more
    assert D.shard_sizes(10, 4) == [3, 3, 2, 2]
    assert D.shard_sizes(8, 8) == [1] * 8
    assert D.shard_sizes(3, 4) == [1, 1, 1, 0]
    ranges = [D.shard_range(11, r, 3) for r in range(3)]
    assert ranges == [(0, 4), (4, 8), (8, 11)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_setup():
    from cat_seg.arch import TINY
    from cat_seg.weights import synthesize_state_dict
    arch = TINY
    sd = synthesize_state_dict(arch, seed=0)
    gen = torch.Generator().manual_seed(5)
    text = torch.nn.functional.normalize(torch.randn(6, arch.embed_dim, generator=gen), dim=-1).unsqueeze(1)
    imgs = [torch.rand(3, 384, 384, generator=gen) * 255 for _ in range(3)]
    return arch, sd, text, imgs


def _oracle_forward(arch, sd, text):
    from oracle import catseg_oracle as O

    def fwd(items):
        if len(items) == 0:
            return torch.empty(0, text.shape[0], 4 * arch.grid, 4 * arch.grid)
        clip, _ = O.preprocess(arch, list(items))
        return O.head_logits(arch, sd, clip, text)
    return fwd


def _worker(rank, world, port, n_items, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arch, sd, text, imgs = _tiny_setup()
        with torch.no_grad():
            full = D.run_sharded(_oracle_forward(arch, sd, text), imgs[:n_items])
        torch.save(full, os.path.join(out_dir, f"rank{rank}.pt"))
        # a preallocated output (the hipGraph-friendly form) gives the same bytes
        b, e = D.shard_range(n_items, rank, world)
        local = full[b:e].clone()
        out = torch.empty_like(full)
        D.gather_logits(local, n_items, out=out)
        assert torch.equal(out, full)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_items", [2, 3])     # even and ragged global batch
def test_gloo_world2_gather_is_exact_copy(n_items):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), n_items, d), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    arch, sd, text, imgs = _tiny_setup()
    fwd = _oracle_forward(arch, sd, text)
    torch.set_num_threads(2)
    with torch.no_grad():
        want = torch.cat([fwd(imgs[slice(*D.shard_range(n_items, r, world))]) for r in range(world)])
    assert want.shape[0] == n_items
    for g in got:
        assert torch.equal(g, want)


def _ring_worker(rank, world, port, out_dir):
    """bench.py's N > 1 loop shape on gloo/CPU: a two-buffer ring of per-step logits, each step's
    gather started with gather_logits_async and waited for two steps later (before its buffer is
    rewritten); every gathered block must equal that step's per-rank logits."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = 3
        bufs = [torch.empty(b, 5, 4, 4) for _ in range(2)]
        gathered = [torch.empty(world * b, 5, 4, 4) for _ in range(2)]
        works = [None, None]
        seen = []
        for i in range(5):
            k = i % 2
            if works[k] is not None:
                works[k].wait()
                seen.append(gathered[k].clone())      # step i-2's gather, complete
            bufs[k].copy_(torch.arange(b * 80, dtype=torch.float32).view(b, 5, 4, 4) + 1000 * rank + 10 * i)
            works[k] = D.gather_logits_async(bufs[k], gathered[k])
        for k in (1, 0):                               # steps 3, 4
            if works[k] is not None:
                works[k].wait()
            seen.append(gathered[k].clone())
        torch.save(torch.stack(seen), os.path.join(out_dir, f"ring{rank}.pt"))
        with pytest.raises(ValueError):
            D.gather_logits_async(bufs[0], torch.empty(world * b + 1, 5, 4, 4))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_async_gather_ring():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ring_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, f"ring{r}.pt"), weights_only=True) for r in range(world)]
    base = torch.arange(3 * 80, dtype=torch.float32).view(3, 5, 4, 4)
    want = torch.stack([torch.cat([base + 1000 * r + 10 * i for r in range(world)]) for i in range(5)])
    for g in got:
        assert torch.equal(g, want)


def test_world1_is_identity():
    x = torch.randn(3, 4)
    assert D.gather_logits(x, 3) is x


def _grad_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gen = torch.Generator().manual_seed(100 + rank)
        params = [torch.nn.Parameter(torch.zeros(s)) for s in ((300, 7), (11,), (5, 5, 5), (4096,), (9,))]
        for p in params:
            p.grad = torch.randn(p.shape, generator=gen)
        params[1].grad = None                        # no gradient on any rank: stays untouched
        if rank == 1:
            params[4].grad = None                    # an unused branch on rank 1 only
        n = D.allreduce_gradients(params, bucket_mb=0.01)
        torch.save({"n": n, "grads": [None if p.grad is None else p.grad for p in params]},
                   os.path.join(out_dir, f"g{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_allreduce_gradients_world2_gloo():
    """Data-parallel gradient averaging (the DDP all-reduce of train_net.py:309-311): every rank ends
    with the mean of the ranks' gradients, bucketed (three buckets at 10 KB), parameters without a
    gradient on any rank untouched, one with a gradient on one rank only reduced on both (the same
    buckets on every rank)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_grad_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"g{k}.pt"), weights_only=True) for k in range(2)]
    assert r[0]["n"] == r[1]["n"] >= 2
    for k in range(2):
        expect = []
        for rank in range(2):
            gen = torch.Generator().manual_seed(100 + rank)
            expect.append([torch.randn(s, generator=gen) for s in ((300, 7), (11,), (5, 5, 5), (4096,), (9,))])
        for i in (0, 2, 3):
            mean = (expect[0][i] + expect[1][i]) / 2
            assert torch.allclose(r[k]["grads"][i], mean, atol=1e-6)
        assert r[k]["grads"][1] is None
        # used on rank 0 only: both ranks reduce it (zeros on rank 1) and hold the same mean
        assert torch.allclose(r[k]["grads"][4], expect[0][4] / 2, atol=1e-6)
    assert all(torch.equal(a, b) for a, b in zip(r[0]["grads"][:1], r[1]["grads"][:1]))


def test_missing_rank_fails_fast_not_hang():
    """with a bounded timeout (init_distributed, what bench.py calls at N > 1) a run
    whose second rank never arrives exits non-zero within the timeout instead of hanging."""
    import subprocess
    import sys
    import time
    port = _free_port()
    code = ("import sys; sys.path[:0] = sys.argv[1:3]\n"
            "from cat_seg.distributed import init_distributed\n"
            "init_distributed('gloo', timeout_s=5)\n"
            "print('joined')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="2")
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code, os.path.join(root, "cat-seg_amd"), root], env=env,
                       capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert p.returncode != 0 and "joined" not in p.stdout
    assert took < 60, took
