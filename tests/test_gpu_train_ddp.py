"""Data-parallel training step on the device (train_net.py:298-311: Trainer = DDP over the ranks'
batches): two ranks (gloo, both on GPU 0 — the 8-GPU RCCL run is the driver's) each run the CATSeg
training step on their own images; after backward every rank's gradients equal the mean of the two
single-process gradients, through torch DistributedDataParallel (cat_seg.distributed.create_ddp_model)
and through the explicit bucketed all-reduce (cat_seg.distributed.allreduce_gradients)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_boundary_cpu import tiny_cfg

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from cat_seg import build_model
    m = build_model(tiny_cfg(**{"MODEL.SEM_SEG_HEAD.POOLING_SIZES": "[2,2]"})).cuda().train()
    T = 6
    toks = torch.zeros(T, 16, dtype=torch.long)
    toks[:, 0] = 1
    toks[:, 1:3] = torch.arange(2 * T).reshape(T, 2) + 5
    toks[:, 3] = 511
    m.sem_seg_head.predictor.set_class_tokens(toks)
    return m, T


def _batch(rank, T):
    gen = torch.Generator().manual_seed(70 + rank)
    return [{"image": torch.randint(0, 256, (3, 384, 384), generator=gen).float(),
             "sem_seg": torch.randint(0, T, (384, 384), generator=gen)}]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cat_seg.distributed import allreduce_gradients, create_ddp_model
        m, T = _model()
        ddp = create_ddp_model(m)
        assert ddp is not m
        ddp(_batch(rank, T))["loss_sem_seg"].backward()
        g_ddp = {k: p.grad.cpu() for k, p in m.named_parameters() if p.grad is not None}
        m.zero_grad(set_to_none=True)
        m(_batch(rank, T))["loss_sem_seg"].backward()
        allreduce_gradients(m.parameters(), bucket_mb=1.0)
        g_ar = {k: p.grad.cpu() for k, p in m.named_parameters() if p.grad is not None}
        torch.save({"ddp": g_ddp, "ar": g_ar}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_data_parallel_training_gradients():
    singles = []
    for rank in range(2):
        m, T = _model()
        m(_batch(rank, T))["loss_sem_seg"].backward()
        singles.append({k: p.grad.cpu() for k, p in m.named_parameters() if p.grad is not None})
        del m
    torch.cuda.synchronize()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    keys = list(singles[0])
    assert set(keys) == set(singles[1]) and len(keys) > 100
    for r in range(2):
        for mode in ("ddp", "ar"):
            got = res[r][mode]
            assert set(got) == set(keys), mode
            for k in keys:
                mean = (singles[0][k] + singles[1][k]) / 2
                err = (got[k] - mean).abs().max().item()
                assert err <= 1e-5 * mean.abs().max().item() + 1e-12, (mode, r, k, err)
    # both ranks hold the same averaged gradients
    for k in keys:
        assert torch.equal(res[0]["ar"][k], res[1]["ar"][k])
