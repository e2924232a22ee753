"""Evaluation harness on the CPU: the oracle (oracle/semseg_eval.py, a restatement of
plain_train_net.py:107-197) against a hand-computed known answer, the product's host-side
metrics against the oracle, and the rank reduction of confusion matrices over gloo."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cat_seg.evaluation import reduce_confusion, semseg_metrics
from oracle import semseg_eval as OE


def test_oracle_known_answer():
    # 2 classes + ignore; 3x3 image
    gt = np.array([[0, 0, 1], [1, 1, 255], [0, 1, 255]])
    pred_lbl = np.array([[0, 1, 1], [1, 0, 0], [0, 1, 1]])
    probs = np.stack([(pred_lbl == 0), (pred_lbl == 1)]).astype(np.float32)
    conf = np.zeros((3, 3), np.int64)
    OE.confusion_update(conf, probs, gt, 2, 255)
    # conf[pred][gt]
    assert conf.tolist() == [[2, 1, 1], [1, 3, 1], [0, 0, 0]]
    m = OE.metrics(conf, ["a", "b"])
    # class a: tp 2, gt 3, pred 3 -> IoU 2/4; class b: tp 3, gt 4, pred 4 -> IoU 3/5
    assert math.isclose(m["IoU-a"], 50.0) and math.isclose(m["IoU-b"], 60.0)
    assert math.isclose(m["mIoU"], 55.0)
    assert math.isclose(m["pACC"], 100 * 5 / 7)
    assert math.isclose(m["mACC"], 100 * (2 / 3 + 3 / 4) / 2)
    assert math.isclose(m["fwIoU"], 50 * 3 / 7 + 60 * 4 / 7)
    # VOC-b fold: predictions >= 1 become 1
    conf2 = np.zeros((3, 3), np.int64)
    OE.confusion_update(conf2, np.stack([probs[0] * 0, probs[0], probs[1]]).astype(np.float32), gt, 2, 255,
                        clamp_pred=1)
    assert conf2[1].sum() == 9 and conf2[0].sum() == 0


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = float(a[k]), float(b[k])
        assert (math.isnan(x) and math.isnan(y)) or math.isclose(x, y, rel_tol=1e-12, abs_tol=1e-12), (k, x, y)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_product_metrics_match_oracle(seed):
    rng = np.random.default_rng(seed)
    n = 12
    conf = rng.integers(0, 50, size=(n + 1, n + 1)).astype(np.int64)
    conf[:, 3] = 0                       # a class absent from the ground truth
    conf[5, :] = 0                       # a class never predicted
    names = [f"c{i}" for i in range(n)]
    _same(semseg_metrics(conf, names), OE.metrics(conf, names))
    extra = names[::3]
    _same(semseg_metrics(conf, names, extra), OE.metrics(conf, names, extra))


def test_product_metrics_rejects_bad_shape():
    with pytest.raises(ValueError):
        semseg_metrics(np.zeros((4, 4), np.int64), ["a", "b"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    conf = torch.arange(9, dtype=torch.int64) * (rank + 1)
    q.put((rank, reduce_confusion(conf).tolist()))
    dist.destroy_process_group()


def test_reduce_confusion_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    expect = [3 * i for i in range(9)]
    assert got[0] == expect and got[1] == expect
