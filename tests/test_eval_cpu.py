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

from cat_seg.evaluation import SemSegEvaluator, coco_rle_encode, reduce_confusion, semseg_metrics
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


# ---- sem_seg_predictions.json: COCO RLE records (plain_train_net.py:125,139-152,207-228) ----

def _column(counts):
    """an N x 1 mask with the given alternating run lengths (zeros first)"""
    v, out = 0, []
    for c in counts:
        out += [v] * c
        v ^= 1
    return np.array(out, np.uint8)[:, None]


@pytest.mark.parametrize("counts,expect", [([4], "4"), ([0, 1], "01"), ([100], "T3"), ([10, 20, 5], ":d05"),
                                           ([10, 20, 5, 3], ":d05_O"), ([0, 40, 2, 40], "0X120")])
def test_coco_rle_hand_vectors(counts, expect):
    """strings derived by hand from maskApi.c rleToString: 100 -> 'T3' (groups 4 | 0x20, 3); 20 ->
    'd0' (0x10 set, so a second group carries the sign); the fourth count as a delta: 3 - 20 = -17
    -> '_O', 40 - 40 = 0 -> '0'; 40 -> 'X1'."""
    m = _column(counts)
    if counts == [4]:
        m = np.zeros((2, 2), np.uint8)
    got = coco_rle_encode(m)
    assert got == OE.rle_encode(m)
    assert got["counts"] == expect, (got["counts"], expect)
    assert got["size"] == list(m.shape)
    assert np.array_equal(OE.rle_decode(got), m)


@pytest.mark.parametrize("shape,density", [((37, 53), 0.5), ((64, 64), 0.02), ((1, 97), 0.7), ((120, 5), 0.98),
                                           ((16, 16), 0.0), ((16, 16), 1.0)])
def test_coco_rle_matches_loop_restatement(shape, density):
    rng = np.random.default_rng(shape[0] * 7 + int(density * 100))
    m = (rng.random(shape) < density).astype(np.uint8)
    if 0 < density < 1:                 # long runs too, so multi-group and negative deltas occur
        m[: shape[0] // 2, : shape[1] // 3] = 1
    got = coco_rle_encode(m)
    assert got == OE.rle_encode(m)
    assert np.array_equal(OE.rle_decode(got), m)


def test_encode_json_sem_seg_records_and_dataset_ids():
    ev = SemSegEvaluator(None, distributed=False, class_names=list("abcde"), ignore_label=255, device="cpu")
    pred = np.random.default_rng(0).integers(0, 5, (23, 31))
    pred[pred == 3] = 4                                     # label 3 absent: no record
    recs = ev.encode_json_sem_seg(pred, "img.jpg")
    assert recs == OE.sem_seg_records(pred, "img.jpg")
    assert [r["category_id"] for r in recs] == [0, 1, 2, 4]
    ev._contiguous_id_to_dataset_id = {0: 10, 1: 11, 2: 12, 3: 13, 4: 20}
    mapped = ev.encode_json_sem_seg(pred, "img.jpg")
    assert [r["category_id"] for r in mapped] == [10, 11, 12, 20]
    ev._contiguous_id_to_dataset_id = {0: 10}
    with pytest.raises(AssertionError):
        ev.encode_json_sem_seg(pred, "img.jpg")


def _rank_dump(rank, world, port, out_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ev = SemSegEvaluator(None, distributed=True, output_dir=out_dir, class_names=["a", "b", "c"], ignore_label=255,
                         device="cpu")
    ev._conf += torch.arange(16, dtype=torch.int64)         # a non-empty matrix; no device kernel on the CPU
    pred = np.full((4, 6), rank, np.int64)
    pred[0, :2] = 2
    ev._predictions.extend(ev.encode_json_sem_seg(pred, f"img{rank}.jpg"))
    res = ev.evaluate()
    q.put((rank, res is not None))
    dist.destroy_process_group()


def test_predictions_json_gathered_over_ranks(tmp_path):
    """evaluate() with an output_dir gathers every rank's records in rank order and rank 0 writes
    sem_seg_predictions.json (plain_train_net.py:139-152) beside sem_seg_evaluation.pth."""
    import json
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_dump, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert got == {0: True, 1: False}
    recs = json.loads((tmp_path / "sem_seg_predictions.json").read_text())
    expect = []
    for r in range(2):
        pred = np.full((4, 6), r, np.int64)
        pred[0, :2] = 2
        expect += OE.sem_seg_records(pred, f"img{r}.jpg")
    assert recs == expect
    assert (tmp_path / "sem_seg_evaluation.pth").exists()
