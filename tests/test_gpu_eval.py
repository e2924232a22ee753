"""catseg_semseg_confusion and cat_seg.evaluation on the device against the numpy oracle
(oracle/semseg_eval.py): integer confusion matrices bit-exact, metrics equal."""
import math

import numpy as np
import pytest
import torch

from cat_seg import ops
from cat_seg import _lib as L
from cat_seg.evaluation import SemSegEvaluator, SemSegGzeroEvaluator, VOCbEvaluator
from oracle import semseg_eval as OE

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _lib():
    L.require_gpu()


def _case(T, H, W, seed, n_levels=4):
    g = torch.Generator().manual_seed(seed)
    # few distinct levels: many exact ties, so the first-maximum rule is exercised
    probs = torch.randint(0, n_levels, (T, H, W), generator=g).float() / n_levels
    gt = torch.randint(0, T, (H, W), generator=g).int()
    gt[torch.rand(H, W, generator=g) < 0.1] = 255
    return probs, gt


@pytest.mark.parametrize("T,H,W,clamp", [(150, 97, 131, -1), (21, 480, 640, 20), (1, 5, 7, -1), (847, 33, 40, -1)])
def test_confusion_kernel_bit_exact(T, H, W, clamp):
    probs, gt = _case(T, H, W, seed=T + H)
    N = T if clamp < 0 else clamp + 1 if clamp + 1 > T else T
    n1 = N + 1
    conf = torch.zeros(n1 * n1, dtype=torch.int64, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(2):       # accumulates across calls
        ops.semseg_confusion(probs.cuda(), gt.cuda(), conf, bad, num_classes=N, ignore_label=255, clamp_pred=clamp)
    ref = np.zeros((n1, n1), np.int64)
    for _ in range(2):
        OE.confusion_update(ref, probs.numpy(), gt.numpy(), N, 255, clamp_pred=clamp)
    assert int(bad.item()) == 0
    assert np.array_equal(conf.cpu().numpy().reshape(n1, n1), ref)


def test_confusion_kernel_nan_ranks_highest():
    """torch.argmax / numpy argmax rank NaN above every number (the first NaN wins); the kernel
    tests NaN on the bits, whatever float mode evaluate.hip is built with."""
    probs, gt = _case(9, 16, 20, seed=7)
    probs[3, 0, :5] = float("nan")         # NaN at a class index > 0
    probs[5, 1, :] = float("nan")
    probs[2, 1, ::2] = float("nan")        # two NaNs: the first (class 2) wins
    probs[0, 2, :3] = float("nan")         # NaN at class 0
    probs[7, 3, 4] = float("inf")
    probs[8, 3, 4] = float("nan")
    conf = torch.zeros(100, dtype=torch.int64, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    ops.semseg_confusion(probs.cuda(), gt.cuda(), conf, bad, num_classes=9, ignore_label=255)
    ref = OE.confusion_update(np.zeros((10, 10), np.int64), probs.numpy(), gt.numpy(), 9, 255)
    pred = probs.argmax(0)
    assert int(pred[0, 0]) == 3 and int(pred[1, 0]) == 2 and int(pred[1, 1]) == 5 and int(pred[3, 4]) == 8
    assert np.array_equal(conf.cpu().numpy().reshape(10, 10), ref)


def test_confusion_kernel_counts_invalid_labels():
    probs, gt = _case(5, 8, 8, seed=3)
    gt[0, 0] = 7          # not a class, not ignore
    gt[1, 1] = -2
    conf = torch.zeros(36, dtype=torch.int64, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    ops.semseg_confusion(probs.cuda(), gt.cuda(), conf, bad, num_classes=5, ignore_label=255)
    assert int(bad.item()) == 2 and int(conf.sum().item()) == 62


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = float(a[k]), float(b[k])
        assert (math.isnan(x) and math.isnan(y)) or math.isclose(x, y, rel_tol=1e-12), (k, x, y)


@pytest.mark.parametrize("cls", [SemSegEvaluator, SemSegGzeroEvaluator, VOCbEvaluator])
def test_evaluator_matches_oracle(cls):
    T = 21 if cls is VOCbEvaluator else 12
    names = [f"c{i}" for i in range(T)]
    kw = {"val_extra_classes": names[::4]} if cls is SemSegGzeroEvaluator else {}
    ev = cls(None, distributed=False, class_names=names, ignore_label=255, **kw)
    ref = np.zeros((T + 1, T + 1), np.int64)
    inputs, outputs = [], []
    for i in range(3):
        probs, gt = _case(T, 60 + i, 70, seed=10 + i, n_levels=50)
        inputs.append({"sem_seg_gt": gt.numpy()})
        outputs.append({"sem_seg": probs.cuda()})
        OE.confusion_update(ref, probs.numpy(), gt.numpy(), T, 255, clamp_pred=cls.clamp_pred)
    ev.process(inputs[:2], outputs[:2])
    ev.process(inputs[2:], outputs[2:])
    assert np.array_equal(ev.confusion_matrix(), ref)
    got = ev.evaluate()["sem_seg"]
    _same(got, OE.metrics(ref, names, kw.get("val_extra_classes", ())))
    ev.reset()
    assert int(ev.confusion_matrix().sum()) == 0


def test_evaluator_raises_on_invalid_gt():
    ev = SemSegEvaluator(None, distributed=False, class_names=["a", "b"], ignore_label=255)
    ev.process([{"sem_seg_gt": np.full((4, 4), 9)}], [{"sem_seg": torch.rand(2, 4, 4).cuda()}])
    with pytest.raises(ValueError):
        ev.evaluate()


@pytest.mark.parametrize("cls", [SemSegEvaluator, VOCbEvaluator])
def test_evaluator_writes_predictions_json(cls, tmp_path):
    """process() with an output_dir keeps the COCO RLE records of every prediction's argmax map
    (VOC-b: folded at 20 first, train_net.py:60,71) and evaluate() writes them as
    sem_seg_predictions.json (plain_train_net.py:125,148-152): equal to the oracle's records of
    the numpy argmax, each decoding back to its label's mask."""
    import json
    T = 23 if cls is VOCbEvaluator else 9
    names = [f"c{i}" for i in range(T)]
    ev = cls(None, distributed=False, output_dir=str(tmp_path), class_names=names, ignore_label=255)
    expect = []
    for i in range(2):
        probs, gt = _case(T, 40 + i, 52, seed=30 + i, n_levels=50)
        ev.process([{"sem_seg_gt": gt.numpy(), "file_name": f"im{i}.png"}], [{"sem_seg": probs.cuda()}])
        pred = probs.numpy().argmax(0)
        if cls.clamp_pred >= 0:
            pred[pred >= cls.clamp_pred] = cls.clamp_pred
        expect += OE.sem_seg_records(pred, f"im{i}.png")
    ev.evaluate()
    recs = json.loads((tmp_path / "sem_seg_predictions.json").read_text())
    assert recs == expect
    for r in recs[:5]:
        assert OE.rle_decode(r["segmentation"]).shape == (40, 52) or OE.rle_decode(r["segmentation"]).shape == (41, 52)
