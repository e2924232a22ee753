"""The eval harness end to end on the GPU: a registered dataset on disk ->
sharded test loader (ResizeShortestEdge 640/2560 mapper) -> CATSeg.forward ->
SemSegEvaluator (confusion on the device) -> metrics, on one GPU and as two gloo ranks
sharing it; plus the reference's head / predictor API (cat_seg_head.py:2003-2010,
cat_seg_predictor.py:151-162) against the reference golden."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from PIL import Image

from cat_seg import build_model
from cat_seg.data import DatasetCatalog, MetadataCatalog, build_test_loader, load_sem_seg
from cat_seg.evaluation import SemSegEvaluator
from cat_seg.inference import inference_on_dataset
from oracle import semseg_eval as OE

from conftest import GOLDEN
from test_boundary_cpu import tiny_cfg

pytestmark = pytest.mark.gpu


def test_head_and_predictor_forward_match_golden():
    """CATSegHead.forward(features (B,1+HW,C), {"res5","res4","res3"} NCHW) and
    CATSegPredictor.forward(x (B,C,H,W), guidance) reproduce the reference logits."""
    g = dict(np.load(os.path.join(GOLDEN, "e2e_tiny_eval.npz")))
    model = build_model(tiny_cfg()).cuda().eval()
    pred = model.sem_seg_head.predictor
    eng = model.engine
    pred.cache = None
    eng.set_text(torch.from_numpy(g["text"]).cuda())
    pred.cache = torch.from_numpy(g["text"]).cuda()            # the eval cache (cat_seg_predictor.py:191-192)
    imgs = [torch.from_numpy(g[k]).float() for k in ("image0", "image1")]
    raw = torch.stack(imgs).cuda()
    sizes = torch.tensor([[384, 384]] * 2, dtype=torch.int32, device="cuda")
    arch = model.arch
    G, Lt = arch.grid, arch.grid ** 2 + 1
    with torch.no_grad():
        feats, hooks = eng.encode_image(raw, sizes)
        r3, r4, r5 = eng.guidance(feats, hooks)
        nchw = lambda t, s: t.float().view(2, s, s, -1).permute(0, 3, 1, 2).contiguous()   # noqa: E731
        guidance = {"res5": nchw(r5, 4 * G), "res4": nchw(r4, 2 * G), "res3": nchw(r3, G)}
        features = feats.view(2, Lt, -1)
        out_head = model.sem_seg_head(features, guidance).cpu()
        x = features[:, 1:, :].reshape(2, G, G, -1).permute(0, 3, 1, 2)
        out_pred = pred(x, guidance).cpu()
    ref = torch.from_numpy(g["logits"])
    assert out_head.shape == ref.shape
    assert (out_head - ref).abs().max().item() < 1e-3
    assert torch.equal(out_head, out_pred)


def _dataset(root, n=5, classes=6, seed=0):
    img_dir, gt_dir = os.path.join(root, "images"), os.path.join(root, "gt")
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(gt_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    shapes = [(240, 320), (300, 200), (256, 256), (200, 360), (280, 280)][:n]
    for i, (h, w) in enumerate(shapes):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(os.path.join(img_dir, f"{i}.png"))
        gt = rng.integers(0, classes, (h, w)).astype(np.uint8)
        gt[:10] = 255                                                  # ignored band
        Image.fromarray(gt).save(os.path.join(gt_dir, f"{i}.png"))
    return img_dir, gt_dir


def _register(name, img_dir, gt_dir, classes):
    if name not in DatasetCatalog.list():
        DatasetCatalog.register(name, lambda: load_sem_seg(gt_dir, img_dir, gt_ext="png", image_ext="png"))
        MetadataCatalog.get(name).set(stuff_classes=[f"class{i}" for i in range(classes)], ignore_label=255,
                                      evaluator_type="sem_seg")


def _tokens(classes, seed=3):
    rng = np.random.default_rng(seed)
    tok = np.zeros((classes, 16), np.int64)
    for t in range(classes):
        tok[t, 0] = 510
        tok[t, 1:5] = rng.integers(1, 500, 4)
        tok[t, 5] = 511
    return tok


class _Recorder:
    """Wraps the evaluator and keeps each output's argmax for the oracle recount."""

    def __init__(self, ev):
        self.ev, self.preds = ev, []

    def reset(self):
        self.ev.reset()

    def process(self, inputs, outputs):
        self.ev.process(inputs, outputs)
        for i, o in zip(inputs, outputs):
            self.preds.append((i["file_name"], o["sem_seg"].cpu().numpy()))

    def evaluate(self):
        return self.ev.evaluate()


def _oracle_conf(preds, dataset, classes):
    table = {d["file_name"]: d["sem_seg_file_name"] for d in DatasetCatalog.get(dataset)}
    conf = np.zeros((classes + 1, classes + 1), np.int64)
    for f, probs in preds:
        gt = np.array(Image.open(table[f]), dtype=np.int64)
        OE.confusion_update(conf, probs, gt, classes, 255)
    return conf


def test_eval_harness_one_gpu(tmp_path):
    classes = 6
    img_dir, gt_dir = _dataset(str(tmp_path), classes=classes)
    name = "catseg_gpu_harness_sem_seg"
    _register(name, img_dir, gt_dir, classes)
    model = build_model(tiny_cfg()).cuda().eval()
    model.sem_seg_head.predictor.set_class_tokens(_tokens(classes))
    loader = build_test_loader(name, cfg=tiny_cfg(), batch_size=2)
    ev = _Recorder(SemSegEvaluator(name, distributed=False, device="cuda"))
    res = inference_on_dataset(model, loader, ev)
    assert len(ev.preds) == 5
    for f, p in ev.preds:              # outputs at the original size, as the evaluator needs
        h, w = Image.open(f).size[::-1]
        assert p.shape == (classes, h, w)
    conf = _oracle_conf(ev.preds, name, classes)
    np.testing.assert_array_equal(ev.ev.confusion_matrix(), conf)
    ref = OE.metrics(conf, [f"class{i}" for i in range(classes)])
    assert abs(res["sem_seg"]["mIoU"] - ref["mIoU"]) < 1e-9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        classes = 6
        name = "catseg_gpu_harness_sem_seg"
        _register(name, os.path.join(root, "images"), os.path.join(root, "gt"), classes)
        torch.cuda.set_device(0)
        model = build_model(tiny_cfg()).cuda().eval()
        model.sem_seg_head.predictor.set_class_tokens(_tokens(classes))
        loader = build_test_loader(name, cfg=tiny_cfg(), batch_size=1)
        ev = _Recorder(SemSegEvaluator(name, distributed=True, device="cuda"))
        res = inference_on_dataset(model, loader, ev)
        local = ev.ev._conf.cpu().numpy().reshape(classes + 1, classes + 1)
        q.put((rank, [f for f, _ in ev.preds], local.tolist(), res.get("sem_seg", {}).get("mIoU")))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_eval_harness_gloo_world2_shares_one_gpu(tmp_path):
    """Two ranks (gloo) split the dataset with the InferenceSampler rule, each runs CATSeg on its
    shard; evaluate() sums the confusion matrices across ranks (plain_train_net.py:136-146) and
    rank 0's metrics equal the single-process run's."""
    classes = 6
    root = str(tmp_path)
    img_dir, gt_dir = _dataset(root, classes=classes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, root, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {}
    for _ in ps:
        r, files, conf, miou = q.get(timeout=240)
        got[r] = (files, np.array(conf), miou)
    for p in ps:
        p.join(timeout=60)
    assert [os.path.basename(f) for f in got[0][0]] == ["0.png", "1.png", "2.png"]
    assert [os.path.basename(f) for f in got[1][0]] == ["3.png", "4.png"]
    # single-process reference over the whole dataset
    name = "catseg_gpu_harness_sem_seg"
    _register(name, img_dir, gt_dir, classes)
    model = build_model(tiny_cfg()).cuda().eval()
    model.sem_seg_head.predictor.set_class_tokens(_tokens(classes))
    ev = SemSegEvaluator(name, distributed=False, device="cuda")
    res = inference_on_dataset(model, build_test_loader(name, cfg=tiny_cfg()), ev)
    np.testing.assert_array_equal(got[0][1] + got[1][1], ev.confusion_matrix())
    assert got[0][2] is not None and abs(got[0][2] - res["sem_seg"]["mIoU"]) < 1e-9
    assert got[1][2] is None
