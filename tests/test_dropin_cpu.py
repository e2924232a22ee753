"""The drop-in surface on the CPU (no GPU calls): every name train_net.py imports from cat_seg,
the datasets eval.sh names, the checkpoint path detectron2's DetectionCheckpointer takes
(fvcore Checkpointer._load_model), OpenAI CLIP state dicts (model_vpt.py:515-531), the test
mapper's ResizeShortestEdge(640, 2560), the registered-dataset loader, the sharded test loader
and the TTA mapper."""
import ast
import os
import re

import numpy as np
import pytest
import torch
from PIL import Image

import cat_seg
from cat_seg import build_model
from cat_seg.data import DatasetCatalog, MetadataCatalog, build_test_loader, load_sem_seg
from cat_seg.data import transforms as T
from cat_seg.data.dataset_mappers import CATSegTestDatasetMapper, MaskFormerSemanticDatasetMapper
from cat_seg.test_time_augmentation import DatasetMapperTTA
from cat_seg.weights import CLIP

from test_boundary_cpu import tiny_cfg

REF = "/root/reference"
# train_net.py:74-80 (the list is read from the reference when it is present)
TRAIN_NET_IMPORTS = ["DETRPanopticDatasetMapper", "MaskFormerPanopticDatasetMapper", "MaskFormerSemanticDatasetMapper",
                     "SemanticSegmentorWithTTA", "add_cat_seg_config"]
# eval.sh:28-104 DATASETS.TEST names + configs/config.yaml DATASETS
EVAL_DATASETS = ["ade20k_150_test_sem_seg", "ade20k_full_sem_seg_freq_val_all", "voc_2012_test_sem_seg",
                 "voc_2012_test_background_sem_seg", "context_59_test_sem_seg", "context_459_test_sem_seg",
                 "coco_2017_train_stuff_all_sem_seg", "coco_2017_test_stuff_all_sem_seg"]


def _train_net_imports():
    path = os.path.join(REF, "train_net.py")
    if not os.path.exists(path):
        return TRAIN_NET_IMPORTS
    names = []
    for node in ast.walk(ast.parse(open(path).read())):
        if isinstance(node, ast.ImportFrom) and node.module == "cat_seg":
            names += [a.name for a in node.names]
    assert sorted(names) == sorted(TRAIN_NET_IMPORTS)
    return names


def test_every_train_net_import_resolves():
    for name in _train_net_imports():
        assert hasattr(cat_seg, name), name


def test_eval_sh_datasets_are_registered():
    names = list(EVAL_DATASETS)
    path = os.path.join(REF, "eval.sh")
    if os.path.exists(path):
        found = re.findall(r'DATASETS.TEST \\\(\\"([a-z0-9_]+)\\"', open(path).read())
        assert found and set(found) <= set(EVAL_DATASETS), found
    for n in names:
        assert n in DatasetCatalog.list(), n
        meta = MetadataCatalog.get(n)
        assert meta.evaluator_type in ("sem_seg", "sem_seg_background")
        assert len(meta.stuff_classes) > 0
    assert len(MetadataCatalog.get("ade20k_150_test_sem_seg").stuff_classes) == 150
    assert len(MetadataCatalog.get("ade20k_full_sem_seg_freq_val_all").stuff_classes) == 847
    assert MetadataCatalog.get("ade20k_full_sem_seg_freq_val_all").ignore_label == 65535
    assert MetadataCatalog.get("context_459_test_sem_seg").ignore_label == 459
    assert MetadataCatalog.get("voc_2012_test_background_sem_seg").stuff_classes[-1] == "background"


def test_panoptic_mappers_fail_loudly():
    for cls in (cat_seg.DETRPanopticDatasetMapper, cat_seg.MaskFormerPanopticDatasetMapper):
        with pytest.raises(NotImplementedError):
            cls(None, True)


def test_detection_checkpointer_load_path():
    """What fvcore's Checkpointer._load_model + DetectionCheckpointer._load_model do with the
    result of model.load_state_dict(sd, strict=False)."""
    m = build_model(tiny_cfg())
    ckpt = {"model": {k: v.clone() for k, v in m.state_dict().items()}}
    sd = ckpt.pop("model")
    model_sd = m.state_dict()
    incorrect = [k for k in sd if k in model_sd and tuple(sd[k].shape) != tuple(model_sd[k].shape)]
    assert not incorrect
    incompatible = m.load_state_dict(sd, strict=False)
    assert isinstance(incompatible.missing_keys, list) and isinstance(incompatible.unexpected_keys, list)
    buffers = dict(m.named_buffers(recurse=False))
    for k in ("pixel_mean", "pixel_std"):
        if k in buffers:
            try:
                incompatible.missing_keys.remove(k)
            except ValueError:
                pass
    for k in incompatible.unexpected_keys[:]:
        if "anchor_generator.cell_anchors" in k:
            incompatible.unexpected_keys.remove(k)
    assert incompatible.missing_keys == [] and incompatible.unexpected_keys == []
    # a partial checkpoint reports what it lacks (strict=False does not raise)
    part = {k: v for k, v in sd.items() if not k.startswith("upsample")}
    inc = m.load_state_dict(part, strict=False)
    assert sorted(inc.missing_keys) == sorted(k for k in sd if k.startswith("upsample"))


def test_openai_clip_state_dict_is_split_like_the_reference():
    """model_vpt.py:515-531: in_proj_weight -> q/k/v_proj_weight (chunk 3 on dim 0), metadata
    keys dropped; an unprefixed OpenAI dict lands under sem_seg_head.predictor.clip_model."""
    m = build_model(tiny_cfg())
    ref = {k: v.clone() for k, v in m.state_dict().items()}     # state_dict() aliases the parameters
    openai = {}
    for k, v in ref.items():
        if not k.startswith(CLIP):
            continue
        k = k[len(CLIP):]
        if k.endswith("attn.q_proj_weight"):
            base = k[: -len("q_proj_weight")]
            openai[base + "in_proj_weight"] = torch.cat(
                [ref[CLIP + base + f"{x}_proj_weight"] for x in "qkv"], 0) * 2.0
        elif not (k.endswith("attn.k_proj_weight") or k.endswith("attn.v_proj_weight")):
            openai[k] = v
    openai.update(input_resolution=torch.tensor(224), context_length=torch.tensor(16), vocab_size=torch.tensor(512))
    inc = m.load_state_dict(openai, strict=False)
    assert not inc.unexpected_keys, inc.unexpected_keys[:5]
    assert all(not k.startswith(CLIP) for k in inc.missing_keys)
    got = m.state_dict()
    for k in ref:
        if k.startswith(CLIP) and re.search(r"attn\.[qkv]_proj_weight$", k):
            assert torch.equal(got[k], ref[k] * 2.0), k
        else:
            assert torch.equal(got[k], ref[k]), k


def _write_dataset(tmp, shapes, ext="png"):
    img_dir, gt_dir = os.path.join(tmp, "img"), os.path.join(tmp, "gt")
    os.makedirs(img_dir)
    os.makedirs(gt_dir)
    rng = np.random.default_rng(0)
    for i, (h, w) in enumerate(shapes):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(os.path.join(img_dir, f"{i:03d}.jpg"))
        Image.fromarray(rng.integers(0, 5, (h, w), dtype=np.uint8)).save(os.path.join(gt_dir, f"{i:03d}.{ext}"))
    # an image without ground truth: load_sem_seg keeps the pairs only
    Image.fromarray(np.zeros((8, 8, 3), np.uint8)).save(os.path.join(img_dir, "zzz.jpg"))
    return img_dir, gt_dir


def test_load_sem_seg_and_test_mapper(tmp_path):
    img_dir, gt_dir = _write_dataset(str(tmp_path), [(480, 640), (700, 500), (300, 3000)])
    dicts = load_sem_seg(gt_dir, img_dir, gt_ext="png", image_ext="jpg")
    assert [os.path.basename(d["file_name"]) for d in dicts] == ["000.jpg", "001.jpg", "002.jpg"]
    mapper = CATSegTestDatasetMapper(tiny_cfg())
    # ResizeShortestEdge(640, 2560): short edge -> 640, long edge capped at 2560, round half up
    expect = [(640, 853), (896, 640), (256, 2560)]
    for d, (h, w), (oh, ow) in zip(dicts, expect, [(480, 640), (700, 500), (300, 3000)]):
        out = mapper(d)
        assert out["image"].dtype == torch.uint8 and tuple(out["image"].shape) == (3, h, w)
        assert (out["height"], out["width"]) == (oh, ow)
        assert "sem_seg_file_name" not in out
        src = np.asarray(Image.open(d["file_name"]).convert("RGB"))
        ref = np.asarray(Image.fromarray(src).resize((w, h), Image.BILINEAR))
        assert np.array_equal(out["image"].permute(1, 2, 0).numpy(), ref)


def test_resize_output_shape_matches_detectron2_rule():
    assert T.resize_output_shape(480, 640, 640, 2560) == (640, 853)
    assert T.resize_output_shape(640, 480, 640, 2560) == (853, 640)
    assert T.resize_output_shape(100, 1000, 640, 2560) == (256, 2560)
    assert T.resize_output_shape(512, 512, 640, 2560) == (640, 640)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_test_loader_covers_dataset_once(tmp_path, world):
    img_dir, gt_dir = _write_dataset(str(tmp_path), [(40, 48)] * 5)
    dicts = load_sem_seg(gt_dir, img_dir)
    seen = []
    for r in range(world):
        loader = build_test_loader(dicts, CATSegTestDatasetMapper(min_size=0), batch_size=2, rank=r, world=world)
        for batch in loader:
            assert 1 <= len(batch) <= 2
            seen += [os.path.basename(x["file_name"]) for x in batch]
    assert seen == [f"{i:03d}.jpg" for i in range(5)]


def test_registered_dataset_through_catalog(tmp_path, monkeypatch):
    img_dir, gt_dir = _write_dataset(str(tmp_path), [(40, 48), (50, 30)])
    name = "catseg_test_synthetic_sem_seg"
    if name not in DatasetCatalog.list():
        DatasetCatalog.register(name, lambda: load_sem_seg(gt_dir, img_dir))
        MetadataCatalog.get(name).set(stuff_classes=[f"c{i}" for i in range(5)], ignore_label=255,
                                      evaluator_type="sem_seg")
    loader = build_test_loader(name, CATSegTestDatasetMapper(min_size=0), rank=0, world=1)
    assert sum(len(b) for b in loader) == 2


def test_train_mapper_shapes(tmp_path):
    img_dir, gt_dir = _write_dataset(str(tmp_path), [(300, 500)])
    cfg = tiny_cfg()
    cfg.merge_from_file(os.path.join(REF, "configs", "vitl_336.yaml")) if os.path.exists(REF) else None
    cfg.merge_from_list(["INPUT.MIN_SIZE_TRAIN", "(384,)", "INPUT.CROP.ENABLED", "True", "INPUT.CROP.TYPE", "absolute",
                         "INPUT.CROP.SIZE", "(384, 384)", "INPUT.COLOR_AUG_SSD", "True", "INPUT.SIZE_DIVISIBILITY", "384"])
    mapper = MaskFormerSemanticDatasetMapper(cfg, True)
    out = mapper(load_sem_seg(gt_dir, img_dir)[0])
    assert tuple(out["image"].shape) == (3, 384, 384) and tuple(out["sem_seg"].shape) == (384, 384)
    assert out["instances"]["gt_masks"].shape[0] == len(out["instances"]["gt_classes"])


def test_tta_mapper_variants():
    cfg = tiny_cfg()
    d = {"image": torch.zeros(3, 60, 80, dtype=torch.uint8), "height": 60, "width": 80}
    augs = DatasetMapperTTA(min_sizes=(30, 60), max_size=4000, flip=True)(d)
    assert len(augs) == 4
    assert [tuple(a["image"].shape[1:]) for a in augs] == [(30, 40), (30, 40), (60, 80), (60, 80)]
    assert sum(any(isinstance(t, T.HFlipTransform) for t in a["transforms"]) for a in augs) == 2
    assert len(DatasetMapperTTA(cfg)(d)) == 18     # detectron2 defaults: 9 sizes x {plain, flip}


def test_inference_on_dataset_loop_with_stub_model(tmp_path):
    """The loop itself (warm-up, eval mode + no_grad, evaluator reset/process/evaluate) with a
    stand-in model on the CPU; the real model + evaluator run in test_gpu_harness.py."""
    from cat_seg.inference import DatasetEvaluators, inference_on_dataset
    img_dir, gt_dir = _write_dataset(str(tmp_path), [(40, 48)] * 7)
    loader = build_test_loader(load_sem_seg(gt_dir, img_dir), CATSegTestDatasetMapper(min_size=0), batch_size=3,
                               rank=0, world=1)

    class Stub(torch.nn.Module):
        def forward(self, inputs):
            assert not self.training and not torch.is_grad_enabled()
            return [{"sem_seg": torch.zeros(5, x["height"], x["width"])} for x in inputs]

    class Count:
        def reset(self):
            self.n = 0

        def process(self, i, o):
            self.n += len(o)

        def evaluate(self):
            return {"count": {"n": self.n}}

    m = Stub().train()
    res = inference_on_dataset(m, loader, DatasetEvaluators([Count()]))
    assert res == {"count": {"n": 7}} and m.training
