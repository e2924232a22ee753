"""CATSeg meta-architecture — the drop-in boundary of the MI355X path (reference
cat_seg/cat_seg_model.py:18-229).

`@META_ARCH_REGISTRY.register() class CATSeg`, built by `build_model(cfg)` from the
same config keys, with `forward(batched_inputs: list[dict]) -> list[dict]`:
  input  {"image": (3, H, W) uint8/float 0-255 (CPU or device), optional "height", "width"}
  output {"sem_seg": (T, height, width) fp32 sigmoid probabilities on the model device}
The reference returns results for batched_inputs[0] only (cat_seg_model.py:227-229);
this boundary returns one result per input image by default
(MODEL.CATSEG_HIP.RETURN_ALL_IMAGES; set False for the reference's exact behaviour).

Everything between the input copy and the returned tensors runs in the HIP kernels of
libcatseg_hip.so through `CatSegEngine`; there is no CPU or PyTorch-op fallback.
Parameters live under the reference checkpoint keys (`state_dict()` /
`load_state_dict()`, detectron2 `{"model": ...}` files accepted), synthesized
deterministically when no checkpoint is given.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Tuple

import torch
from torch import nn
from torch.nn.modules.module import _IncompatibleKeys

from . import custom_ops, ops
from .arch import CatSegArch, arch_from_cfg
from .engine import CatSegEngine
from .modeling.heads.cat_seg_head import CATSegHead  # noqa: F401  (registers the head)
from .params import apply_clip_finetune, attach_parameters
from .registry import META_ARCH_REGISTRY, build_sem_seg_head, configurable
from .training import clip_image_train_forward, clip_text_train_forward, head_train_forward
from .weights import CLIP as CLIP_PREFIX, synthesize_state_dict

_DTYPES = {"bf16": torch.bfloat16, "f32": torch.float32, "fp32": torch.float32}


def _weights_version(params: Iterable[nn.Parameter]) -> int:
    """Sum of the parameters' in-place version counters: an optimizer step or a copy_ bumps it."""
    return sum(p._version for p in params)


def convert_openai_clip_keys(sd: Dict[str, torch.Tensor], prefix: str = "") -> Dict[str, torch.Tensor]:
    """OpenAI CLIP `attn.in_proj_weight` -> q/k/v_proj_weight split (model_vpt.py:520-528), the
    metadata entries input_resolution / context_length / vocab_size dropped (:511-512), every
    key prefixed with `prefix`."""
    out = {}
    for k, v in sd.items():
        if k.endswith("attn.in_proj_weight"):
            q, kk, vv = v.chunk(3, dim=0)
            out[prefix + k.replace("in_proj", "q_proj")] = q
            out[prefix + k.replace("in_proj", "k_proj")] = kk
            out[prefix + k.replace("in_proj", "v_proj")] = vv
        elif k not in ("input_resolution", "context_length", "vocab_size"):
            out[prefix + k] = v
    return out


@META_ARCH_REGISTRY.register()
class CATSeg(nn.Module):
    @configurable
    def __init__(self, *, backbone, sem_seg_head: nn.Module, size_divisibility: int, pixel_mean: Tuple[float],
                 pixel_std: Tuple[float], clip_pixel_mean: Tuple[float], clip_pixel_std: Tuple[float],
                 train_class_json: str, test_class_json: str, sliding_window: bool, clip_finetune: str,
                 backbone_multiplier: float, clip_pretrained: str, arch: Optional[CatSegArch] = None,
                 dtype: str = "bf16", return_all_images: bool = True, synthetic_seed: int = 0,
                 vit_fp8: bool = False, graph: bool = True):
        super().__init__()
        self.backbone = backbone
        self.sem_seg_head = sem_seg_head
        self.size_divisibility = size_divisibility
        self.register_buffer("pixel_mean", torch.Tensor(pixel_mean).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.Tensor(pixel_std).view(-1, 1, 1), False)
        self.register_buffer("clip_pixel_mean", torch.Tensor(clip_pixel_mean).view(-1, 1, 1), False)
        self.register_buffer("clip_pixel_std", torch.Tensor(clip_pixel_std).view(-1, 1, 1), False)
        self.train_class_json, self.test_class_json = train_class_json, test_class_json
        self.clip_finetune = clip_finetune
        self.sliding_window = sliding_window
        arch = arch or arch_from_cfg_defaults(clip_pretrained)
        # cat_seg_model.py:78 (384 for ViT-B/16, else 336); non-reference presets keep their own
        self.clip_resolution = ((384, 384) if clip_pretrained == "ViT-B/16" else
                                (336, 336) if clip_pretrained.startswith("ViT-") else (arch.clip_resolution,) * 2)
        self.arch = arch.replace(
            clip_resolution=self.clip_resolution[0], size_divisibility=size_divisibility,
            clip_pixel_mean=tuple(clip_pixel_mean), clip_pixel_std=tuple(clip_pixel_std))
        self.compute_dtype = _DTYPES[dtype]
        self.return_all_images = return_all_images
        self.vit_fp8 = bool(vit_fp8)
        # eval forward: host images through one reused pinned canvas, the network replayed from a
        # hipGraph captured per input geometry (MODEL.CATSEG_HIP.GRAPH)
        self.use_graph = bool(graph)
        self._stage: Dict[tuple, dict] = {}
        self._graphs: Dict[tuple, dict] = {}
        # the weights as real nn.Parameters under the reference's module names (cat_seg.params):
        # CLIP under sem_seg_head.predictor.clip_model, the Aggregator under .transformer, and the
        # guidance upsamplers (cat_seg_model.py:81-82); requires_grad per CLIP_FINETUNE (:57-75)
        sd = synthesize_state_dict(self.arch, seed=synthetic_seed)
        attach_parameters(self, sd)
        apply_clip_finetune(self.sem_seg_head.predictor.clip_model, clip_finetune)
        # the engines hold kernel-layout copies of the weights, keyed by the parameters' version counters
        self._engine: Optional[CatSegEngine] = None
        self._train_engine: Optional[CatSegEngine] = None
        self._engine_key = self._train_engine_key = None
        self.input_format = "RGB"          # read by SemanticSegmentorWithTTA / DefaultPredictor
        self._op_handle = custom_ops.register_model(self)   # catseg::head_logits (torch.compile path)

    @classmethod
    def from_config(cls, cfg):
        hip = cfg.MODEL.get("CATSEG_HIP", {}) if hasattr(cfg.MODEL, "get") else {}
        return {
            "backbone": None,
            "sem_seg_head": build_sem_seg_head(cfg, None),
            "size_divisibility": cfg.MODEL.MASK_FORMER.SIZE_DIVISIBILITY,
            "pixel_mean": cfg.MODEL.PIXEL_MEAN,
            "pixel_std": cfg.MODEL.PIXEL_STD,
            "clip_pixel_mean": cfg.MODEL.CLIP_PIXEL_MEAN,
            "clip_pixel_std": cfg.MODEL.CLIP_PIXEL_STD,
            "train_class_json": cfg.MODEL.SEM_SEG_HEAD.TRAIN_CLASS_JSON,
            "test_class_json": cfg.MODEL.SEM_SEG_HEAD.TEST_CLASS_JSON,
            "sliding_window": cfg.TEST.SLIDING_WINDOW,
            "clip_finetune": cfg.MODEL.SEM_SEG_HEAD.CLIP_FINETUNE,
            "backbone_multiplier": cfg.SOLVER.BACKBONE_MULTIPLIER,
            "clip_pretrained": cfg.MODEL.SEM_SEG_HEAD.CLIP_PRETRAINED,
            "arch": arch_from_cfg(cfg),
            "dtype": hip.get("DTYPE", "bf16") if hip else "bf16",
            "return_all_images": bool(hip.get("RETURN_ALL_IMAGES", True)) if hip else True,
            "synthetic_seed": int(hip.get("SYNTHETIC_SEED", 0)) if hip else 0,
            "vit_fp8": bool(hip.get("VIT_FP8", False)) if hip else False,
            "graph": bool(hip.get("GRAPH", True)) if hip else True,
        }

    # ------------------------------------------------------------------ parameters
    @property
    def device(self):
        return self.pixel_mean.device

    @property
    def _sd(self) -> Dict[str, torch.Tensor]:
        """The weights by reference checkpoint key (detached views of the nn.Parameters)."""
        return OrderedDict((k, p.detach()) for k, p in self.named_parameters())

    def state_dict(self, *args, **kwargs):        # reference checkpoint keys
        return OrderedDict(self._sd)

    def load_state_dict(self, state_dict, strict: bool = True, **_):
        """Reference checkpoint keys (detectron2 `{"model": sd}` accepted, OpenAI `in_proj_weight`
        split).  Returns torch's `_IncompatibleKeys(missing_keys, unexpected_keys)` (lists), which
        fvcore's Checkpointer._load_model reads and edits (DetectionCheckpointer drops
        pixel_mean / pixel_std from missing_keys)."""
        sd = state_dict.get("model", state_dict)
        sd = {k: (v if torch.is_tensor(v) else torch.as_tensor(v)) for k, v in sd.items()}
        if any(k.endswith("attn.in_proj_weight") for k in sd):
            # an OpenAI CLIP state dict (clip.load -> build_model, model_vpt.py:515-531) has no
            # module prefix: its keys belong under sem_seg_head.predictor.clip_model.
            prefix = "" if any(k.startswith(CLIP_PREFIX) for k in sd) else CLIP_PREFIX
            sd = convert_openai_clip_keys(sd, prefix)
        params = dict(self.named_parameters())
        missing = [k for k in params if k not in sd]
        unexpected = [k for k in sd if k not in params]
        if strict and (missing or unexpected):
            raise KeyError(f"load_state_dict: missing {missing[:5]}... unexpected {unexpected[:5]}...")
        with torch.no_grad():
            for k, p in params.items():
                if k in sd:
                    if tuple(sd[k].shape) != tuple(p.shape):
                        raise ValueError(f"{k}: shape {tuple(sd[k].shape)} != {tuple(p.shape)}")
                    p.copy_(sd[k].to(p.device, p.dtype))
        self._engine = self._train_engine = None
        self._graphs.clear()
        return _IncompatibleKeys(list(missing), list(unexpected))

    def _engine_device(self) -> torch.device:
        """The CUDA device the engine runs on: the module's device when it is on the GPU,
        else the current CUDA device (the HIP path has no CPU fallback)."""
        d = self.device
        if d.type == "cuda":
            return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())
        return torch.device("cuda", torch.cuda.current_device())

    @property
    def engine(self) -> CatSegEngine:
        """Built once per resolved device (weights converted / uploaded once), rebuilt only when
        the model moves to another GPU or new weights are loaded."""
        dev = self._engine_device()
        key = (dev, _weights_version(self.parameters()))
        if self._engine is None or self._engine_key != key:
            self._engine = CatSegEngine(self.arch, self._sd, dtype=self.compute_dtype, device=dev,
                                        vit_fp8=self.vit_fp8)
            self._engine_key = key
            self._graphs.clear()           # captured forwards point at the old engine's weights
            self.sem_seg_head.predictor.attach_engine(self._engine)
        return self._engine

    @property
    def train_engine(self) -> CatSegEngine:
        """fp32 engine for the training step's CLIP encoders (the reference trains in fp32).  With CLIP
        fine-tuning the autograd path reads the trained block weights from the parameters directly and
        uses the engine only for the frozen embeddings, so it is rebuilt when a frozen CLIP weight changed
        (a checkpoint load bumps its version), not after every optimizer step."""
        dev = self._engine_device()
        clip = self.sem_seg_head.predictor.clip_model
        trains = any(p.requires_grad for p in clip.parameters())
        key = (dev, _weights_version(p for p in clip.parameters() if not (trains and p.requires_grad)))
        if self._train_engine is None or self._train_engine_key != key:
            self._train_engine = CatSegEngine(self.arch, self._sd, dtype=torch.float32, device=dev)
            self._train_engine_key = key
        return self._train_engine

    # ------------------------------------------------------------------ forward
    def _batch(self, eng: CatSegEngine, images: List[torch.Tensor]):
        """Stage the images into one zero-padded fp32 canvas on the device (ImageList.from_tensors
        geometry: batch max, rounded up to size_divisibility).  Host images go through one pinned
        canvas and one H2D copy; images already on the device are copied in place there."""
        d = max(self.size_divisibility, 1)
        H = max(int(i.shape[-2]) for i in images)
        W = max(int(i.shape[-1]) for i in images)
        H, W = -(-H // d) * d, -(-W // d) * d
        dev = eng.device
        on_dev = all(i.is_cuda for i in images)
        raw = torch.zeros(len(images), 3, H, W, dtype=torch.float32, device=dev if on_dev else "cpu",
                          pin_memory=not on_dev)
        for k, im in enumerate(images):
            raw[k, :, : im.shape[-2], : im.shape[-1]].copy_(im)
        sizes = [[int(i.shape[-2]), int(i.shape[-1])] for i in images]
        sizes_dev = torch.tensor(sizes, dtype=torch.int32).to(dev, non_blocking=True)
        return (raw if on_dev else raw.to(dev, non_blocking=True)), sizes_dev, sizes

    def _forward_traced(self, batched_inputs: List[dict]):
        """The eval forward as dynamo traces it (torch.compile): the canvas staging in torch ops, the
        network as the one registered operator catseg::head_logits (custom_ops), the resize through
        catseg::postprocess; same kernels and results as the eager branch below."""
        handle = self._op_handle
        n_classes, res = custom_ops.head_meta(handle)
        images = [x["image"] for x in batched_inputs]
        d = max(self.size_divisibility, 1)
        H = max(int(i.shape[-2]) for i in images)
        W = max(int(i.shape[-1]) for i in images)
        H, W = -(-H // d) * d, -(-W // d) * d
        dev = self._engine_device()
        raw = torch.zeros(len(images), 3, H, W, dtype=torch.float32, device=dev)
        for k, im in enumerate(images):
            raw[k, :, : im.shape[-2], : im.shape[-1]] = im.to(dev, torch.float32)
        sizes = [(int(i.shape[-2]), int(i.shape[-1])) for i in images]
        sizes_dev = torch.tensor(sizes, dtype=torch.int32, device=dev)
        logits = torch.ops.catseg.head_logits(raw, sizes_dev, handle, n_classes, res)
        n = len(batched_inputs) if self.return_all_images else 1
        results = []
        for i in range(n):
            ih, iw = sizes[i]
            h = int(batched_inputs[i].get("height", ih))
            w = int(batched_inputs[i].get("width", iw))
            out = torch.ops.catseg.postprocess(logits[i:i + 1], h, w, min(res, ih), min(res, iw))
            results.append({"sem_seg": out[0]})
        return results

    def _stage_canvas(self, eng: CatSegEngine, images: List[torch.Tensor], canvas: torch.Tensor) -> None:
        """Write the images into the zero-padded fp32 device canvas (ImageList.from_tensors geometry;
        the padding stays zero: every call of one geometry writes the same regions).  Host images go
        through pinned staging canvases of their own dtype (uint8 from detectron2's mappers: 4x fewer
        bytes than fp32), reused across calls in two slots; the H2D copy and the device-side dtype
        conversion run on the compute stream, and an event per slot keeps the host from rewriting a
        slot whose copy has not run yet (the host runs at most two calls ahead).  A separate copy
        stream ordered by events measured slower on the box (tools/probe_boundary.py: 10.20 vs 10.11
        ms per bs-8 call, 10.05 with the images already on the device): the cross-stream waits cost
        more than the ~0.1 ms copy they would hide."""
        if all(i.is_cuda for i in images):
            for k, im in enumerate(images):
                canvas[k, :, : im.shape[-2], : im.shape[-1]].copy_(im)
            return
        dt = images[0].dtype if all(i.dtype == images[0].dtype for i in images) else torch.float32
        key = (tuple(canvas.shape), dt, canvas.device)
        st = self._stage.get(key)
        if st is None:
            st = {"slots": [{"host": torch.zeros(canvas.shape, dtype=dt, pin_memory=True),
                             "dev": torch.zeros(canvas.shape, dtype=dt, device=canvas.device),
                             "done": None} for _ in range(2)],
                  "next": 0}
            self._stage[key] = st
        slot = st["slots"][st["next"]]
        st["next"] ^= 1
        if slot["done"] is not None:
            slot["done"].synchronize()         # this slot's previous H2D has read the pinned canvas
        host = slot["host"]
        for k, im in enumerate(images):
            host[k, :, : im.shape[-2], : im.shape[-1]].copy_(im)
        slot["dev"].copy_(host, non_blocking=True)
        canvas.copy_(slot["dev"])              # device-side dtype conversion
        slot["done"] = torch.cuda.Event()
        slot["done"].record(torch.cuda.current_stream(canvas.device))

    def _canvas_geometry(self, images: List[torch.Tensor]):
        d = max(self.size_divisibility, 1)
        H = max(int(i.shape[-2]) for i in images)
        W = max(int(i.shape[-1]) for i in images)
        return -(-H // d) * d, -(-W // d) * d

    def _forward_graph(self, eng: CatSegEngine, batched_inputs: List[dict]):
        """The eval forward as one hipGraph replay per input geometry (what bench.py times): the
        first call of a geometry captures engine.head_logits, every call stages its images into the
        captured canvas, replays, and resizes the captured logits into fresh output tensors."""
        images = [x["image"] for x in batched_inputs]
        H, W = self._canvas_geometry(images)
        sizes = tuple((int(i.shape[-2]), int(i.shape[-1])) for i in images)
        n = len(batched_inputs) if self.return_all_images else 1
        outs = tuple((int(batched_inputs[i].get("height", sizes[i][0])), int(batched_inputs[i].get("width", sizes[i][1])))
                     for i in range(n))
        key = (id(eng), id(eng._text), len(images), H, W, sizes)
        g = self._graphs.get(key)
        dev = eng.device
        if g is None:
            raw = torch.zeros(len(images), 3, H, W, dtype=torch.float32, device=dev)
            sizes_dev = torch.tensor(sizes, dtype=torch.int32, device=dev)
            stream = torch.cuda.Stream(device=dev)
            stream.wait_stream(torch.cuda.current_stream(dev))

            with torch.cuda.stream(stream):
                eng.head_logits(raw, sizes_dev)  # warm the allocator outside the capture
            torch.cuda.current_stream(dev).wait_stream(stream)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                logits = eng.head_logits(raw, sizes_dev)
            # the graph replays raw device pointers: hold every tensor it reads that was allocated
            # outside the capture (the canvas, the sizes), the engine and its class-set buffers (ids in
            # the key stay unique while referenced); keep the 4 newest geometries
            g = {"graph": graph, "raw": raw, "sizes": sizes_dev, "logits": logits, "refs": (eng, eng._text)}
            while len(self._graphs) >= 4:
                self._graphs.pop(next(iter(self._graphs)))
            self._graphs[key] = g
        self._stage_canvas(eng, images, g["raw"])
        g["graph"].replay()
        # the resize to each image's output size runs after the replay into FRESH tensors (the caller
        # may keep the results across calls), as the eager path does
        logits = g["logits"]
        h_l, w_l = logits.shape[-2:]
        if n > 1 and len(set(outs)) == 1 and len(set(sizes[:n])) == 1:
            # one launch for the whole batch (the engine leg's form); each result is a view of it
            out = torch.empty(n, logits.shape[1], outs[0][0], outs[0][1], device=dev)
            ops.postprocess(logits[:n], out, crop=(min(h_l, sizes[0][0]), min(w_l, sizes[0][1])))
            return [{"sem_seg": out[i]} for i in range(n)]
        results = []
        for i in range(n):
            out = torch.empty(1, logits.shape[1], outs[i][0], outs[i][1], device=dev)
            ops.postprocess(logits[i:i + 1], out, crop=(min(h_l, sizes[i][0]), min(w_l, sizes[i][1])))
            results.append({"sem_seg": out[0]})
        return results

    def forward(self, batched_inputs: List[dict]):
        if self.training:
            return self._training_loss(batched_inputs)
        if self.sliding_window:
            return self._forward_sliding(batched_inputs)
        if torch.compiler.is_compiling():
            return self._forward_traced(batched_inputs)
        with torch.no_grad():
            eng = self.engine
            self.sem_seg_head.predictor.get_text_embeds()
            if self.use_graph:
                return self._forward_graph(eng, batched_inputs)
            raw, sizes_dev, sizes = self._batch(eng, [x["image"] for x in batched_inputs])
            logits = eng.head_logits(raw, sizes_dev)
            n = len(batched_inputs) if self.return_all_images else 1
            results = []
            h_l, w_l = logits.shape[-2:]
            for i in range(n):
                ih, iw = sizes[i]
                h = int(batched_inputs[i].get("height", ih))
                w = int(batched_inputs[i].get("width", iw))
                out = torch.empty(1, logits.shape[1], h, w, device=eng.device)
                ops.postprocess(logits[i:i + 1], out, crop=(min(h_l, ih), min(w_l, iw)))
                results.append({"sem_seg": out[0]})
            return results


    def _training_loss(self, batched_inputs: List[dict]):
        """The training branch (cat_seg_model.py:136-146,178-203): fp32 CLIP dense features + hooks and
        the training class set's text embeddings (re-encoded every step, cat_seg_predictor.py:190-224),
        the head with its HIP backward (cat_seg.training.head_train_forward), the logits upsampled to
        the targets' size and BCE-with-logits against one-hot targets (ops.BCEOneHotLoss).
        Returns {"loss_sem_seg": 0-d tensor}; `loss.backward()` fills `.grad` of every Aggregator and
        upsampler parameter and of the CLIP parameters CLIP_FINETUNE trains (cat_seg_model.py:57-75:
        'attention' = the q / v projections of both encoders' blocks): with any of those the CLIP
        encoders run as autograd Functions too (cat_seg.training.clip_*_train_forward), else without
        a graph on the engine."""
        if self.device.type != "cuda":
            raise RuntimeError("CATSeg training runs on the GPU: move the model there first (model.to('cuda'))")
        eng = self.train_engine
        pred = self.sem_seg_head.predictor
        params = dict(self.named_parameters())
        raw, sizes_dev, _ = self._batch(eng, [x["image"] for x in batched_inputs])
        if any(p.requires_grad for p in pred.clip_model.parameters()):
            text = clip_text_train_forward(self.arch, params, eng, pred.class_tokens("train"))
            feats, hooks = clip_image_train_forward(self.arch, params, eng, raw, sizes_dev)
        else:
            with torch.no_grad():
                text = eng.encode_text(pred.class_tokens("train"))
                feats, hooks = eng.encode_image(raw, sizes_dev)
        logits = head_train_forward(self.arch, params, feats, hooks, text)
        targets = torch.stack([x["sem_seg"].to(eng.device) for x in batched_inputs], dim=0)
        loss = ops.BCEOneHotLoss.apply(logits, targets, self.sem_seg_head.ignore_value)
        return {"loss_sem_seg": loss}

    def _forward_sliding(self, batched_inputs: List[dict]):
        """TEST.SLIDING_WINDOW eval (cat_seg_model.py:156-176,204-218): every image (or image 0 in
        the reference mode) through 4 Unfold tiles + 1 global crop; height/width default to 640."""
        with torch.no_grad():
            eng = self.engine
            self.sem_seg_head.predictor.get_text_embeds()
            n = len(batched_inputs) if self.return_all_images else 1
            inputs = batched_inputs[:n]
            raw, sizes_dev, _ = self._batch(eng, [x["image"] for x in inputs])
            res = eng.SLIDE_OUT
            out_hw = [(int(x.get("height", res)), int(x.get("width", res))) for x in inputs]
            return [{"sem_seg": o} for o in eng.forward_sliding(raw, sizes_dev, out_hw)]


def arch_from_cfg_defaults(clip_pretrained: str) -> CatSegArch:
    from .arch import PRESETS
    return PRESETS[clip_pretrained]
