"""CATSegPredictor — class texts, prompt templates, the cached class embeddings and the
Aggregator call (reference cat_seg/modeling/transformer/cat_seg_predictor.py:20-224).

The CLIP text encoder and the Aggregator run on the MI355X engine
(`cat_seg.engine.CatSegEngine`), which the owning CATSeg meta-arch attaches after
it has its weights (`attach_engine`).  Class names are tokenized with the CLIP BPE
tokenizer (`MODEL.CATSEG_HIP.BPE_VOCAB`), or, for the reference's own class lists,
with the bundled token ids produced by the reference tokenizer.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import List, Optional

import numpy as np
import torch
from torch import nn

from ...registry import configurable
from ...tokenizer import BPETokenizer, class_prompts

_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data")


def bundled_tokens(class_names: List[str]) -> Optional[np.ndarray]:
    """Token ids of the reference datasets' class lists (made with the reference tokenizer)."""
    key = hashlib.sha1("\n".join(class_names).encode()).hexdigest()
    with open(os.path.join(_DATA, "class_lists.json")) as f:
        table = json.load(f)
    if key not in table:
        return None
    return np.load(os.path.join(_DATA, "class_tokens.npz"))[table[key]].astype(np.int64)


class CATSegPredictor(nn.Module):
    @configurable
    def __init__(self, *, train_class_json: str, test_class_json: str, clip_pretrained: str,
                 prompt_ensemble_type: str, text_guidance_dim: int, text_guidance_proj_dim: int,
                 appearance_guidance_dim: int, appearance_guidance_proj_dim: int, prompt_depth: int,
                 prompt_length: int, decoder_dims: list, decoder_guidance_dims: list,
                 decoder_guidance_proj_dims: list, num_heads: int, num_layers: int, hidden_dims: int,
                 pooling_sizes: list, feature_resolution: list, window_sizes: int, attention_type: str,
                 bpe_vocab: str = ""):
        super().__init__()
        self.class_texts = self._load_json(train_class_json)
        self.test_class_texts = self._load_json(test_class_json) or self.class_texts
        if prompt_ensemble_type != "single":
            # the reference's own eval text path cannot run these: its (T, P, 77) token stack
            # (cat_seg_predictor.py:196-208) reaches CLIP.encode_text's 3-d permute (model_vpt.py:428)
            # and raises (tests/golden/prompt_ensemble_probe.json, made by running the reference)
            raise NotImplementedError(
                f"PROMPT_ENSEMBLE_TYPE {prompt_ensemble_type!r}: only 'single' (the shipped configs' setting); "
                "the reference's multi-template path raises in CLIP.encode_text (model_vpt.py:428)")
        if attention_type not in ("linear", "full"):       # AttentionLayer (model.py:331-336)
            raise NotImplementedError(f"ATTENTION_TYPE {attention_type!r}")
        self.attention_type = attention_type
        # visual prompt tuning (PROMPT_DEPTH / PROMPT_LENGTH, model_vpt.py:243-265) reaches the engine through
        # the arch (arch_from_cfg); CatSegEngine refuses a depth below the vision layer count
        self.prompt_depth, self.prompt_length = int(prompt_depth), int(prompt_length)
        self.prompt_templates = ["A photo of a {} in the scene"]
        self.clip_pretrained = clip_pretrained
        self.bpe_vocab = bpe_vocab
        self.engine = None
        # class-prompt token ids per mode: the training step encodes TRAIN_CLASS_JSON every step,
        # eval encodes TEST_CLASS_JSON once and caches it (cat_seg_predictor.py:190-224)
        self.tokens = {"train": None, "test": None}
        self.cache = None

    @staticmethod
    def _load_json(path):
        if path and os.path.exists(path):
            with open(path) as f:
                return json.load(f)
        return None

    @classmethod
    def from_config(cls, cfg):
        h = cfg.MODEL.SEM_SEG_HEAD
        hip = cfg.MODEL.get("CATSEG_HIP", {}) if hasattr(cfg.MODEL, "get") else {}
        return dict(
            train_class_json=h.TRAIN_CLASS_JSON, test_class_json=h.TEST_CLASS_JSON,
            clip_pretrained=h.CLIP_PRETRAINED, prompt_ensemble_type=cfg.MODEL.PROMPT_ENSEMBLE_TYPE,
            text_guidance_dim=h.TEXT_GUIDANCE_DIM, text_guidance_proj_dim=h.TEXT_GUIDANCE_PROJ_DIM,
            appearance_guidance_dim=h.APPEARANCE_GUIDANCE_DIM,
            appearance_guidance_proj_dim=h.APPEARANCE_GUIDANCE_PROJ_DIM,
            decoder_dims=h.DECODER_DIMS, decoder_guidance_dims=h.DECODER_GUIDANCE_DIMS,
            decoder_guidance_proj_dims=h.DECODER_GUIDANCE_PROJ_DIMS, prompt_depth=h.PROMPT_DEPTH,
            prompt_length=h.PROMPT_LENGTH, num_layers=h.NUM_LAYERS, num_heads=h.NUM_HEADS,
            hidden_dims=h.HIDDEN_DIMS, pooling_sizes=h.POOLING_SIZES, feature_resolution=h.FEATURE_RESOLUTION,
            window_sizes=h.WINDOW_SIZES, attention_type=h.ATTENTION_TYPE,
            bpe_vocab=(hip.get("BPE_VOCAB", "") if hip else "") or os.environ.get("CATSEG_BPE_VOCAB", ""),
        )

    def attach_engine(self, engine):
        self.engine = engine
        self.cache = None

    def tokenize(self, classnames: List[str]) -> torch.Tensor:
        toks = None
        if self.bpe_vocab:
            toks = BPETokenizer(self.bpe_vocab).tokenize(class_prompts(classnames))
        else:
            toks = bundled_tokens(list(classnames))
        if toks is None:
            raise RuntimeError("class list is not one of the bundled reference lists: set "
                               "MODEL.CATSEG_HIP.BPE_VOCAB to CLIP's bpe_simple_vocab_16e6.txt.gz")
        return torch.from_numpy(toks)

    def class_tokens(self, mode: str) -> torch.Tensor:
        """Prompt token ids of the train ("train": TRAIN_CLASS_JSON) or test class set, cached."""
        if self.tokens[mode] is None:
            self.tokens[mode] = self.tokenize(self.class_texts if mode == "train" else self.test_class_texts)
        return self.tokens[mode]

    def get_text_embeds(self, classnames=None, templates=None, clip_model=None, prompt=None):
        """Encode + L2-normalize (cat_seg_predictor.py:190-224).  Returns (T, 1, C_o).

        Eval: the test class set is encoded once and cached; whenever the engine holds another
        class set (a training step ran in between) the cache is re-installed, so train / eval
        alternation (Trainer with EVAL_PERIOD) always evaluates on the test classes.
        Training: the train class set is re-encoded every call (uncached, as the reference)."""
        mode = "train" if self.training else "test"
        if mode == "test" and self.cache is not None and classnames is None:
            if self.engine.text_source() is not self.cache:
                self.engine.set_text(self.cache)
            return self.cache
        if classnames is not None:
            toks = self.tokenize(classnames)
        else:
            if self.tokens[mode] is None:
                self.tokens[mode] = self.tokenize(self.class_texts if mode == "train" else self.test_class_texts)
            toks = self.tokens[mode]
        emb = self.engine.encode_text(toks).unsqueeze(1)
        self.engine.set_text(emb)
        if mode == "test" and classnames is None:
            self.cache = emb
        return emb

    def set_class_tokens(self, tokens, mode: str = "both"):
        """Use pre-tokenized prompts (T, context) for the train / test / both class sets."""
        t = torch.as_tensor(tokens).long()
        for m in (("train", "test") if mode == "both" else (mode,)):
            self.tokens[m] = t
        self.cache = None

    def set_class_texts(self, class_texts: List[str]):
        """Switch the evaluated class set (a new TEST_CLASS_JSON)."""
        self.test_class_texts = list(class_texts)
        self.tokens["test"] = None
        self.cache = None

    def forward(self, x, vis_guidance, prompt=None, gt_cls=None):
        """x: (B, C_o, H, W) CLIP features; vis_guidance {res5, res4, res3} NCHW (reference layout).
        Runs the Aggregator on the engine; returns fp32 logits (B, T, 4H, 4W)."""
        if gt_cls is not None or prompt is not None:
            raise NotImplementedError("MI355X path: eval without gt_cls/prompt only")
        self.get_text_embeds()
        eng = self.engine
        B, C, H, W = x.shape
        dt = eng.dt
        tok = x.permute(0, 2, 3, 1).reshape(B, H * W, C)
        feats = torch.cat([tok.new_zeros(B, 1, C), tok], 1).reshape(B * (H * W + 1), C).float().contiguous()
        vis = [vis_guidance[k] for k in vis_guidance.keys()][::-1]       # [res3, res4, res5]
        nhwc = [v.permute(0, 2, 3, 1).reshape(-1, v.shape[1]).to(dt).contiguous() for v in vis]
        return eng.aggregate(feats, *nhwc)
