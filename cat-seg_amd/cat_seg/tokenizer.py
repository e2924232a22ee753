"""CLIP byte-level BPE tokenizer + `tokenize` (the text side of the reference:
cat_seg/third_party/simple_tokenizer.py and clip.tokenize, clip.py:200-214).

Restated from the published CLIP tokenizer algorithm: UTF-8 bytes are mapped to
printable unicode symbols, words are split by CLIP's regex, each word is merged
greedily by BPE rank (the lowest-ranked adjacent pair first, all its occurrences at
once), and `</w>` marks a word end.  The merge table is the vocabulary file CLIP
ships (`bpe_simple_vocab_16e6.txt.gz`); pass its path — it is data, not bundled here.
`ftfy.fix_text` is not applied (ftfy is not installed); class-name lists are ASCII.
"""
from __future__ import annotations

import gzip
import html
import os
from functools import lru_cache
from typing import List, Sequence, Union

import numpy as np
import regex as re

_PAT = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                  re.IGNORECASE)


@lru_cache()
def byte_symbols():
    """Byte -> printable unicode character (printable latin-1 bytes map to themselves)."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    table = {b: chr(b) for b in keep}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def default_vocab_path() -> str:
    return os.environ.get("CATSEG_BPE_VOCAB", "")


class BPETokenizer:
    def __init__(self, vocab_path: str):
        if not vocab_path or not os.path.exists(vocab_path):
            raise FileNotFoundError(
                f"CLIP BPE vocabulary not found at {vocab_path!r} (set MODEL.CATSEG_HIP.BPE_VOCAB or CATSEG_BPE_VOCAB)")
        with gzip.open(vocab_path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges = [tuple(l.split()) for l in lines[1: 49152 - 256 - 2 + 1]]
        syms = list(byte_symbols().values())
        vocab = syms + [s + "</w>" for s in syms] + ["".join(m) for m in merges]
        vocab += ["<|startoftext|>", "<|endoftext|>"]
        self.encoder = {t: i for i, t in enumerate(vocab)}
        self.ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {"<|startoftext|>": "<|startoftext|>", "<|endoftext|>": "<|endoftext|>"}
        self.sot = self.encoder["<|startoftext|>"]
        self.eot = self.encoder["<|endoftext|>"]

    def _bpe(self, word: str) -> List[str]:
        if word in self.cache:
            return self.cache[word].split(" ")
        parts = list(word[:-1]) + [word[-1] + "</w>"]
        while len(parts) > 1:
            best, best_rank = None, None
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = (parts[i], parts[i + 1]), r
            if best is None:
                break
            merged, i = [], 0
            while i < len(parts):
                if i < len(parts) - 1 and (parts[i], parts[i + 1]) == best:
                    merged.append(parts[i] + parts[i + 1])
                    i += 2
                else:
                    merged.append(parts[i])
                    i += 1
            parts = merged
        self.cache[word] = " ".join(parts)
        return parts

    def encode(self, text: str) -> List[int]:
        text = html.unescape(html.unescape(text)).strip()
        text = re.sub(r"\s+", " ", text).strip().lower()
        sym = byte_symbols()
        ids = []
        for w in _PAT.findall(text):
            w = "".join(sym[b] for b in w.encode("utf-8"))
            ids.extend(self.encoder[p] for p in self._bpe(w))
        return ids

    def tokenize(self, texts: Union[str, Sequence[str]], context_length: int = 77) -> np.ndarray:
        """clip.tokenize: [SOT] + ids + [EOT], zero-padded to context_length (int64)."""
        if isinstance(texts, str):
            texts = [texts]
        out = np.zeros((len(texts), context_length), dtype=np.int64)
        for i, t in enumerate(texts):
            ids = [self.sot] + self.encode(t) + [self.eot]
            if len(ids) > context_length:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            out[i, : len(ids)] = ids
        return out


def class_prompts(class_names: Sequence[str], template: str = "A photo of a {} in the scene") -> List[str]:
    """cat_seg_predictor.py:196-201 (first alias before ', ') with the single template (:84-85)."""
    return [template.format(n.split(", ")[0] if ", " in n else n) for n in class_names]
