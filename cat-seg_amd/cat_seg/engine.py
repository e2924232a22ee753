"""MI355X execution engine of the CAT-Seg dense-inference path.

`CatSegEngine` owns the device-resident, kernel-ready weights and drives the HIP
kernels of libcatseg_hip.so (through `ops`) for:

  * the CLIP ViT dense image encoder + hooks        (model_vpt.py:288-314, cat_seg_model.py:84-87)
  * the CLIP text encoder / cached class embeddings (model_vpt.py:421-438, cat_seg_predictor.py:190-224)
  * the Aggregator: cost volume, top-k, corr_embed, Swin + class-attention layers,
    guided upsampler                                 (model.py:683-725)
  * pre/post-processing of CATSeg.forward (eval)     (cat_seg_model.py:147-155,220-229)

Layouts (device, row-major, channels-last):
  ViT residual stream x      fp32 [B*L][width]        (L = 1 + grid^2, token-major per image)
  cost embedding X            act  [B*T*HW][128]       (image, class, pixel) rows
  decoder maps                act  [B*T][h][w][c]      NHWC
  logits                      fp32 [B][T0][96][96]
`act` is bf16 (MFMA bf16, fp32 accumulate) or fp32 (exact-f32 MFMA) — the engine dtype.

Algebraic savings taken (exact in real arithmetic):
  * guidance halves of the Swin / class-attention q,k projections are computed once
    per image / per class and added in the GEMM epilogue;
  * class-attention padding rows: constant K/V contributions, their own rows skipped;
  * forward_dense: the dead q/k projections of the last ViT block are skipped;
  * the decoder guidance concat and repeat over classes are read in place by the conv.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import ops
from . import _lib as L
from ._lib import rowmap
from .arch import CatSegArch
from .weights import AGG, CLIP

_f32 = torch.float32


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class _NS(dict):
    __getattr__ = dict.__getitem__


class CatSegEngine:
    def __init__(self, arch: CatSegArch, state_dict: Dict[str, torch.Tensor], dtype=torch.bfloat16,
                 device="cuda", vit_fp8: bool = False):
        L.require_gpu()
        if arch.hidden_dim != 128 or arch.nheads != 4:
            raise NotImplementedError("HIP path: hidden_dim 128 / 4 heads only")
        if arch.attention_type not in ("linear", "full"):     # AttentionLayer (model.py:331-336)
            raise NotImplementedError(f"ATTENTION_TYPE {arch.attention_type!r}")
        if arch.prompt_length > 0 and arch.prompt_depth < arch.vision_layers:
            # every vision block drops PROMPT_LENGTH rows after CLS (model_vpt.py:213-214, 238-239) but only
            # the first PROMPT_DEPTH insert them (:258-259): past the depth the reference drops patch tokens
            raise NotImplementedError("visual prompt tuning needs PROMPT_DEPTH >= the vision layer count "
                                      "(the reference's blocks past the depth drop patch tokens)")
        self.arch = arch
        self._cache = {}
        self.dt = dtype
        self.fused_swin = True          # bf16: fused norm1 + q/k/v + window attention (A/B switch)
        self.fused_class = True         # bf16: fused norm1 + q/k/v + linear class attention (A/B switch)
        self.split_guidance = True      # bf16: decoder conv guidance half once per image (A/B switch)
        self.fused_swin_mlp = True      # bf16: Swin output proj + residual + Mlp(norm2) in one kernel (A/B switch)
        self.fold_upconv = True         # bf16: the Up blocks' ConvTranspose folded into their first conv (A/B switch)
        self.device = torch.device(device)
        # config 5: the CLIP image encoder's block GEMMs (q/k/v, out-proj, c_fc, c_proj) in
        # OCP e4m3 with per-row scales (catseg_gemm_fp8); bf16 engine only
        # vit_fp8: True = all four, or an iterable naming the ones to run in fp8
        names = ("wqkv", "wo", "wfc", "wpr")
        self.vit_fp8_gemms = (names if vit_fp8 is True else tuple(n for n in names if n in vit_fp8)
                              if vit_fp8 else ())
        self.vit_fp8 = bool(self.vit_fp8_gemms)
        if self.vit_fp8 and dtype != torch.bfloat16:
            raise ValueError("vit_fp8 needs the bf16 engine")
        self._text = None
        self.last_corr = self.last_topk = None
        with torch.no_grad():
            self.w = self._prepare(state_dict)

    # ------------------------------------------------------------------ weights
    def _W(self, t):
        return t.detach().to(self.device, self.dt).contiguous()

    def _F(self, t):
        return t.detach().to(self.device, _f32).contiguous()

    def _Q8(self, t):
        """nn.Linear weight [N][K] -> (e4m3 [N][K], fp32 per-row scale [N]), quantized on device."""
        wf = self._F(t)
        q = torch.empty(wf.shape, device=self.device, dtype=torch.float8_e4m3fn)
        sc = torch.empty(wf.shape[0], device=self.device, dtype=_f32)
        ops.quant_fp8_rows(wf, q, sc)
        return q, sc

    def _block(self, sd, p, dense=False, fp8=False, heads=0):
        """One ResidualAttentionBlock's weights.  heads > 0 (bf16 ViT image blocks): the q rows of the
        in-projection (weight and bias) are multiplied by head_dim^-0.5 * log2(e) in fp32 before the
        bf16 / e4m3 rounding, for catseg_attention mode 2 (the scores come out of q.k in log2 units)."""
        width = sd[p + "attn.q_proj_weight"].shape[0]
        b = sd[p + "attn.in_proj_bias"]
        wq = sd[p + "attn.q_proj_weight"]
        if heads and not dense:
            c = (width // heads) ** -0.5 * 1.4426950408889634
            wq = wq.float() * c
            b = torch.cat([b[:width].float() * c, b[width:].float()])
        blk = _NS(
            ln1w=self._F(sd[p + "ln_1.weight"]), ln1b=self._F(sd[p + "ln_1.bias"]),
            wo=self._W(sd[p + "attn.out_proj.weight"]), bo=self._F(sd[p + "attn.out_proj.bias"]),
            ln2w=self._F(sd[p + "ln_2.weight"]), ln2b=self._F(sd[p + "ln_2.bias"]),
            wfc=self._W(sd[p + "mlp.c_fc.weight"]), bfc=self._F(sd[p + "mlp.c_fc.bias"]),
            wpr=self._W(sd[p + "mlp.c_proj.weight"]), bpr=self._F(sd[p + "mlp.c_proj.bias"]),
        )
        wqkv = None if dense else torch.cat([wq.float(), sd[p + "attn.k_proj_weight"].float(),
                                             sd[p + "attn.v_proj_weight"].float()], 0)
        if dense:   # forward_dense: v path only (model_vpt.py:219-240)
            blk["wv"] = self._W(sd[p + "attn.v_proj_weight"])
            blk["bv"] = self._F(b[2 * width:])
        else:
            blk["wqkv"] = self._W(wqkv)
            blk["bqkv"] = self._F(b)
        if fp8:
            g = self.vit_fp8_gemms
            if "wo" in g:
                blk["q8_wo"] = self._Q8(sd[p + "attn.out_proj.weight"])
            if "wfc" in g:
                blk["q8_wfc"] = self._Q8(sd[p + "mlp.c_fc.weight"])
            if "wpr" in g:
                blk["q8_wpr"] = self._Q8(sd[p + "mlp.c_proj.weight"])
            if "wqkv" in g and dense:
                blk["q8_wv"] = self._Q8(sd[p + "attn.v_proj_weight"])
            elif "wqkv" in g:
                blk["q8_wqkv"] = self._Q8(wqkv)
        return blk

    @staticmethod
    def _conv_w(w):      # (co, ci, 3, 3) -> [co][ky][kx][ci] flattened K
        return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)

    @staticmethod
    def _convt_w(w, b):  # ConvTranspose2d (ci, co, k, k) -> GEMM W [(ky, kx, co)][ci], bias per n
        ci, co, k, _ = w.shape
        return w.permute(2, 3, 1, 0).reshape(k * k * co, ci), b.repeat(k * k)

    @staticmethod
    def _upconv_weights(wt, bt, wc):
        """Composite weights of ConvTranspose2d(k=2, s=2) followed by a 3x3 / pad-1 conv (the x half
        of Up's first conv, model.py:546-555) as catseg_upconv3x3 reads them.  wt (ci, m, 2, 2),
        bt (m,), wc (co, m, 3, 3).  The conv tap (dy, dx) at output pixel (2y + a, 2x + b) reads
        ConvTranspose output (2y + a + dy, 2x + b + dx) = source pixel (y + (a+dy)//2, x + (b+dx)//2)
        through kernel entry ((a+dy)%2, (b+dx)%2); summed per source tap in float64.
        Returns the bf16-ready fp32 [4*co][9*ci] (row block 2a+b = parity (a, b)) and the fp32
        tap bias [9][co] = wc[:, :, tap] . bt (the ConvTranspose bias through each conv tap)."""
        ci, m = wt.shape[:2]
        co = wc.shape[0]
        wt64, wc64 = wt.double(), wc.double()
        comp = torch.zeros(4, co, 3, 3, ci, dtype=torch.float64, device=wt64.device)
        for a_ in (0, 1):
            for b_ in (0, 1):
                for dy in (-1, 0, 1):
                    for dx in (-1, 0, 1):
                        sy, sx = (a_ + dy) // 2, (b_ + dx) // 2
                        py, px = (a_ + dy) % 2, (b_ + dx) % 2
                        comp[2 * a_ + b_, :, sy + 1, sx + 1, :] += wc64[:, :, dy + 1, dx + 1] @ wt64[:, :, py, px].t()
        tap_b = torch.einsum("omyx,m->yxo", wc64, bt.double()).reshape(9, co)
        return comp.reshape(4 * co, 9 * ci).float(), tap_b.float()

    def _prepare(self, sd):
        a = self.arch
        w = _NS()
        # ---------------- CLIP visual ----------------
        p = CLIP + "visual."
        W = a.vision_width
        kc = 3 * a.vision_patch ** 2
        kp = _round_up(kc, 64)          # K % 64: the patch GEMM takes the pipelined MFMA kernel
        pw = torch.zeros(W, kp)
        pw[:, :kc] = sd[p + "conv1.weight"].reshape(W, kc)
        w.patch_w, w.patch_k = self._W(pw), kp
        w.pix_mean = self._F(torch.tensor(a.clip_pixel_mean))
        w.pix_std = self._F(torch.tensor(a.clip_pixel_std))
        w.cls = self._F(sd[p + "class_embedding"])
        pos = self._F(sd[p + "positional_embedding"])
        if a.grid != a.pretrain_grid:   # resized_pos_embed (model_vpt.py:316-329), on device
            out = torch.empty(a.grid * a.grid, W, device=self.device)
            ops.bicubic_resize(pos[1:].contiguous(), a.pretrain_grid, W, out, a.grid)
            pos = torch.cat([pos[:1], out], 0).contiguous()
        w.pos = pos
        w.ln_pre = (self._F(sd[p + "ln_pre.weight"]), self._F(sd[p + "ln_pre.bias"]))
        # bf16: the image blocks' q projection carries the softmax scale in log2 units (attention mode 2)
        self.vit_l2s = self.dt == torch.bfloat16 and W // a.vision_heads == 64
        w.vblocks = [self._block(sd, f"{p}transformer.resblocks.{i}.", dense=(i == a.vision_layers - 1),
                                 fp8=self.vit_fp8, heads=a.vision_heads if self.vit_l2s else 0)
                     for i in range(a.vision_layers)]
        w.ln_post = (self._F(sd[p + "ln_post.weight"]), self._F(sd[p + "ln_post.bias"]))
        w.proj_t = self._W(sd[p + "proj"].t())
        # visual prompt tokens (model_vpt.py:252): one fp32 row of P*W per layer
        w.vpt = (self._F(sd[p + "transformer.prompt_tokens"]).reshape(a.prompt_depth, -1).contiguous()
                 if a.vpt else None)
        # ---------------- CLIP text ----------------
        w.tok_emb = self._F(sd[CLIP + "token_embedding.weight"])
        w.tpos = self._F(sd[CLIP + "positional_embedding"])
        w.tblocks = [self._block(sd, f"{CLIP}transformer.resblocks.{i}.") for i in range(a.text_layers)]
        w.ln_final = (self._F(sd[CLIP + "ln_final.weight"]), self._F(sd[CLIP + "ln_final.bias"]))
        w.tproj_t = self._W(sd[CLIP + "text_projection"].t())
        # ---------------- upsamplers (cat_seg_model.py:81-82) ----------------
        for i in (1, 2):
            ww, bb = self._convt_w(sd[f"upsample{i}.weight"], sd[f"upsample{i}.bias"])
            w[f"up{i}_w"], w[f"up{i}_b"] = self._W(ww), self._F(bb)
        # ---------------- Aggregator ----------------
        D = a.hidden_dim
        w.ce_w = self._F(sd[AGG + "conv1.weight"].reshape(D, 49))
        w.ce_b = self._F(sd[AGG + "conv1.bias"])
        w.gp_w = self._W(self._conv_w(sd[AGG + "guidance_projection.0.weight"]))
        w.gp_b = self._F(sd[AGG + "guidance_projection.0.bias"])
        w.dgp = [(self._W(self._conv_w(sd[f"{AGG}decoder_guidance_projection.{i}.0.weight"])),
                  self._F(sd[f"{AGG}decoder_guidance_projection.{i}.0.bias"])) for i in range(2)]
        w.tg_w = self._W(sd[AGG + "text_guidance_projection.0.weight"])
        w.tg_b = self._F(sd[AGG + "text_guidance_projection.0.bias"])
        w.layers = []
        for l in range(a.num_layers):
            sw = f"{AGG}layers.{l}.swin_block."
            lay = _NS(gnw=self._F(sd[sw + "guidance_norm.weight"]), gnb=self._F(sd[sw + "guidance_norm.bias"]))
            for name in ("block_1", "block_2"):
                q = f"{sw}{name}."
                wq, wk = sd[q + "attn.q.weight"], sd[q + "attn.k.weight"]
                lay[name] = _NS(
                    n1w=self._F(sd[q + "norm1.weight"]), n1b=self._F(sd[q + "norm1.bias"]),
                    wqkv=self._W(torch.cat([wq[:, :D], wk[:, :D], sd[q + "attn.v.weight"]], 0)),
                    bqkv=self._F(torch.cat([sd[q + "attn.q.bias"], sd[q + "attn.k.bias"], sd[q + "attn.v.bias"]])),
                    wqk_g=self._W(torch.cat([wq[:, D:], wk[:, D:]], 0)),
                    wproj=self._W(sd[q + "attn.proj.weight"]), bproj=self._F(sd[q + "attn.proj.bias"]),
                    n2w=self._F(sd[q + "norm2.weight"]), n2b=self._F(sd[q + "norm2.bias"]),
                    wfc1=self._W(sd[q + "mlp.fc1.weight"]), bfc1=self._F(sd[q + "mlp.fc1.bias"]),
                    wfc2=self._W(sd[q + "mlp.fc2.weight"]), bfc2=self._F(sd[q + "mlp.fc2.bias"]),
                )
            c = f"{AGG}layers.{l}.attention."
            wq, wk = sd[c + "attention.q.weight"], sd[c + "attention.k.weight"]
            ca = _NS(
                n1w=self._F(sd[c + "norm1.weight"]), n1b=self._F(sd[c + "norm1.bias"]),
                wqkv=self._W(torch.cat([wq[:, :D], wk[:, :D], sd[c + "attention.v.weight"]], 0)),
                bqkv=self._F(torch.cat([sd[c + "attention.q.bias"], sd[c + "attention.k.bias"],
                                        sd[c + "attention.v.bias"]])),
                wqk_t=self._W(torch.cat([wq[:, D:], wk[:, D:]], 0)),
                n2w=self._F(sd[c + "norm2.weight"]), n2b=self._F(sd[c + "norm2.bias"]),
                w0=self._W(sd[c + "MLP.0.weight"]), b0=self._F(sd[c + "MLP.0.bias"]),
                w2=self._W(sd[c + "MLP.2.weight"]), b2=self._F(sd[c + "MLP.2.bias"]),
            )
            if a.pad_len > 0:
                ca["kpad"], ca["vpad"] = self._pad_kv(ca, sd[c + "padding_tokens"].reshape(1, D),
                                                      sd[c + "padding_guidance"].reshape(1, -1))
            lay["ca"] = ca
            w.layers.append(lay)
        w.dec = []
        for i in (1, 2):
            q = f"{AGG}decoder{i}."
            ww, bb = self._convt_w(sd[q + "up.weight"], sd[q + "up.bias"])
            cu = sd[q + "up.weight"].shape[1]
            c0 = sd[q + "conv.double_conv.0.weight"]
            upc_w, upc_tb = self._upconv_weights(sd[q + "up.weight"], sd[q + "up.bias"], c0[:, :cu])
            w.dec.append(_NS(
                upc_w=self._W(upc_w), upc_tb=self._F(upc_tb),
                up_w=self._W(ww), up_b=self._F(bb), up_c=cu,
                c0=self._W(self._conv_w(c0)),
                # [x | g] split of the first conv (model.py:551-554): the guidance half runs
                # once per image (fp32, catseg_conv3x3_partial), the class half per slice
                c0_x=self._W(self._conv_w(c0[:, :cu])), c0_g=self._F(self._conv_w(c0[:, cu:])),
                g0=(self._F(sd[q + "conv.double_conv.1.weight"]), self._F(sd[q + "conv.double_conv.1.bias"])),
                c3=self._W(self._conv_w(sd[q + "conv.double_conv.3.weight"])),
                g3=(self._F(sd[q + "conv.double_conv.4.weight"]), self._F(sd[q + "conv.double_conv.4.bias"])),
            ))
        hw = sd[AGG + "head.weight"]            # (1, C, 3, 3) -> [ky][kx][c]
        w.head_w = self._F(hw[0].permute(1, 2, 0).reshape(-1))
        w.head_b = float(sd[AGG + "head.bias"].reshape(-1)[0])
        return w

    def _pad_kv(self, ca, pad_tok, pad_guid):
        """Constant K/V projections of the learned class padding (model.py:397-410)."""
        dev, D = self.device, self.arch.hidden_dim
        x = pad_tok.to(dev, _f32).contiguous()
        h = torch.empty(1, D, device=dev, dtype=self.dt)
        ops.layernorm(x, ca.n1w, ca.n1b, h)
        g = pad_guid.to(dev, self.dt).contiguous()
        tg = torch.empty(1, 2 * D, device=dev, dtype=_f32)
        ops.gemm(g, ca.wqk_t, tg)
        qkv = torch.empty(1, 3 * D, device=dev, dtype=_f32)
        ops.gemm(h, ca.wqkv, qkv, bias=ca.bqkv, add=tg, add_ncols=2 * D)
        return qkv[0, D:2 * D].contiguous(), qkv[0, 2 * D:].contiguous()

    def _class_attn(self, qkv, X, Y, *, B, T, HW, n_pad, ca):
        """Y = X + AttentionLayer's attention over the classes (model.py:331-334,352): LinearAttention or,
        for ATTENTION_TYPE "full", FullAttention.  qkv: the fused [q | k | v] projection rows."""
        a, D = self.arch, self.arch.hidden_dim
        kw = dict(B=B, T=T, HW=HW, n_heads=a.nheads, head_dim=D // a.nheads, n_pad=n_pad,
                  k_pad=ca.get("kpad"), v_pad=ca.get("vpad"))
        if a.attention_type == "full":
            return ops.full_attention(qkv, X, Y, **kw)
        return ops.linear_attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], X, Y, **kw)

    # ------------------------------------------------------------------ shared transformer block
    class _Fp8Linear:
        """Per-row e4m3 quantization of the activation rows, then catseg_gemm_fp8 (config 5)."""

        def __init__(self, M, width, dev):
            self.a8 = torch.empty(M, 4 * width, device=dev, dtype=torch.float8_e4m3fn)
            self.sa = torch.empty(M, device=dev, dtype=_f32)

        def __call__(self, a, wq, out, **kw):
            a8 = self.a8[:, :a.shape[1]]
            ops.quant_fp8_rows(a, a8, self.sa)
            ops.gemm_fp8(a8, self.sa, wq[0], wq[1], out, **kw)
            return out

        def ln(self, x, g, b, wq, out, **kw):
            """LayerNorm straight to e4m3 rows, then the GEMM (no bf16 round trip)."""
            a8 = self.a8[:, :x.shape[1]]
            ops.layernorm_fp8(x, g, b, a8, self.sa)
            ops.gemm_fp8(a8, self.sa, wq[0], wq[1], out, **kw)
            return out

    def _ln_linear(self, fp8_lin, x, g, b, h, blk, name, out, **kw):
        """LN(x) -> linear; fp8 GEMMs take the LayerNorm output as e4m3 rows directly."""
        if fp8_lin is not None and "q8_" + name in blk:
            return fp8_lin.ln(x, g, b, blk["q8_" + name], out, **kw)
        ops.layernorm(x, g, b, h)
        return self._linear(fp8_lin, h, blk, name, out, **kw)

    def _linear(self, fp8_lin, a, blk, name, out, **kw):
        if fp8_lin is not None and "q8_" + name in blk:
            return fp8_lin(a, blk["q8_" + name], out, **kw)
        return ops.gemm(a, blk[name], out, **kw)

    def _resblocks(self, x, blocks, n_seq, seq_len, n_heads, causal, hooks_at=(), hooks=None, fp8=False, l2s=False,
                   prompts=None):
        """ResidualAttentionBlock.forward over a stack (model_vpt.py:208-217, 256-266).  l2s: the blocks'
        q projections carry scale * log2(e) (_block heads > 0): attention mode 2."""
        M, width = x.shape
        dt, dev = self.dt, self.device
        h = torch.empty(M, width, device=dev, dtype=dt)
        qkv = torch.empty(M, 3 * width, device=dev, dtype=dt)
        o = torch.empty(M, width, device=dev, dtype=dt)
        u = torch.empty(M, 4 * width, device=dev, dtype=dt)
        f8 = self._Fp8Linear(M, width, dev) if fp8 else None
        fresh = False
        for i, blk in enumerate(blocks):
            if prompts is not None and i < self.arch.prompt_depth:
                prompts(i, x)                        # this block's visual prompt rows (model_vpt.py:258-259)
            self._ln_linear(f8, x, blk.ln1w, blk.ln1b, h, blk, "wqkv", qkv, bias=blk.bqkv)
            ops.attention(qkv[:, :width], qkv[:, width:2 * width], qkv[:, 2 * width:], o,
                          n_seq=n_seq, seq_len=seq_len, n_heads=n_heads, head_dim=width // n_heads,
                          scale=(width // n_heads) ** -0.5, causal=causal, mode=2 if l2s else 0)
            x_new = torch.empty_like(x) if fresh else x
            self._linear(f8, o, blk, "wo", x_new, bias=blk.bo, res=x)
            x = x_new
            self._ln_linear(f8, x, blk.ln2w, blk.ln2b, h, blk, "wfc", u, bias=blk.bfc, act=L.ACT_QUICKGELU)
            self._linear(f8, u, blk, "wpr", x, bias=blk.bpr, res=x)
            fresh = i in hooks_at
            if fresh:
                hooks.append(x)
        return x

    # ------------------------------------------------------------------ text
    def encode_text(self, tokens: torch.Tensor, truncate: bool = True) -> torch.Tensor:
        """CLIP.encode_text + L2 norm (cat_seg_predictor.py:214-216).  tokens (T, ctx) int.

        truncate: run the text transformer on the first max_t(argmax tokens[t]) + 1 positions only
        (SURVEY Appendix B #6).  The blocks are causal (model_vpt.py:400-406) and only the EOT row
        (the argmax id, :436) is read, so positions after the last EOT never reach the output; the
        CLIP prompts end by position 14 of 77.  Every kernel computes a row from the same keys /
        weights in the same order either way, so the embeddings are bit-identical (tested)."""
        a, dev = self.arch, self.device
        if truncate:
            last = int(torch.as_tensor(tokens).argmax(dim=1).max()) + 1
            tokens = torch.as_tensor(tokens)[:, :last]
        tokens = tokens.to(dev, torch.int32).contiguous()
        n, ctx = tokens.shape
        TW = a.text_width
        x = torch.empty(n * ctx, TW, device=dev, dtype=_f32)
        ops.token_embed(tokens, self.w.tok_emb, self.w.tpos[:ctx].contiguous(), x)
        x = self._resblocks(x, self.w.tblocks, n, ctx, a.text_heads, causal=True)
        e = torch.empty(n, TW, device=dev, dtype=_f32)
        ops.eot_gather(x, tokens, e)
        h = torch.empty(n, TW, device=dev, dtype=self.dt)
        ops.layernorm(e, *self.w.ln_final, h)
        t = torch.empty(n, a.embed_dim, device=dev, dtype=_f32)
        ops.gemm(h, self.w.tproj_t, t)
        out = torch.empty_like(t)
        ops.l2normalize(t, out)
        return out

    def text_source(self):
        """The class-embedding tensor the current set_text() call was given (None before any)."""
        return None if self._text is None else self._text.src

    @property
    def n_classes(self) -> int:
        """T0, the class count of the current set_text() (the logits' channel count)."""
        if self._text is None:
            raise RuntimeError("set_text() / encode_text() must run first")
        return int(self._text.T)

    def set_text(self, text: torch.Tensor):
        """Cache the per-class-set terms (the predictor's eval cache, cat_seg_predictor.py:191-192,221-222).
        text: (T, C_o) or (T, 1, C_o) L2-normalized class embeddings."""
        dev, dt, D = self.device, self.dt, self.arch.hidden_dim
        t = text.reshape(text.shape[0], -1).to(dev, _f32).contiguous()
        T = t.shape[0]
        txn = torch.empty(T, t.shape[1], device=dev, dtype=dt)
        ops.l2normalize(t, txn)                           # correlation's F.normalize (model.py:650)
        tg = torch.empty(T, D, device=dev, dtype=dt)       # text_guidance_projection (model.py:712-715)
        ops.gemm(txn, self.w.tg_w, tg, bias=self.w.tg_b, act=L.ACT_RELU)
        tgqk, tgkt = [], []
        for lay in self.w.layers:
            o = torch.empty(T, 2 * D, device=dev, dtype=dt)
            ops.gemm(tg, lay.ca.wqk_t, o)
            tgqk.append(o)
            if dt == torch.bfloat16 and T <= self.arch.pad_len:   # the fused class attention's k half, transposed
                tgkt.append(ops.class_attention_kt(o, T))
        self._text = _NS(T=T, txn=txn, tgqk=tgqk, tgkt=tgkt or None, src=text)

    # ------------------------------------------------------------------ image encoder
    def embed_image(self, raw: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
        """cat_seg_model.py:149-154 + VisualTransformer.forward up to the transformer (model_vpt.py:288-300):
        normalize, pad, resize, patch conv, CLS + pos, ln_pre.  Returns fp32 (B*(1+grid^2), width) rows."""
        a, dev, dt, w = self.arch, self.device, self.dt, self.w
        B = raw.shape[0]
        G2 = a.grid * a.grid
        W = a.vision_width
        cols = torch.empty(B * G2, w.patch_k, device=dev, dtype=dt)
        ops.preprocess_im2col(raw, sizes, mean=w.pix_mean, std=w.pix_std, res=a.clip_resolution,
                              patch=a.vision_patch, out=cols)
        patches = torch.empty(B * G2, W, device=dev, dtype=_f32)
        ops.gemm(cols, w.patch_w, patches)
        x = torch.empty(B * (G2 + 1), W, device=dev, dtype=_f32)
        ops.vit_embed(patches, w.cls, w.pos, *w.ln_pre, x, B=B, G2=G2, width=W)
        return x

    @property
    def vision_seq_len(self) -> int:
        """Rows per image of the vision residual stream: CLS + grid^2 tokens (+ the PROMPT_LENGTH visual
        prompt rows, kept at the END of each sequence: the blocks mix tokens only through attention,
        which is order-free over keys, so their position changes no result beyond summation order)."""
        a = self.arch
        return a.grid * a.grid + 1 + a.vpt

    def _vpt_rows(self, x, B):
        """Visual prompt tuning (model_vpt.py:255-265): the (B*(1+HW), W) embedded rows moved into a
        (B*(1+HW+P), W) stream, and the prompt writer run before each block i < PROMPT_DEPTH (the
        reference's cat after CLS + drop after the block; the rows of a block's prompts are rewritten
        by the next block's, so nothing is dropped here).  Both copies are catseg_gather_rows."""
        a, dev, W, P = self.arch, self.device, self.arch.vision_width, self.arch.vpt
        L0 = a.grid * a.grid + 1
        Ls = L0 + P
        xs = torch.empty(B * Ls, W, device=dev, dtype=_f32)
        key = ("vpt_idx", B)
        if key not in self._cache:
            self._cache[key] = (torch.arange(B, device=dev, dtype=torch.int32),
                                torch.zeros(B, device=dev, dtype=torch.int32))
        ar, zero = self._cache[key]
        ops.gather_rows(x.view(B, L0 * W), ar, xs.view(B, Ls * W)[:, :L0 * W])

        def write(i, stream_rows):
            ops.gather_rows(self.w.vpt[i:i + 1], zero, stream_rows.view(B, Ls * W)[:, L0 * W:])
        return xs, write

    def embed_text(self, tokens: torch.Tensor) -> torch.Tensor:
        """CLIP.encode_text up to the transformer (model_vpt.py:421-427): token + positional embedding.
        tokens (n, ctx) int32 on the device.  Returns fp32 (n*ctx, text_width) rows."""
        n, ctx = tokens.shape
        x = torch.empty(n * ctx, self.arch.text_width, device=self.device, dtype=_f32)
        ops.token_embed(tokens, self.w.tok_emb, self.w.tpos[:ctx].contiguous(), x)
        return x

    def encode_image(self, raw: torch.Tensor, sizes: torch.Tensor):
        """Pre-processing + CLIP dense encoder + hooks.  raw (B,3,Hp,Wp) fp32 0-255 on device,
        sizes (B,2) int32 valid (h, w).  Returns feats fp32 (B*L, C_o), [hook0, hook1] fp32 (B*L, W)."""
        a, dev, dt, w = self.arch, self.device, self.dt, self.w
        B = raw.shape[0]
        Lt = self.vision_seq_len
        W = a.vision_width
        x = self.embed_image(raw, sizes)
        vpt = None
        if a.vpt:
            x, vpt = self._vpt_rows(x, B)
        hooks: List[torch.Tensor] = []
        x = self._resblocks(x, w.vblocks[:-1], B, Lt, a.vision_heads, False,
                            hooks_at=set(a.hook_layers), hooks=hooks, fp8=self.vit_fp8, l2s=self.vit_l2s,
                            prompts=vpt)
        if a.vision_layers - 1 in a.hook_layers:
            raise NotImplementedError("hook on the dense block")
        # forward_dense (model_vpt.py:219-240)
        blk = w.vblocks[-1]
        M = B * Lt
        f8 = self._Fp8Linear(M, W, dev) if self.vit_fp8 else None
        h = torch.empty(M, W, device=dev, dtype=dt)
        v = torch.empty(M, W, device=dev, dtype=dt)
        self._ln_linear(f8, x, blk.ln1w, blk.ln1b, h, blk, "wv", v, bias=blk.bv)
        vo = torch.empty(M, W, device=dev, dtype=_f32)
        self._linear(f8, v, blk, "wo", vo, bias=blk.bo, add=x, addmap=rowmap(d1=Lt, s1=Lt))   # + x[:1] (CLS residual)
        u = torch.empty(M, 4 * W, device=dev, dtype=dt)
        self._ln_linear(f8, vo, blk.ln2w, blk.ln2b, h, blk, "wfc", u, bias=blk.bfc, act=L.ACT_QUICKGELU)
        self._linear(f8, u, blk, "wpr", vo, bias=blk.bpr, res=vo)
        ops.layernorm(vo, *w.ln_post, h)                                        # ln_post (all tokens)
        feats = torch.empty(M, a.embed_dim, device=dev, dtype=_f32)
        ops.gemm(h, w.proj_t, feats)                                           # @ proj
        return feats, hooks

    # ------------------------------------------------------------------ head
    def head_logits(self, raw: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
        """cat_seg_model.py:155-188 -> Aggregator.forward (model.py:683-725).
        Returns fp32 logits (B, T0, 4*grid, 4*grid)."""
        if self._text is None:
            raise RuntimeError("set_text() / encode_text() must run before the image forward")
        feats, hooks = self.encode_image(raw, sizes)
        res3, res4, res5 = self.guidance(feats, hooks)
        return self.aggregate(feats, res3, res4, res5)

    def _fold_ok(self, i, Hc, gch):
        """Whether Up block i runs catseg_upconv3x3 (the ConvTranspose folded into its conv)."""
        if not (self.fold_upconv and self.split_guidance and self.dt == torch.bfloat16 and (Hc * Hc) % 64 == 0
                and gch in (16, 32)):
            return False
        dec = self.w.dec[i]
        cin, cout = dec.upc_w.shape[1] // 9, dec.c0.shape[0]
        return (i == 1 and cin == 64 and cout == 32 and Hc == 48) or (i == 0 and cin == 128 and cout == 64 and Hc == 24)

    def guidance(self, feats, hooks):
        """res3 / res4 / res5 guidance maps, NHWC in the engine dtype (cat_seg_model.py:178-186):
        res3 = dense tokens w/o CLS, res4/res5 = ConvTranspose2d(k=s=2/4) of the hook tokens."""
        a, dev, dt, w = self.arch, self.device, self.dt, self.w
        G = a.grid
        HW = G * G
        Ls = self.vision_seq_len
        B = feats.shape[0] // Ls
        drop_cls = rowmap(d1=HW, s1=Ls, d2=1, m2=HW, s2=1, off=1)
        res3 = torch.empty(B * HW, a.embed_dim, device=dev, dtype=dt)
        ops.convert(feats, res3, inmap=drop_cls)
        res45 = []
        for i, (k, cout) in enumerate(((2, a.decoder_guidance_dims[0]), (4, a.decoder_guidance_dims[1]))):
            hk = torch.empty(B * HW, a.vision_width, device=dev, dtype=dt)
            ops.convert(hooks[i], hk, inmap=drop_cls)
            r = torch.empty(B * HW * k * k, cout, device=dev, dtype=dt)
            ops.gemm(hk, w[f"up{i + 1}_w"], r, bias=w[f"up{i + 1}_b"], store=(k, G, G, cout))
            res45.append(r)
        return res3, res45[0], res45[1]

    def aggregate(self, feats, res3, res4, res5) -> torch.Tensor:
        """Aggregator.forward (model.py:683-725) on engine-layout inputs: feats fp32 (B*(1+HW), C_o)
        dense CLIP tokens, res3 (B*HW, C_o), res4 (B*4HW, 256), res5 (B*16HW, 128) NHWC.
        Returns fp32 logits (B, T0, 4G, 4G)."""
        if self._text is None:
            raise RuntimeError("set_text() / encode_text() must run before the aggregator")
        a, dev, dt, w, tx = self.arch, self.device, self.dt, self.w, self._text
        G = a.grid
        HW = G * G
        Lt = self.vision_seq_len
        B = feats.shape[0] // Lt
        D = a.hidden_dim
        Co = a.embed_dim
        res45 = [res4, res5]
        drop_cls = rowmap(d1=HW, s1=Lt, d2=1, m2=HW, s2=1, off=1)
        # ---- cost volume (model.py:648-652) ----
        fn = torch.empty(B * HW, Co, device=dev, dtype=dt)
        ops.l2normalize(feats, fn, inmap=drop_cls)
        T0 = tx.T
        corr = torch.empty(T0, B * HW, device=dev, dtype=_f32)
        ops.gemm(tx.txn, fn, corr)                         # corr[t][b*HW + p]
        classes = None
        T = T0
        if a.pad_len > 0 and T0 > a.pad_len:               # top-k truncation (model.py:694-702)
            T = a.pad_len
            classes = torch.empty(B, T, device=dev, dtype=torch.int32)
            ops.topk_classes(corr, t_stride=B * HW, b_stride=HW, B=B, T=T0, HW=HW, k=T, out=classes)
        # the last call's cost volume [T0][B*HW] and top-k selection (B, pad_len) stay readable
        # (device tensors, no copy): parity tests check the selection against the fp32 margins
        self.last_corr, self.last_topk = corr, classes
        S = B * T
        R = S * HW
        X = torch.empty(R, D, device=dev, dtype=dt)
        ops.corr_embed(corr, t_stride=B * HW, b_stride=HW, B=B, T=T, H=G, W=G, weight=w.ce_w, bias=w.ce_b,
                       out=X, classes=classes)
        # ---- guidance projections (model.py:706-711) ----
        G3 = torch.empty(B * HW, a.appearance_guidance_proj_dim, device=dev, dtype=dt)
        ops.conv3x3(res3, w.gp_w, G3, S=B, H=G, W=G, c1=Co, bias=w.gp_b, act=L.ACT_RELU)
        GD = []
        for i, (src, cin) in enumerate(zip(res45, a.decoder_guidance_dims)):
            k = 2 ** (i + 1)
            g = torch.empty(B * HW * k * k, a.decoder_guidance_proj_dims[i], device=dev, dtype=dt)
            ops.conv3x3(src, w.dgp[i][0], g, S=B, H=G * k, W=G * k, c1=cin, bias=w.dgp[i][1], act=L.ACT_RELU)
            GD.append(g)
        # ---- class-attention pooling geometry (ClassTransformerLayer.pool, model.py:358,374-385) ----
        H_, W_ = a.feature_resolution
        ph, pw = a.pooling_size
        pooled = (ph, pw) != (1, 1)
        HWc = (H_ // ph) * (W_ // pw)          # pixels per class-attention slice
        # ---- text guidance terms per class (gathered per image after top-k) ----
        if classes is not None:
            tgqk, tgkt = [], []
            idx = classes.reshape(-1).contiguous()
            for t in tx.tgqk:
                o = torch.empty(S, 2 * D, device=dev, dtype=dt)
                ops.gather_rows(t, idx, o)
                tgqk.append(o)
                if dt == torch.bfloat16:
                    tgkt.append(ops.class_attention_kt(o, T, B))
            tmap = rowmap(d1=HWc)
            tg_bstride = T
        else:
            tgqk, tgkt = tx.tgqk, tx.tgkt
            tmap = rowmap(d1=HWc, m1=T)
            tg_bstride = 0
        # ---- aggregation layers (model.py:717-718) ----
        qkv = torch.empty(R, 3 * D, device=dev, dtype=dt)
        o = torch.empty(R, D, device=dev, dtype=dt)
        Y = torch.empty(R, D, device=dev, dtype=dt)
        gn = torch.empty(B * HW, D, device=dev, dtype=dt)
        gqk = torch.empty(B * HW, 2 * D, device=dev, dtype=dt)
        if pooled:
            Rp = S * HWc
            Xp = torch.empty(Rp, D, device=dev, dtype=dt)
            Yp = torch.empty(Rp, D, device=dev, dtype=dt)
        ws = a.window_size
        shift2 = ws // 2
        if min(H_, W_) <= ws:   # model.py:146-149
            ws, shift2 = min(H_, W_), 0
        nwin = (H_ // ws) * (W_ // ws)
        # the fused window kernel covers CAT-Seg's geometry (24x24 map, 12x12 windows, 4 x 32 heads)
        fused_swin = (self.fused_swin and dt == torch.bfloat16 and (H_, W_, ws) == (24, 24, 12)
                      and a.nheads == 4 and D == 128)
        gmap = rowmap(d1=T * HW, s1=HW, d2=1, m2=HW, s2=1)     # (b, t, p) -> (b, p)
        # the fused class attention holds one pixel's T <= 256 class rows on chip (pad_len bounds T)
        fused_class = (self.fused_class and dt == torch.bfloat16 and a.nheads == 4 and D == 128 and T <= 256 and
                       a.attention_type == "linear")
        n_pad = a.pad_len - T if a.pad_len > 0 and T < a.pad_len else 0
        for l, lay in enumerate(w.layers):
            ops.layernorm(G3, lay.gnw, lay.gnb, gn)           # guidance_norm, once per image
            for name, shift in (("block_1", 0), ("block_2", shift2)):
                blk = lay[name]
                ops.gemm(gn, blk.wqk_g, gqk)                   # W_g . LN(g): per image
                if fused_swin:
                    # norm1 + q/k/v (+ guidance half) + window attention in one kernel per window
                    ops.swin_window_attention(X, (blk.n1w, blk.n1b), blk.wqkv, blk.bqkv, gqk, gmap, o, S=S,
                                              img_hw=(H_, W_), window=ws, shift=shift, n_heads=a.nheads,
                                              head_dim=D // a.nheads, scale=(D // a.nheads) ** -0.5)
                else:
                    # LN1 + [q|k|v] projection + guidance half, one pass over X
                    ops.rows_gemm(X, blk.wqkv, qkv, ln=(blk.n1w, blk.n1b), bias=blk.bqkv, add=gqk, addmap=gmap,
                                  add_ncols=2 * D)
                    ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, n_seq=S * nwin,
                                  seq_len=ws * ws, n_heads=a.nheads, head_dim=D // a.nheads,
                                  scale=(D // a.nheads) ** -0.5, mode=1, img_hw=(H_, W_), window=ws, shift=shift)
                if self.fused_swin_mlp and dt == torch.bfloat16 and D == 128 and blk.wfc1.shape[0] == 512:
                    # x = shortcut + proj(attn); x = x + Mlp(norm2(x)) in one pass (x1 on chip)
                    ops.swin_proj_mlp(o, X, blk.wproj, blk.bproj, blk.wfc1, blk.bfc1, blk.wfc2, blk.bfc2, X,
                                      ln=(blk.n2w, blk.n2b))
                else:
                    ops.rows_gemm(o, blk.wproj, X, bias=blk.bproj, res=X)      # x = shortcut + proj(attn)
                    ops.rows_mlp(X, blk.wfc1, blk.bfc1, blk.wfc2, X, ln=(blk.n2w, blk.n2b), b2=blk.bfc2,
                                 act=L.ACT_GELU, res=X)                          # x = x + Mlp(norm2(x))
            ca = lay.ca
            if not pooled:
                if fused_class:
                    ops.class_attention(X, (ca.n1w, ca.n1b), ca.wqkv, ca.bqkv, tgqk[l], Y, B=B, T=T, HW=HW,
                                        n_heads=a.nheads, head_dim=D // a.nheads, tg_bstride=tg_bstride,
                                        n_pad=n_pad, k_pad=ca.get("kpad"), v_pad=ca.get("vpad"),
                                        tgk_t=tgkt[l] if tgkt else None)
                else:
                    ops.rows_gemm(X, ca.wqkv, qkv, ln=(ca.n1w, ca.n1b), bias=ca.bqkv, add=tgqk[l], addmap=tmap,
                                  add_ncols=2 * D)
                    self._class_attn(qkv, X, Y, B=B, T=T, HW=HW, n_pad=n_pad, ca=ca)
                # x + (x_pool + MLP(norm2(x_pool)))  (model.py:413,423)
                ops.rows_mlp(Y, ca.w0, ca.b0, ca.w2, X, ln=(ca.n2w, ca.n2b), b2=ca.b2, act=L.ACT_RELU, res=Y,
                             res2=X, ref_rows=B * HW * (T + n_pad))
            else:
                # x_pool = AvgPool(x); x_pool += attn; x_pool += MLP; x += interp_ac(x_pool) (model.py:387-423)
                ops.avgpool_rows(X, Xp, S=S, H=H_, W=W_, C=D, pool=(ph, pw))
                if fused_class:
                    ops.class_attention(Xp, (ca.n1w, ca.n1b), ca.wqkv, ca.bqkv, tgqk[l], Yp, B=B, T=T, HW=HWc,
                                        n_heads=a.nheads, head_dim=D // a.nheads, tg_bstride=tg_bstride,
                                        n_pad=n_pad, k_pad=ca.get("kpad"), v_pad=ca.get("vpad"),
                                        tgk_t=tgkt[l] if tgkt else None)
                else:
                    qkvp = qkv[:Rp]
                    ops.rows_gemm(Xp, ca.wqkv, qkvp, ln=(ca.n1w, ca.n1b), bias=ca.bqkv, add=tgqk[l], addmap=tmap,
                                  add_ncols=2 * D)
                    self._class_attn(qkvp, Xp, Yp, B=B, T=T, HW=HWc, n_pad=n_pad, ca=ca)
                ops.rows_mlp(Yp, ca.w0, ca.b0, ca.w2, Yp, ln=(ca.n2w, ca.n2b), b2=ca.b2, act=L.ACT_RELU, res=Yp)
                ops.upsample_add_rows(Yp, X, S=S, Hp=H_ // ph, Wp=W_ // pw, C=D, H=H_, W=W_)
        del qkv, o, Y, gn, gqk
        # ---- guided upsampler (model.py:674-681, 540-555) ----
        src, Hc, src_gn = X, G, None
        for i, dec in enumerate(w.dec):
            cu = dec.up_c
            Ho = Hc * 2
            cout = dec.c0.shape[0]
            groups = cout // 16
            fold = (self._fold_ok(i, Hc, GD[i].shape[1]) and src.shape[1] * 9 == dec.upc_w.shape[1] and
                    (src_gn is not None) == (i == 1))
            if fold:
                # ConvTranspose + conv over [up | guidance] as one 4-parity conv over the
                # GroupNorm+ReLU'd source (catseg_upconv3x3); guidance half + ConvT bias as addend
                gpart = torch.empty(B * Hc * Hc, 4 * cout, device=dev, dtype=_f32)
                ops.upconv_addend(GD[i], dec.c0_g, dec.upc_tb, gpart, B=B, H2=Ho, W2=Ho)
                tile = ops.upconv3x3_stats_tile()
                ntl = 4 * Hc * Hc // tile
                st = torch.empty(S * ntl * groups * 2, device=dev, dtype=_f32)
                c1 = torch.empty(S * Ho * Ho, cout, device=dev, dtype=dt)
                ops.upconv3x3(src, dec.upc_w, c1, S=S, H=Hc, W=Hc, c1=src.shape[1], gn=src_gn, stats=st,
                              addend=gpart, addend_div=T, ref_convt_out=cu, ref_guid=GD[i].shape[1])
                m1 = torch.empty(S * groups, device=dev, dtype=_f32)
                r1 = torch.empty_like(m1)
                ops.groupnorm_stats(st, S, ntl, groups, tile * 16, m1, r1)
            else:
                up = torch.empty(S * Ho * Ho, cu, device=dev, dtype=dt)
                if src_gn is not None and dt == torch.bfloat16 and tuple(dec.up_w.shape) == (192, 64):
                    # GroupNorm+ReLU of the previous DoubleConv fused into this ConvTranspose
                    ops.convt64_gn(src, dec.up_w, up, HW=Hc * Hc, gn=src_gn, bias=dec.up_b, store=(2, Hc, Hc, cu))
                else:
                    if src_gn is not None:
                        z = torch.empty_like(src)
                        m_, r_, g_, b_, cpg_ = src_gn
                        ops.groupnorm_relu(src, z, S=S, HW=Hc * Hc, C=src.shape[1], cpg=cpg_, mean=m_, rstd=r_,
                                           gamma=g_, beta=b_)
                        src = z
                    if src.shape[1] == 128 and dec.up_w.shape[0] % 128 == 0:
                        ops.rows_gemm(src, dec.up_w, up, bias=dec.up_b, store=(2, Hc, Hc, cu))
                    else:
                        ops.gemm(src, dec.up_w, up, bias=dec.up_b, store=(2, Hc, Hc, cu))
                c1 = torch.empty(S * Ho * Ho, cout, device=dev, dtype=dt)
                gd = GD[i]
                if self.split_guidance and dt == torch.bfloat16 and (cu, Ho) in ((96, 48), (48, 96)) and cout in (64, 32):
                    gpart = torch.empty(B * Ho * Ho, cout, device=dev, dtype=_f32)
                    ops.conv3x3_partial(gd, dec.c0_g, gpart, B=B, H=Ho, W=Ho)
                    kw = dict(S=S, H=Ho, W=Ho, c1=cu, addend=gpart, addend_div=T)
                    wc0 = dec.c0_x
                else:
                    kw = dict(S=S, H=Ho, W=Ho, c1=cu, src2=gd, c2=gd.shape[1], src2_div=T)
                    wc0 = dec.c0
                tile = ops.conv3x3_stats_tile(up, wc0, **kw)
                st = torch.empty(S * (Ho * Ho // tile) * groups * 2, device=dev, dtype=_f32)
                ops.conv3x3(up, wc0, c1, stats=st, **kw)
                m1 = torch.empty(S * groups, device=dev, dtype=_f32)
                r1 = torch.empty_like(m1)
                ops.groupnorm_stats(st, S, Ho * Ho // tile, groups, tile * 16, m1, r1)
            c2 = torch.empty_like(c1)
            kw2 = dict(S=S, H=Ho, W=Ho, c1=cout, gn=(m1, r1, *dec.g0, 16))
            tile = ops.conv3x3_stats_tile(c1, dec.c3, **kw2)
            st = torch.empty(S * (Ho * Ho // tile) * groups * 2, device=dev, dtype=_f32)
            ops.conv3x3(c1, dec.c3, c2, stats=st, **kw2)
            m2 = torch.empty_like(m1)
            r2 = torch.empty_like(m1)
            ops.groupnorm_stats(st, S, Ho * Ho // tile, groups, tile * 16, m2, r2)
            if i == 0:
                src, Hc, src_gn = c2, Ho, (m2, r2, dec.g3[0], dec.g3[1], 16)
            else:
                logits = torch.empty(B, T0, Ho, Ho, device=dev, dtype=_f32)
                if classes is not None:
                    ops.fill(logits, -100.0)
                ops.conv3x3_head(c2, B=B, T=T, H=Ho, W=Ho, C=cout, weight=w.head_w, bias=w.head_b, out=logits,
                                 T_out=T0, classes=classes, gn=(m2, r2, *dec.g3, 16))
        return logits

    # ------------------------------------------------------------------ full eval forward
    def forward(self, raw: torch.Tensor, sizes: torch.Tensor, out_hw, image_hw) -> torch.Tensor:
        """Sigmoid probabilities upsampled to out_hw for every image (cat_seg_model.py:220-229).
        image_hw: the host-side (h, w) of the valid image region, which sem_seg_postprocess crops
        to (one size for the whole batch; CATSeg.forward handles ragged batches per image)."""
        logits = self.head_logits(raw, sizes)
        B, T0, h, w = logits.shape
        H, W = out_hw
        out = torch.empty(B, T0, H, W, device=self.device, dtype=_f32)
        ih, iw = (int(v) for v in image_hw)
        ops.postprocess(logits, out, crop=(min(h, ih), min(w, iw)))
        return out

    # ------------------------------------------------------------------ sliding-window eval
    SLIDE_KERNEL, SLIDE_OVERLAP, SLIDE_OUT = 384, 0.333, 640      # cat_seg_model.py:158-160

    def sliding_logits(self, raw: torch.Tensor, sizes: torch.Tensor, return_crops: bool = False):
        """TEST.SLIDING_WINDOW branch up to the merged probabilities (cat_seg_model.py:156-176,204-213),
        for every image of the batch: 640² resize, Unfold(384, stride 256) tiles + the 384² global
        crop through the head, then sigmoid / Fold / average.  raw (N,3,Hc,Wc) fp32 0-255 canvas,
        sizes (N,2) int32 valid (h, w).  Returns fp32 probabilities (N, T0, 640, 640), and with
        return_crops also the crops' head logits (N*(nb²+1), T0, 96, 96) (what a batch-sharded run
        all-gathers: 640² probabilities are 7x larger)."""
        k, res = self.SLIDE_KERNEL, self.SLIDE_OUT
        stride = int(k * (1 - self.SLIDE_OVERLAP))
        nb = (res - k) // stride + 1
        N = raw.shape[0]
        crops = torch.empty(N * (nb * nb + 1), 3, k, k, device=self.device, dtype=_f32)
        ops.sliding_crops(raw, sizes, crops, out_res=res, kernel=k, stride=stride)
        csz = torch.full((crops.shape[0], 2), k, dtype=torch.int32, device=self.device)
        logits = self.head_logits(crops, csz)                      # (N*(nb²+1), T0, 96, 96)
        merged = torch.empty(N, logits.shape[1], res, res, device=self.device, dtype=_f32)
        ops.sliding_merge(logits, merged, kernel=k, stride=stride, out_res=res)
        return (merged, logits) if return_crops else merged

    def forward_sliding(self, raw: torch.Tensor, sizes: torch.Tensor, out_hw) -> List[torch.Tensor]:
        """Sliding-window probabilities resized to out_hw[n] = (height, width) per image
        (sem_seg_postprocess of the 640² merge, cat_seg_model.py:215-217)."""
        merged = self.sliding_logits(raw, sizes)
        res = self.SLIDE_OUT
        outs = []
        for n, (H, W) in enumerate(out_hw):
            if (H, W) == (res, res):      # same-size bilinear (align_corners=False) is the identity
                outs.append(merged[n])
                continue
            o = torch.empty(1, merged.shape[1], H, W, device=self.device, dtype=_f32)
            ops.resize_bilinear(merged[n:n + 1], o, crop=(res, res))
            outs.append(o[0])
        return outs
