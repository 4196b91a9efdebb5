"""FlashMHA / FlashAttention with the reference's API, computed by the gfx950
attention kernel (cmt_attn_fwd) instead of flash-attn 0.2.2.

Reference: projects/mmdet3d_plugin/models/utils/attention.py
  _in_projection_packed 21-27, FlashAttention 30-92, FlashMHA 95-138.
Numerics: the reference casts q and kv to fp16 (auto_fp16, :46) and returns
fp32 (out_fp32=True).  Here q/k/v are produced by the projection epilogue in
the policy's attention dtype (fp16 under the 'ref' policy) and the output is
fp32.  Masked (key_padding_mask) and causal paths are dead in every reference
config (petr_transformer.py:316 passes key_padding_mask=None) and raise here.
"""
import math

import torch
import torch.nn as nn
from torch.nn.init import constant_, xavier_uniform_

from ... import native
from ...runtime import SPLIT, get_precision, is_split, op_empty
from .packing import PackCache, to_dtype

__all__ = ["FlashAttention", "FlashMHA", "project_attend_project"]


class FlashAttention(nn.Module):
    """Scaled dot-product attention core (attention.py:30-92)."""

    def __init__(self, softmax_scale=None, attention_dropout=0.0, device=None, dtype=None):
        super().__init__()
        self.softmax_scale = softmax_scale
        self.dropout_p = attention_dropout
        self.fp16_enabled = True

    def forward(self, q, kv, causal=False, key_padding_mask=None):
        """q [B, T, H, D], kv [B, S, 2, H, D] -> ([B, T, H, D] fp32, None)."""
        if causal:
            raise NotImplementedError("causal attention is not used by CMT configs")
        if key_padding_mask is not None:
            raise NotImplementedError("key_padding_mask path is dead in CMT configs (petr_transformer.py:316)")
        if self.training and self.dropout_p > 0:
            raise NotImplementedError("FlashAttention attention_dropout > 0: CMT keeps flash-attn's default 0 "
                                      "(attention.py:36); the training core takes dropout only for the "
                                      "self-attention (train_ops.attention dropout_p)")
        B, T, H, D = q.shape
        S = kv.shape[1]
        if D != 32:
            raise NotImplementedError("the gfx950 attention kernel is specialised for head_dim 32")
        adt = q.dtype if q.dtype in (torch.float16, torch.bfloat16) else get_precision().attn
        if q.dtype != adt:
            q16 = torch.empty(q.shape, dtype=adt, device=q.device)
            native.cast(q.contiguous(), q16)
            q = q16
        if kv.dtype != adt:
            kv16 = torch.empty(kv.shape, dtype=adt, device=kv.device)
            native.cast(kv.contiguous(), kv16)
            kv = kv16
        q, kv = q.contiguous(), kv.contiguous()
        out = torch.empty((B, T, H, D), dtype=torch.float32, device=q.device)
        scale = self.softmax_scale if self.softmax_scale is not None else 1.0 / math.sqrt(D)
        native.attention(q, kv, kv, out, B=B, H=H, Nq=T, Nk=S,
                         q_strides=(T * H * D, D, H * D),
                         k_strides=(S * 2 * H * D, D, 2 * H * D),
                         v_strides=(S * 2 * H * D, D, 2 * H * D), v_offset=H * D,
                         o_strides=(T * H * D, H * D), scale=scale)
        return out, None


class FlashMHA(nn.Module):
    """attention.py:95-138.  ``bias`` receives the third positional argument of
    PETRMultiheadFlashAttention (attn_drop, petr_transformer.py:226), so with
    dropout=0.1 the in/out projection biases exist (quirk reproduced)."""

    def __init__(self, embed_dim, num_heads, bias=True, batch_first=True, attention_dropout=0.0, causal=False,
                 device=None, dtype=None, **kwargs):
        assert batch_first
        super().__init__()
        self.embed_dim = embed_dim
        self.causal = causal
        self.bias = bias
        self.num_heads = num_heads
        assert self.embed_dim % num_heads == 0, "self.kdim must be divisible by num_heads"
        self.head_dim = self.embed_dim // num_heads
        assert self.head_dim % 8 == 0 and self.head_dim <= 128, "Only support head_dim <= 128 and divisible by 8"
        self.in_proj_weight = nn.Parameter(torch.empty((3 * embed_dim, embed_dim)))
        if bias:
            self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        else:
            self.register_parameter("in_proj_bias", None)
        self.inner_attn = FlashAttention(attention_dropout=attention_dropout)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bool(bias))
        self._pack = PackCache()
        self._reset_parameters()

    def _reset_parameters(self):
        xavier_uniform_(self.in_proj_weight)
        if self.in_proj_bias is not None:
            constant_(self.in_proj_bias, 0.0)
            constant_(self.out_proj.bias, 0.0)

    def packed(self, prec=None):
        prec = get_precision(prec)
        ps = [self.in_proj_weight, self.out_proj.weight]
        return self._pack.get("w", ps, prec.name, lambda: dict(
            w_in=to_dtype(self.in_proj_weight, prec.gemm), w_out=to_dtype(self.out_proj.weight, prec.gemm)))

    def forward(self, q, k, v, key_padding_mask=None):
        """q [B, T, C], k/v [B, S, C] (fp32) -> ([B, T, C] fp32, None)."""
        if key_padding_mask is not None:
            raise NotImplementedError("key_padding_mask path is dead in CMT configs")
        prec = get_precision()
        pk = self.packed(prec)
        B, T, C = q.shape
        S = k.shape[1]
        qr, kr, vr = (x.reshape(-1, C).contiguous().float() for x in (q, k, v))
        out = project_attend_project(qr, kr, vr, None, None, pk["w_in"], self.in_proj_bias, pk["w_out"],
                                     self.out_proj.bias, None, prec.attn, prec.round_cross_out, B=B, Nq=T, Nk=S,
                                     H=self.num_heads, layout="batch_first")
        return out.view(B, T, C), None


def project_attend_project(q, k, v, q_pos, k_pos, w_in, b_in, w_out, b_out, identity, adt, round_out, *, B, Nq,
                           Nk, H, layout):
    """Shared native path of FlashMHA / PETRMultiheadFlashAttention / mmcv
    MultiheadAttention: packed in-projection (pos add fused), attention core,
    out-projection (+ identity residual fused).  Rows of q/k/v are either
    batch-first (b*S + s) or sequence-first (s*B + b).  Returns fp32 rows."""
    C = q.shape[1]
    D = C // H
    dev = q.device
    split = is_split(w_in)
    proj = []
    for i, (x, pos, n) in enumerate(((q, q_pos, Nq), (k, k_pos, Nk), (v, None, Nk))):
        y = torch.empty((x.shape[0], C), dtype=adt, device=dev)
        w = w_in[i * C:(i + 1) * C]
        if split:
            # split f16 operand of x (+ pos): one native pass writes the pair rows
            xs = op_empty(x.shape[0], C, SPLIT, dev)
            if pos is not None:
                native.add_cast(x.contiguous(), rows=x.shape[0], C=C, Yp=xs, P=pos.contiguous())
            else:
                native.split_rows(x, xs)
            native.gemm(xs, w, y, M=x.shape[0], N=C, K=C, lda=C, ldw=C, ldc=C,
                        bias=None if b_in is None else b_in[i * C:(i + 1) * C])
        else:
            native.gemm(x, w, y, M=x.shape[0], N=C, K=C, lda=x.stride(0), ldw=w.stride(0), ldc=C,
                        bias=None if b_in is None else b_in[i * C:(i + 1) * C], A2=pos,
                        lda2=pos.stride(0) if pos is not None else 0, a2_cols=C if pos is not None else 0)
        proj.append(y)
    o = op_empty(q.shape[0], C, SPLIT if split else torch.float32, dev)

    def strides(n):
        if layout == "batch_first":
            return (n * C, D, C)
        return (C, D, B * C)

    ob, orow = (Nq * C, C) if layout == "batch_first" else (C, B * C)
    native.attention(proj[0], proj[1], proj[2], o, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=strides(Nq),
                     k_strides=strides(Nk), v_strides=strides(Nk), o_strides=(ob, orow), scale=1.0 / math.sqrt(D),
                     round_output=round_out)
    out = torch.empty((q.shape[0], C), dtype=torch.float32, device=dev)
    native.gemm(o, w_out, out, M=o.shape[0], N=C, K=C, lda=C, ldw=native.lstride(w_out), ldc=C, bias=b_out,
                R=identity, ldr=identity.stride(0) if identity is not None else 0)
    return out
