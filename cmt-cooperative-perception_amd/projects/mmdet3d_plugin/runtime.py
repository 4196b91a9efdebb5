"""Numerics policy of the native path.

The reference computes every projection / MLP / conv in fp32 and only the
cross-attention core in fp16 (FlashAttention with auto_fp16,
models/utils/attention.py:46,57; the head stays fp32 through
custom_fp16=dict(pts_bbox_head=False), e.g.
configs/CMT_Nuscenes/lidar/cmt_lidar_voxel0075_cbgs.py:284-286).

Policies (``set_precision`` / env ``CMT_PRECISION``):
  'ref'  -- the reference's numerics: GEMMs on the exact-f32 MFMA
            (v_mfma_f32_32x32x2_f32), self-attention core in exact f32
            (nn.MultiheadAttention), cross-attention core in fp16 with fp32
            accumulation and an fp16-rounded output (flash-attn 0.2.2).
  'fp16' -- GEMMs and attention in fp16 MFMA (fp32 accumulate).
  'bf16' -- GEMMs and attention in bf16 MFMA (fp32 accumulate).
Activations between kernels stay fp32 in HBM in every policy; K/V/Q for the
attention kernels are written by the projection epilogue in the attention
dtype.
"""
import os
from dataclasses import dataclass

import torch

__all__ = ["Precision", "get_precision", "set_precision", "PRECISIONS"]


@dataclass(frozen=True)
class Precision:
    name: str
    gemm: torch.dtype          # GEMM compute dtype (weights packed to it)
    attn: torch.dtype          # cross-attention core dtype
    self_attn: torch.dtype     # self-attention core dtype
    round_cross_out: bool      # round the cross-attention output to ``attn``


PRECISIONS = {
    "ref": Precision("ref", torch.float32, torch.float16, torch.float32, True),
    "fp16": Precision("fp16", torch.float16, torch.float16, torch.float16, False),
    "bf16": Precision("bf16", torch.bfloat16, torch.bfloat16, torch.bfloat16, False),
}

_current = PRECISIONS[os.environ.get("CMT_PRECISION", "ref")]


def get_precision(override=None):
    if override is None:
        return _current
    if isinstance(override, Precision):
        return override
    return PRECISIONS[override]


def set_precision(name):
    global _current
    _current = PRECISIONS[name] if isinstance(name, str) else name
    return _current
