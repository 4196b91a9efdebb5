"""Numerics policy of the native path.

The reference computes every projection / MLP / conv in fp32 and only the
cross-attention core in fp16 (FlashAttention with auto_fp16,
models/utils/attention.py:46,57; the head stays fp32 through
custom_fp16=dict(pts_bbox_head=False), e.g.
configs/CMT_Nuscenes/lidar/cmt_lidar_voxel0075_cbgs.py:284-286).

Policies (``set_precision`` / env ``CMT_PRECISION``):
  'ref'   -- the reference's numerics with fp32-accurate split GEMMs: every
             fp32 GEMM operand is carried as an f16 pair (hi, lo) (``SPLIT``,
             cmt_hip.h CMT_F16P) and multiplied in three f16 MFMA passes
             (hi*hi + lo*hi + hi*lo, fp32 accumulate: per operand an error
             <= max(2^-22 |x|, 2^-25) -- 2^-22 relative for |x| >= ~2^-3, the
             absolute 2^-25 of an f16-subnormal lo below, ~2^-19 relative
             for xavier-scale weights; TF32 would be 2^-11); self-attention core
             in exact f32 (nn.MultiheadAttention); cross-attention core in
             fp16 with fp32 accumulation, P rounded to fp16 and an fp16-rounded
             output (flash-attn 0.2.2 under auto_fp16).
  'exact' -- as 'ref' but the GEMMs on the exact-f32 MFMA
             (v_mfma_f32_32x32x2_f32, 1/16 of the bf16 rate): the yardstick the
             split GEMMs are checked against.
  'fp16'  -- GEMMs and attention in fp16 MFMA (fp32 accumulate).
  'bf16'  -- GEMMs and attention in bf16 MFMA (fp32 accumulate).
Input range of 'ref' and 'fp16': an operand written as f16 (or an f16 pair)
must stay below 65504 in magnitude, where the reference's fp32 GEMMs would
stay finite.  The head checks its external inputs (BEV / image feature maps)
against that limit on every eager forward (``check_f16_range``; skipped while a
graph is being captured, where a host read cannot run) and raises ValueError
pointing at the 'exact' policy.
The residual stream and LayerNorm statistics stay fp32 in every policy; the
producer of each GEMM operand writes it in the policy's operand format, and
K/V/Q for the attention kernels are written by the projection epilogue in the
attention dtype.
"""
import contextlib
import os
from dataclasses import dataclass

import torch

__all__ = ["Precision", "get_precision", "set_precision", "PRECISIONS", "SPLIT", "op_empty", "is_split",
           "Options", "OPTIONS", "options", "check_f16_range", "F16_MAX"]

# Storage dtype of a split operand: 16-bit words, a tensor of logical shape
# [..., C] stored as [..., 2, C] (the C f16 hi values, then the C f16 lo values).
SPLIT = torch.uint16


def is_split(t):
    return t is not None and t.dtype == SPLIT


def op_empty(rows, C, dtype, device, lead=()):
    """An operand buffer of logical shape [*lead, rows, C] in ``dtype`` (SPLIT:
    [*lead, rows, 2, C] 16-bit words)."""
    shape = tuple(lead) + ((rows, 2, C) if dtype == SPLIT else (rows, C))
    return torch.empty(shape, dtype=dtype, device=device)


F16_MAX = 65504.0


def check_f16_range(prec, tensors):
    """Raise ValueError if an external input of an f16-operand policy ('ref',
    'fp16') holds a value the f16 (pair) format cannot carry (|x| > 65504, inf
    or NaN).  One fused max-abs per tensor and ONE host read; a no-op under
    graph capture and for the f32/bf16 policies."""
    ts = [t for t in tensors if t is not None and t.numel()]
    if prec.gemm not in (SPLIT, torch.float16) or not ts:
        return
    if ts[0].is_cuda and torch.cuda.is_current_stream_capturing():
        return
    m = torch.stack([t.detach().abs().amax().float() for t in ts]).max().item()
    if not m <= F16_MAX:   # also catches NaN
        raise ValueError(f"input feature map max |x| = {m} exceeds the f16 operand range ({F16_MAX}) of the "
                         f"'{prec.name}' policy; use set_precision('exact') for such inputs")


@dataclass(frozen=True)
class Precision:
    name: str
    gemm: torch.dtype          # GEMM compute dtype (weights packed to it)
    attn: torch.dtype          # cross-attention core dtype
    self_attn: torch.dtype     # self-attention core dtype
    round_cross_out: bool      # round the cross-attention output to ``attn``
    fold_q: bool = False       # fold scale*log2(e) into the low-precision cross-attention Q
                               # (one more rounding of Q; off where Q must stay the reference's)


PRECISIONS = {
    "ref": Precision("ref", SPLIT, torch.float16, SPLIT, True),
    "exact": Precision("exact", torch.float32, torch.float16, torch.float32, True),
    "fp16": Precision("fp16", torch.float16, torch.float16, torch.float16, False, True),
    "bf16": Precision("bf16", torch.bfloat16, torch.bfloat16, torch.bfloat16, False, True),
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


@dataclass
class Options:
    """Path selections of the head, read ONCE from the environment when this
    module is imported (``options()`` overrides them for a block of code).
    Each selects between two paths that produce the same outputs and that the
    GPU tests run both of."""
    side_stream: bool      # CMT_SIDE_STREAM=0: everything on the caller's stream
    chain: bool            # CMT_CHAIN=0: f16/bf16 decoder as separate GEMM / LayerNorm launches
    bev_pos_cache: bool    # CMT_BEV_POS_CACHE=0: rebuild the BEV position-MLP hidden rows per call
    conv_halo: bool        # CMT_CONV_HALO=0: shared_conv via an NCHW->rows pass + per-tap gathered GEMM instead
                           # of the halo kernel reading the NCHW map (3 split passes at 'ref', 1 at f16 / bf16)
    mlp_fused: bool        # CMT_MLP_FUSED=0: split rv_embedding as two GEMMs (hidden pair rows via HBM)
    chain_combine: bool    # CMT_CHAIN_COMBINE=0: split cross-attention combined by its own launch (pair rows
                           # via HBM) instead of inside chain B1
    rv_geo: bool           # CMT_RV_GEO=0: the camera rows' frustum coordinates and layout pass as launches of
                           # their own instead of inside the one-launch RV position MLP
    train_graph: bool      # CMT_TRAIN_GRAPH=1 (off by default): the training decoder's forward / backward
                           # replayed as HIP graphs instead of issued op by op (train_engine._decoder_t):
                           # host issue 39.2 -> 34.9 ms/step, step rate 27.7 vs 28.8 steps/s (r5ai).
                           # Limits: one capture per DN padding (it follows the GT count; 8 kept), and
                           # a second forward before the first one's backward runs eagerly


def _env_on(name):
    return os.environ.get(name, "1") != "0"


OPTIONS = Options(side_stream=_env_on("CMT_SIDE_STREAM"), chain=_env_on("CMT_CHAIN"),
                  bev_pos_cache=_env_on("CMT_BEV_POS_CACHE"), conv_halo=_env_on("CMT_CONV_HALO"),
                  mlp_fused=_env_on("CMT_MLP_FUSED"), chain_combine=_env_on("CMT_CHAIN_COMBINE"),
                  rv_geo=_env_on("CMT_RV_GEO"), train_graph=os.environ.get("CMT_TRAIN_GRAPH", "0") == "1")


@contextlib.contextmanager
def options(**kw):
    """Temporarily override fields of OPTIONS: ``with options(side_stream=False): ...``."""
    old = {k: getattr(OPTIONS, k) for k in kw}
    for k, v in kw.items():
        if not hasattr(OPTIONS, k):
            raise AttributeError(f"unknown option {k}")
        setattr(OPTIONS, k, bool(v))
    try:
        yield OPTIONS
    finally:
        for k, v in old.items():
            setattr(OPTIONS, k, v)
