"""MI355X-native drop-in for the reference's ``projects.mmdet3d_plugin`` hot
path (CMT / CMTCoop decoder heads, transformer, attention, voxelization).

Importing the package registers the reference's type names
(CmtHead, CmtLidarHead, CmtImageHead, CmtHeadCoop, CmtLidarHeadCoop,
CmtImageHeadCoop, CmtTransformer, CmtLidarTransformer, CmtImageTransformer,
PETRTransformerDecoder, PETRTransformerDecoderLayer,
PETRMultiheadFlashAttention, MultiheadAttention, FFN, SeparateTaskHead,
MultiTaskBBoxCoder, SPConvVoxelization) so the reference's
``pts_bbox_head`` config dicts build unchanged with ``build_head``.
"""
from . import core, mmcv_custom, models  # noqa: F401
from .registry import (ATTENTION, BBOX_CODERS, HEADS, TRANSFORMER, TRANSFORMER_LAYER,  # noqa: F401
                       TRANSFORMER_LAYER_SEQUENCE, build_from_cfg, build_head)
from .runtime import get_precision, set_precision  # noqa: F401
