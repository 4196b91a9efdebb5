from .attention import FlashAttention, FlashMHA  # noqa: F401
from .cmt_transformer import CmtImageTransformer, CmtLidarTransformer, CmtTransformer  # noqa: F401
from .petr_transformer import (FFN, MultiheadAttention, PETRMultiheadAttention,  # noqa: F401
                               PETRMultiheadFlashAttention, PETRTransformerDecoder, PETRTransformerDecoderLayer)
