from .cmt_head import CmtHead, CmtImageHead, CmtLidarHead, SeparateTaskHead, pos2embed  # noqa: F401
from .cmt_head_coop import CmtHeadCoop, CmtImageHeadCoop, CmtLidarHeadCoop  # noqa: F401
