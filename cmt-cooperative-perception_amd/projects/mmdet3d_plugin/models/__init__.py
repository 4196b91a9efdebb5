from .dense_heads import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
