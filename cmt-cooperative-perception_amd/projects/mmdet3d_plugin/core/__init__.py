from .bbox import MultiTaskBBoxCoder  # noqa: F401
