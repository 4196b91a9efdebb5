from .coders import MultiTaskBBoxCoder  # noqa: F401
