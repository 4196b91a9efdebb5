from .multi_task_bbox_coder import MultiTaskBBoxCoder, denormalize_bbox  # noqa: F401
