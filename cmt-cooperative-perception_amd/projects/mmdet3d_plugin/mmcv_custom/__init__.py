from .ops import SPConvVoxelization, voxelize_batch  # noqa: F401
