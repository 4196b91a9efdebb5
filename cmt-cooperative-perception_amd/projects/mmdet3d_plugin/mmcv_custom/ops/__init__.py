from .voxel import SPConvVoxelization, voxelize_batch  # noqa: F401
