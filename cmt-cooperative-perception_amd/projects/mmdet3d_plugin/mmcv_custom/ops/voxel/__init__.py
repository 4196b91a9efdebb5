from .spconv_voxelize import SPConvVoxelization, voxelize_batch  # noqa: F401
