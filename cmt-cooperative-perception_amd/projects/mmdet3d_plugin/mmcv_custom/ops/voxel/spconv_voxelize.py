"""SPConvVoxelization with the reference's API on the gfx950 scatter kernels.

Reference: projects/mmdet3d_plugin/mmcv_custom/ops/voxel/spconv_voxelize.py:11-71
(spconv 2.1.21 PointToVoxel) and its caller models/detectors/cmt.py:88-113.
Semantics (deterministic): voxels in first-appearance order of their points,
the first ``max_num_points`` points of each voxel in input order, at most
``max_voxels[0]`` (train) / ``max_voxels[1]`` (eval) voxels, coordinates z, y, x,
zero-padded point slots -- spconv's CPU point2voxel order (its CUDA hash
order is nondeterministic).  ``forward_mean`` additionally returns the
HardSimpleVFE mean computed in the same kernel.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .... import native
from ....registry import VOXEL_LAYERS

__all__ = ["SPConvVoxelization", "voxelize_batch"]


@VOXEL_LAYERS.register_module()
class SPConvVoxelization(nn.Module):
    def __init__(self, voxel_size, point_cloud_range, max_num_points, max_voxels, num_point_features,
                 device=None):
        super().__init__()
        assert len(voxel_size) == 3
        assert len(point_cloud_range) == 6
        self.voxel_size = np.array(voxel_size)
        self.point_cloud_range = np.array(point_cloud_range)
        self.max_num_points = max_num_points
        self.num_point_features = num_point_features
        self.max_voxels = tuple(max_voxels) if isinstance(max_voxels, (tuple, list)) else (max_voxels, max_voxels)
        grid_size = (self.point_cloud_range[3:6] - self.point_cloud_range[0:3]) / np.array(voxel_size)
        self.grid_size = np.round(grid_size).astype(np.int64)

    def _run(self, points, nfeat_mean):
        mv = self.max_voxels[0] if self.training else self.max_voxels[1]
        vox, coors, num, means, nvox = native.voxelize(
            points.float(), voxel_size=self.voxel_size.tolist(), coors_range=self.point_cloud_range.tolist(),
            grid=self.grid_size.tolist(), max_points=self.max_num_points, max_voxels=mv, nfeat_mean=nfeat_mean)
        m = int(nvox.item())
        return vox[:m], coors[:m], num[:m], means[:m]

    def forward(self, points):
        """points [N, F] -> (voxels [M, max_points, F], coors [M, 3] zyx int32, num_points [M] int32)."""
        vox, coors, num, _ = self._run(points, min(points.shape[1], 8))
        return vox, coors, num

    def forward_mean(self, points, num_features=5):
        """(+ HardSimpleVFE) -> (voxels, coors, num_points, mean [M, num_features])."""
        return self._run(points, num_features)

    def __repr__(self):
        return (f"{self.__class__.__name__}(voxel_size={self.voxel_size}, point_cloud_range={self.point_cloud_range}"
                f", max_num_points={self.max_num_points}, max_voxels={self.max_voxels}, "
                f"num_point_features={self.num_point_features})")


def voxelize_batch(layer, points_list, num_features=5):
    """CmtDetector.voxelize (cmt.py:88-113) + HardSimpleVFE: per-sample voxelize,
    concatenate, prepend the sample index to the coordinates."""
    feats, nums, coors = [], [], []
    for i, pts in enumerate(points_list):
        _, c, n, mean = layer.forward_mean(pts, num_features)
        feats.append(mean)
        nums.append(n)
        coors.append(F.pad(c, (1, 0), mode="constant", value=i))
    return torch.cat(feats, 0), torch.cat(nums, 0), torch.cat(coors, 0)
