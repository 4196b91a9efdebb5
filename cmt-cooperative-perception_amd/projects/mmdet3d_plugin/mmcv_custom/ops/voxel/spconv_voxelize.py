"""SPConvVoxelization with the reference's API on the gfx950 scatter kernels.

Reference: projects/mmdet3d_plugin/mmcv_custom/ops/voxel/spconv_voxelize.py:11-71
(spconv 2.1.21 PointToVoxel) and its caller models/detectors/cmt.py:88-113.
Semantics (deterministic): voxels in first-appearance order of their points,
the first ``max_num_points`` points of each voxel in input order, at most
``max_voxels[0]`` (train) / ``max_voxels[1]`` (eval) voxels, coordinates z, y, x,
zero-padded point slots -- spconv's CPU point2voxel order (its CUDA hash
order is nondeterministic).  ``forward_mean`` additionally returns the
HardSimpleVFE mean computed in the same kernel.

The native voxelizer is three launches with no host synchronisation
(csrc/voxelize.hip).  ``forward_padded`` keeps the voxel count on the device
(outputs sized max_voxels + a device count) and is graph-capturable; the
reference-shaped ``forward`` / ``forward_mean`` trim to the count, which is
a host read.  The layer owns a reusable workspace (kept clean by the kernels).
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
        self._ws, self._ws_cap = None, 0

    def _workspace(self, n, device):
        if self._ws is None or self._ws.device != device or self._ws_cap < n:
            cap = 1024
            while cap < n:
                cap <<= 1
            self._ws, self._ws_cap = native.voxelize_workspace(cap, device), cap
        return self._ws

    def forward_padded(self, points, nfeat_mean=5):
        """points [N, F] -> (voxels [V, max_points, F], coors [V, 3], num_points [V], mean [V, nfeat_mean],
        num_voxels [1] device int32) with V = the active max_voxels; rows >= num_voxels are unspecified.
        No host synchronisation: capturable in a HIP graph."""
        mv = self.max_voxels[0] if self.training else self.max_voxels[1]
        points = points.float()
        return native.voxelize(points, voxel_size=self.voxel_size.tolist(), coors_range=self.point_cloud_range.tolist(),
                               grid=self.grid_size.tolist(), max_points=self.max_num_points, max_voxels=mv,
                               nfeat_mean=nfeat_mean, workspace=self._workspace(points.shape[0], points.device))

    def _run(self, points, nfeat_mean):
        vox, coors, num, means, nvox = self.forward_padded(points, nfeat_mean)
        m = int(nvox.item())   # the reference's outputs are sized by the voxel count (a host read)
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
