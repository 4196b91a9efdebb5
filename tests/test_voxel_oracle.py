"""Known answers for the C restatement of the point->voxel scatter-mean
(oracle/voxelize_oracle.c), hand-derived from spconv's CPU point2voxel
semantics (first-appearance voxel order, first max_points points, zyx
coordinates, drop out-of-range) and HardSimpleVFE (mean of kept points)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "oracle", "_build", "libvoxel_oracle.so")


@pytest.fixture(scope="module")
def vox():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(LIB)
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int)

    def run(points, vsize, rng, grid, max_points, max_voxels, nmean=None):
        pts = np.ascontiguousarray(points, np.float32)
        N, F = pts.shape
        nmean = nmean or F
        v = np.zeros((max_voxels, max_points, F), np.float32)
        c = np.zeros((max_voxels, 3), np.int32)
        n = np.zeros((max_voxels,), np.int32)
        m = np.zeros((max_voxels, nmean), np.float32)
        M = lib.cmt_oracle_voxelize(pts.ctypes.data_as(fp), N, F, np.array(vsize, np.float32).ctypes.data_as(fp),
                                    np.array(rng, np.float32).ctypes.data_as(fp),
                                    np.array(grid, np.int32).ctypes.data_as(ip), max_points, max_voxels, nmean,
                                    v.ctypes.data_as(fp), c.ctypes.data_as(ip), n.ctypes.data_as(ip),
                                    m.ctypes.data_as(fp))
        return M, v[:M], c[:M], n[:M], m[:M]
    return run


def test_first_appearance_order_and_zyx(vox):
    pts = [[1.5, 0.5, 0.5, 10, 0], [0.5, 0.5, 0.5, 20, 0], [1.6, 0.6, 0.6, 30, 0], [0.5, 2.5, 1.5, 40, 1]]
    M, v, c, n, m = vox(pts, [1, 1, 1], [0, 0, 0, 4, 4, 4], [4, 4, 4], 10, 100)
    assert M == 3
    assert c.tolist() == [[0, 0, 1], [0, 0, 0], [1, 2, 0]]          # z, y, x in first-appearance order
    assert n.tolist() == [2, 1, 1]
    assert np.allclose(m[0], [1.55, 0.55, 0.55, 20.0, 0.0])
    assert v[0, 2:].sum() == 0                                          # zero padded


def test_max_points_keeps_first_in_input_order(vox):
    pts = [[0.5, 0.5, 0.5, float(i), 0] for i in range(15)]
    M, v, c, n, m = vox(pts, [1, 1, 1], [0, 0, 0, 4, 4, 4], [4, 4, 4], 10, 100)
    assert M == 1 and n[0] == 10
    assert v[0, :, 3].tolist() == [float(i) for i in range(10)]
    assert m[0, 3] == np.float32(45.0) / np.float32(10.0)


def test_out_of_range_dropped_and_voxel_budget(vox):
    pts = [[-0.1, 0.5, 0.5, 1, 0], [4.0, 0.5, 0.5, 1, 0], [0.5, 0.5, 0.5, 1, 0], [1.5, 0.5, 0.5, 1, 0],
           [2.5, 0.5, 0.5, 1, 0], [1.5, 0.5, 0.5, 2, 0]]
    M, v, c, n, m = vox(pts, [1, 1, 1], [0, 0, 0, 4, 4, 4], [4, 4, 4], 10, 2)
    assert M == 2                                                       # third voxel dropped by the budget
    assert c.tolist() == [[0, 0, 0], [0, 0, 1]]
    assert n.tolist() == [1, 2]


def test_empty_input(vox):
    M, *_ = vox(np.zeros((0, 5), np.float32), [1, 1, 1], [0, 0, 0, 4, 4, 4], [4, 4, 4], 10, 10)
    assert M == 0
