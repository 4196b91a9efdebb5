/*
 * CPU restatement of the point -> voxel scatter-mean (TEST INFRASTRUCTURE ONLY).
 *
 * Restates, for the hot path's row a17:
 *   - reference mmcv_custom/ops/voxel/spconv_voxelize.py:11-71
 *     (SPConvVoxelization -> spconv 2.1.21 PointToVoxel, params 25-32,
 *      max_voxels[0] train / [1] eval 36-56, clone copies 58-61),
 *   - reference models/detectors/cmt.py:88-113 (per-sample loop, batch index
 *     prepended with F.pad at 107-111),
 *   - mmdet3d 1.0.0rc6 HardSimpleVFE (mean of the first num_features channels
 *     over the kept points), configured at e.g.
 *     configs/CMT_Nuscenes/lidar/cmt_lidar_voxel0075_cbgs.py:169-172.
 *
 * spconv is a third-party dependency (spconv-cu111 2.1.21, Dockerfile:69) that
 * is not vendored in the reference and not installed here.  Its published CPU
 * algorithm (point2voxel_cpu) is restated: points are visited in input order,
 * c = floor((p - range_min) / vsize) per axis in fp32, points outside
 * [0, grid) on any axis are dropped, a voxel id is assigned at the first point
 * that falls into a new voxel (first-appearance order) until max_voxels ids
 * exist, each voxel keeps its first max_points points in input order, voxels
 * are zero padded, coordinates are written z, y, x.  The CUDA hash voxelizer
 * orders voxels/points by atomics (nondeterministic); this build defines the
 * CPU order as the contract.  Parity unpinned: the reference has no tests or
 * fixtures for this op.
 *
 * The HardSimpleVFE mean is the fp32 sum of the kept points in slot order,
 * divided by (float)num_points.
 *
 * Built by oracle/Makefile into oracle/_build/libvoxel_oracle.so; loaded by
 * tests/ through ctypes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t key;
    int vid;
} slot_t;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

/* Returns the number of voxels M (<= max_voxels), or -1 on allocation error.
 * points: [N, F] row-major fp32 (F = num_point_features >= nfeat_mean)
 * voxel_size[3], coors_range[6] (xmin,ymin,zmin,xmax,ymax,zmax), grid[3] (x,y,z)
 * outputs (caller-allocated for max_voxels):
 *   voxels [max_voxels, max_points, F], coors [max_voxels, 3] (z,y,x),
 *   num_points [max_voxels], means [max_voxels, nfeat_mean] (HardSimpleVFE). */
int cmt_oracle_voxelize(const float* points, int N, int F, const float* voxel_size,
                        const float* coors_range, const int* grid, int max_points,
                        int max_voxels, int nfeat_mean, float* voxels, int* coors,
                        int* num_points, float* means) {
    size_t cap = 16;
    while (cap < (size_t)N * 2 + 16) cap <<= 1;
    slot_t* table = (slot_t*)malloc(cap * sizeof(slot_t));
    if (!table) return -1;
    for (size_t i = 0; i < cap; ++i) table[i].key = -1;
    memset(voxels, 0, sizeof(float) * (size_t)max_voxels * max_points * F);
    memset(num_points, 0, sizeof(int) * (size_t)max_voxels);
    int M = 0;
    for (int i = 0; i < N; ++i) {
        const float* p = points + (size_t)i * F;
        int c[3];
        int ok = 1;
        for (int j = 0; j < 3; ++j) {
            float v = (p[j] - coors_range[j]) / voxel_size[j];
            c[j] = (int)floorf(v);
            if (c[j] < 0 || c[j] >= grid[j]) { ok = 0; break; }
        }
        if (!ok) continue;
        int64_t key = ((int64_t)c[2] * grid[1] + c[1]) * grid[0] + c[0];
        size_t h = (size_t)(mix64((uint64_t)key) & (cap - 1));
        while (table[h].key != -1 && table[h].key != key) h = (h + 1) & (cap - 1);
        int vid;
        if (table[h].key == -1) {
            if (M >= max_voxels) continue;   /* voxel budget exhausted: drop */
            table[h].key = key;
            table[h].vid = M;
            vid = M++;
            coors[vid * 3 + 0] = c[2];
            coors[vid * 3 + 1] = c[1];
            coors[vid * 3 + 2] = c[0];
        } else {
            vid = table[h].vid;
        }
        int n = num_points[vid];
        if (n < max_points) {
            memcpy(voxels + ((size_t)vid * max_points + n) * F, p, sizeof(float) * F);
            num_points[vid] = n + 1;
        }
    }
    for (int v = 0; v < M; ++v) {
        for (int f = 0; f < nfeat_mean; ++f) {
            float s = 0.f;
            for (int k = 0; k < max_points; ++k) s += voxels[((size_t)v * max_points + k) * F + f];
            means[(size_t)v * nfeat_mean + f] = s / (float)num_points[v];
        }
    }
    free(table);
    return M;
}
