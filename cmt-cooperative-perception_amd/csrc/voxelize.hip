// Point -> voxel scatter-mean (SPConvVoxelization + HardSimpleVFE) for gfx950.
//
// Deterministic, sync-free pipeline (every launch is sized by N; voxel-count
// dependent kernels read M from device memory and exit early):
//   1 bin:      per point, fp32 voxel coordinate, drop out-of-grid, insert the
//               voxel key into an open-addressing hash table (atomicCAS) and
//               record the smallest point index that hit it (atomicMin)
//   2 leaders:  point i is its voxel's leader iff it is that smallest index
//   3 scan:     exclusive scan of leader flags -> voxel id in first-appearance
//               order (== spconv's CPU point2voxel order); ids >= max_voxels
//               are dropped exactly like the CPU budget check
//   4 count:    points per voxel, exclusive scan -> segment offsets
//   5 scatter:  point indices into per-voxel segments (order not yet fixed)
//   6 gather:   per voxel, select its first max_points point indices in input
//               order, copy the rows into the zero-padded [max_points, F]
//               block and write the fp32 mean of the kept rows (sum in slot
//               order / count -- HardSimpleVFE).
#include "cmt_common.h"

namespace {

constexpr int SCAN_BS = 1024;

struct VoxGeo {
    float vsize[3];
    float rmin[3];
    int grid[3];
};

__device__ __forceinline__ uint32_t hash_key(int key, uint32_t mask) {
    return ((uint32_t)key * 2654435761u) & mask;
}

__global__ void vox_bin_kernel(const float* __restrict__ pts, int N, int F, VoxGeo g, int* tkey, int* tfirst,
                               uint32_t mask, int* pslot, int* pkey) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float* p = pts + (int64_t)i * F;
    int c[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float v = (p[j] - g.rmin[j]) / g.vsize[j];
        c[j] = (int)floorf(v);
        if (c[j] < 0 || c[j] >= g.grid[j]) {
            pslot[i] = -1;
            return;
        }
    }
    const int key = (c[2] * g.grid[1] + c[1]) * g.grid[0] + c[0];
    pkey[i] = key;
    uint32_t s = hash_key(key, mask);
    while (true) {
        const int old = atomicCAS(&tkey[s], -1, key);
        if (old == -1 || old == key) break;
        s = (s + 1) & mask;
    }
    atomicMin(&tfirst[s], i);
    pslot[i] = (int)s;
}

__global__ void vox_leader_kernel(const int* __restrict__ pslot, const int* __restrict__ tfirst, int N, int* flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int s = pslot[i];
    flag[i] = (s >= 0 && tfirst[s] == i) ? 1 : 0;
}

// ---- two-level exclusive scan (n <= SCAN_BS * SCAN_BS) ----------------------
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int* total) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    if (wv == 0) {
        int t = lane < (int)(blockDim.x >> 6) ? sh[lane] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            int y = __shfl_up(t, off);
            if (lane >= off) t += y;
        }
        if (lane < (int)(blockDim.x >> 6)) sh[lane] = t;
    }
    __syncthreads();
    const int wave_base = wv ? sh[wv - 1] : 0;
    *total = sh[(blockDim.x >> 6) - 1];
    __syncthreads();
    return wave_base + x - v;
}

// n taken from *n_dev when non-null (voxel-count dependent scans)
__global__ __launch_bounds__(SCAN_BS) void scan_blocks_kernel(const int* in, int* out, int* bsum, int n_static,
                                                               const int* n_dev) {
    __shared__ int sh[SCAN_BS / 64];
    const int n = n_dev ? *n_dev : n_static;
    const int i = blockIdx.x * SCAN_BS + threadIdx.x;
    const int v = i < n ? in[i] : 0;
    int total;
    const int e = block_excl_scan(v, sh, &total);
    if (i < n) out[i] = e;
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_BS) void scan_sums_kernel(int* bsum, int nb, int* total_out) {
    __shared__ int sh[SCAN_BS / 64];
    const int v = (int)threadIdx.x < nb ? bsum[threadIdx.x] : 0;
    int total;
    const int e = block_excl_scan(v, sh, &total);
    if ((int)threadIdx.x < nb) bsum[threadIdx.x] = e;
    if (threadIdx.x == 0 && total_out) *total_out = total;
}

__global__ void scan_add_kernel(int* out, const int* bsum, int n_static, const int* n_dev) {
    const int n = n_dev ? *n_dev : n_static;
    const int i = blockIdx.x * SCAN_BS + threadIdx.x;
    if (i < n) out[i] += bsum[blockIdx.x];
}

__global__ void vox_assign_kernel(const int* __restrict__ flag, const int* __restrict__ scan,
                                  const int* __restrict__ pslot, const int* __restrict__ pkey, int N, VoxGeo g,
                                  int max_voxels, int* tvid, int* coors, const int* n_leaders, int* num_voxels) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *num_voxels = min(*n_leaders, max_voxels);
    if (i >= N || !flag[i]) return;
    const int v = scan[i];
    const int s = pslot[i];
    if (v < max_voxels) {
        tvid[s] = v;
        const int key = pkey[i];
        const int cx = key % g.grid[0];
        const int cy = (key / g.grid[0]) % g.grid[1];
        const int cz = key / (g.grid[0] * g.grid[1]);
        coors[v * 3 + 0] = cz;
        coors[v * 3 + 1] = cy;
        coors[v * 3 + 2] = cx;
    } else {
        tvid[s] = -1;
    }
}

__global__ void vox_count_kernel(const int* __restrict__ pslot, const int* __restrict__ tvid, int N, int* pvid,
                                 int* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int s = pslot[i];
    const int v = s >= 0 ? tvid[s] : -1;
    pvid[i] = v;
    if (v >= 0) atomicAdd(&cnt[v], 1);
}

__global__ void vox_scatter_kernel(const int* __restrict__ pvid, const int* __restrict__ voff, int N, int* cursor,
                                   int* list) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int v = pvid[i];
    if (v < 0) return;
    const int pos = voff[v] + atomicAdd(&cursor[v], 1);
    list[pos] = i;
}

__global__ void vox_gather_kernel(const float* __restrict__ pts, int F, const int* __restrict__ voff,
                                  const int* __restrict__ cnt, const int* __restrict__ list,
                                  const int* __restrict__ num_voxels, int max_points, int nfeat_mean,
                                  float* voxels, int* num_points, float* means) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= *num_voxels) return;
    const int base = voff[v];
    const int n = cnt[v];
    const int kept = min(n, max_points);
    float* vox = voxels + (int64_t)v * max_points * F;
    float sum[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) sum[f] = 0.f;
    int prev = -1;
    for (int r = 0; r < kept; ++r) {
        int best = 0x7fffffff;
        for (int j = 0; j < n; ++j) {
            const int idx = list[base + j];
            if (idx > prev && idx < best) best = idx;
        }
        prev = best;
        const float* p = pts + (int64_t)best * F;
        for (int f = 0; f < F; ++f) {
            const float x = p[f];
            vox[r * F + f] = x;
            if (f < nfeat_mean && f < 8) sum[f] += x;
        }
    }
    for (int r = kept; r < max_points; ++r)
        for (int f = 0; f < F; ++f) vox[r * F + f] = 0.f;
    num_points[v] = kept;
    for (int f = 0; f < nfeat_mean && f < 8; ++f) means[(int64_t)v * nfeat_mean + f] = sum[f] / (float)kept;
}

struct VoxWs {
    uint32_t cap;
    int *tkey, *tfirst, *tvid, *pslot, *pkey, *flag, *scan, *pvid, *cnt, *voff, *cursor, *list, *bsum, *misc;
};

uint32_t table_cap(int N) {
    uint32_t cap = 1024;
    while (cap < (uint32_t)N * 2u) cap <<= 1;
    return cap;
}

int64_t ws_layout(int N, int max_voxels, char* base, VoxWs* w) {
    (void)max_voxels;
    const uint32_t cap = table_cap(N);
    const int64_t n = N > 0 ? N : 1;
    const int64_t nbs = cdiv64(n, SCAN_BS) + 1;
    int64_t off = 0;
    auto take = [&](int64_t count) {
        int* p = base ? (int*)(base + off) : nullptr;
        off += ((count * 4 + 255) / 256) * 256;
        return p;
    };
    int* tkey = take(cap);
    int* tfirst = take(cap);
    int* tvid = take(cap);
    int* pslot = take(n);
    int* pkey = take(n);
    int* flag = take(n);
    int* scan = take(n);
    int* pvid = take(n);
    int* cnt = take(n);
    int* voff = take(n);
    int* cursor = take(n);
    int* list = take(n);
    int* bsum = take(2 * nbs);
    int* misc = take(64);
    if (w) *w = VoxWs{cap, tkey, tfirst, tvid, pslot, pkey, flag, scan, pvid, cnt, voff, cursor, list, bsum, misc};
    return off;
}

}  // namespace

extern "C" int64_t cmt_voxelize_workspace_bytes(int N, int max_voxels) {
    return ws_layout(N, max_voxels, nullptr, nullptr);
}

extern "C" int cmt_voxelize(const float* points, int N, int F, const float* voxel_size3, const float* coors_range6,
                            const int* grid3, int max_points, int max_voxels, int nfeat_mean, float* voxels,
                            int* coors, int* num_points, float* means, int* num_voxels, void* workspace,
                            int64_t workspace_bytes, void* stream) {
    CMT_REQUIRE(voxel_size3 && coors_range6 && grid3, "cmt_voxelize: null geometry");
    CMT_REQUIRE(N >= 0 && F >= 3 && max_points > 0 && max_voxels > 0 && nfeat_mean <= F && nfeat_mean <= 8,
                "cmt_voxelize: bad sizes");
    CMT_REQUIRE(N <= SCAN_BS * SCAN_BS, "cmt_voxelize: at most 1M points per call");
    CMT_REQUIRE((int64_t)grid3[0] * grid3[1] * grid3[2] < 2147483647LL, "cmt_voxelize: grid too large");
    CMT_REQUIRE(voxels && coors && num_points && means && num_voxels, "cmt_voxelize: null output");
    const int64_t need = cmt_voxelize_workspace_bytes(N, max_voxels);
    if (workspace == nullptr || workspace_bytes < need)
        return cmt_fail(CMT_EWORKSPACE, "cmt_voxelize: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        (void)hipMemsetAsync(num_voxels, 0, sizeof(int), s);
        return cmt_check_launch("cmt_voxelize");
    }
    CMT_REQUIRE(points != nullptr, "cmt_voxelize: null points");
    VoxWs w;
    ws_layout(N, max_voxels, (char*)workspace, &w);
    VoxGeo g;
    for (int j = 0; j < 3; ++j) {
        g.vsize[j] = voxel_size3[j];
        g.rmin[j] = coors_range6[j];
        g.grid[j] = grid3[j];
    }
    (void)hipMemsetAsync(w.tkey, 0xff, sizeof(int) * w.cap, s);
    (void)hipMemsetAsync(w.tfirst, 0x7f, sizeof(int) * w.cap, s);
    (void)hipMemsetAsync(w.cnt, 0, sizeof(int) * N, s);
    (void)hipMemsetAsync(w.cursor, 0, sizeof(int) * N, s);
    const unsigned gb = (unsigned)cdiv(N, 256);
    const int nb = cdiv(N, SCAN_BS);
    int* n_leaders = w.misc;
    vox_bin_kernel<<<gb, 256, 0, s>>>(points, N, F, g, w.tkey, w.tfirst, w.cap - 1, w.pslot, w.pkey);
    vox_leader_kernel<<<gb, 256, 0, s>>>(w.pslot, w.tfirst, N, w.flag);
    scan_blocks_kernel<<<nb, SCAN_BS, 0, s>>>(w.flag, w.scan, w.bsum, N, nullptr);
    scan_sums_kernel<<<1, SCAN_BS, 0, s>>>(w.bsum, nb, n_leaders);
    scan_add_kernel<<<nb, SCAN_BS, 0, s>>>(w.scan, w.bsum, N, nullptr);
    vox_assign_kernel<<<gb, 256, 0, s>>>(w.flag, w.scan, w.pslot, w.pkey, N, g, max_voxels, w.tvid, coors,
                                         n_leaders, num_voxels);
    vox_count_kernel<<<gb, 256, 0, s>>>(w.pslot, w.tvid, N, w.pvid, w.cnt);
    // voxel segments: exclusive scan of counts over the M (<= N) voxels
    scan_blocks_kernel<<<nb, SCAN_BS, 0, s>>>(w.cnt, w.voff, w.bsum, N, num_voxels);
    scan_sums_kernel<<<1, SCAN_BS, 0, s>>>(w.bsum, nb, nullptr);
    scan_add_kernel<<<nb, SCAN_BS, 0, s>>>(w.voff, w.bsum, N, num_voxels);
    vox_scatter_kernel<<<gb, 256, 0, s>>>(w.pvid, w.voff, N, w.cursor, w.list);
    vox_gather_kernel<<<gb, 256, 0, s>>>(points, F, w.voff, w.cnt, w.list, num_voxels, max_points, nfeat_mean,
                                         voxels, num_points, means);
    return cmt_check_launch("cmt_voxelize");
}
