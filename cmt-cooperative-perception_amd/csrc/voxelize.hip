// Point -> voxel scatter-mean (SPConvVoxelization + HardSimpleVFE) for gfx950.
//
// Three launches, no host synchronisation, graph-capturable; deterministic
// (spconv's CPU point2voxel order):
//   1 bin     (1024 points per workgroup): coalesced point loads, fp32 voxel
//             coordinate, out-of-grid points dropped.  LDS binning: the
//             workgroup's keys go into an LDS hash table first (LDS atomics),
//             so each distinct voxel of the workgroup probes the global table
//             once (atomicCAS on the key) and posts its smallest point index
//             once (atomicMin); then every point pushes itself on its voxel's
//             point list (one atomicExch per point).
//   2 assign  (2048 points per workgroup, single-pass decoupled look-back
//             scan in ticket order): point i leads its voxel iff it is the
//             voxel's smallest index; the exclusive count of leaders before
//             it is the voxel id (first-appearance order), ids >= max_voxels
//             are dropped exactly like the CPU budget check; writes coors and
//             the voxel -> table-slot map, and the voxel count M.
//   3 gather  (one thread per voxel < M): walks its point list, keeps the
//             max_points smallest indices in increasing order, copies those
//             rows into the zero-padded [max_points, F] block and writes the
//             fp32 mean of the kept rows (slot order / count -- HardSimpleVFE).
//
// Workspace contract: every word starts and ends all-ones ("clean"): the
// table slots a call dirties are reset by the call itself (dropped voxels in
// launch 2, kept voxels in launch 3, the look-back words and the ticket in
// launch 3).  cmt_voxelize_workspace_init fills a new workspace once; after
// that any number of calls with N <= its capacity reuse it on one stream.
#include "cmt_common.h"

namespace {

constexpr int BIN_PTS = 256;         // points per bin workgroup (one per thread)
constexpr int BIN_LDS = 512;         // LDS hash entries
constexpr int ASG_T = 256;           // assign threads
constexpr int ASG_PER = 8;           // points per assign thread
constexpr int ASG_PTS = ASG_T * ASG_PER;
constexpr uint32_t EMPTY = 0xffffffffu;
constexpr unsigned long long ST_EMPTY = ~0ull;
constexpr unsigned long long ST_AGG = 1ull << 62, ST_PREFIX = 2ull << 62, ST_VAL = (1ull << 62) - 1;
constexpr int kSpinLimit = 1 << 22;  // look-back guard: a stuck predecessor ends the call with M = -1

struct VoxGeo {
    float vsize[3];
    float rmin[3];
    int grid[3];
};

__device__ __forceinline__ uint32_t hash_key(uint32_t key, uint32_t mask) { return (key * 2654435761u) & mask; }

// workspace views (layout from the capacity P, see ws_layout)
struct VoxWs {
    int P;                     // point capacity
    uint32_t cap;              // global table slots (2 P)
    uint32_t* tkey;            // [cap] voxel key or EMPTY
    uint32_t* tfirst;          // [cap] smallest point index (EMPTY = none)
    int* thead;                // [cap] point-list head (-1 = empty)
    int* pslot;                // [P]   point -> table slot (-1 = dropped)
    int* pnext;                // [P]   point-list link
    int* vslot;                // [P]   voxel id -> table slot
    unsigned long long* st;    // [P / ASG_PTS + 1] look-back words
    uint32_t* misc;            // [0] ticket, [1] error
};

__global__ __launch_bounds__(BIN_PTS) void vox_bin_kernel(const float* __restrict__ pts, int N, int F, VoxGeo g,
                                                          VoxWs w) {
    __shared__ uint32_t lkey[BIN_LDS];
    __shared__ uint32_t lmin[BIN_LDS];
    __shared__ int lslot[BIN_LDS];
    __shared__ int lnew[BIN_PTS];     // compact list of this workgroup's distinct voxels (LDS entries)
    __shared__ int nnew;
    const int tid = threadIdx.x;
    for (int e = tid; e < BIN_LDS; e += BIN_PTS) {
        lkey[e] = EMPTY;
        lmin[e] = EMPTY;
    }
    if (tid == 0) nnew = 0;
    __syncthreads();
    const int i = blockIdx.x * BIN_PTS + tid;   // one point per thread: consecutive lanes, consecutive rows
    uint32_t key = EMPTY;
    int le = -1;
    if (i < N) {
        const float* p = pts + (int64_t)i * F;
        int c[3];
        bool in = true;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            c[j] = (int)floorf((p[j] - g.rmin[j]) / g.vsize[j]);
            in = in && c[j] >= 0 && c[j] < g.grid[j];
        }
        if (in) {
            key = (uint32_t)((c[2] * g.grid[1] + c[1]) * g.grid[0] + c[0]);
            uint32_t s = hash_key(key, BIN_LDS - 1);
            while (true) {
                const uint32_t old = atomicCAS(&lkey[s], EMPTY, key);
                if (old == EMPTY) lnew[atomicAdd(&nnew, 1)] = (int)s;   // first of its voxel here
                if (old == EMPTY || old == key) break;
                s = (s + 1) & (BIN_LDS - 1);
            }
            atomicMin(&lmin[s], (uint32_t)i);
            le = (int)s;
        }
    }
    __syncthreads();
    // one global probe + one atomicMin per distinct voxel of the workgroup (one per thread at most)
    if (tid < nnew) {
        const int e = lnew[tid];
        const uint32_t kk = lkey[e];
        const uint32_t gmask = w.cap - 1;
        uint32_t s = hash_key(kk, gmask);
        while (true) {
            const uint32_t old = atomicCAS(&w.tkey[s], EMPTY, kk);
            if (old == EMPTY || old == kk) break;
            s = (s + 1) & gmask;
        }
        atomicMin(&w.tfirst[s], lmin[e]);
        lslot[e] = (int)s;
    }
    __syncthreads();
    if (i < N) {
        const int s = le >= 0 ? lslot[le] : -1;
        w.pslot[i] = s;
        if (s >= 0) w.pnext[i] = atomicExch(&w.thead[s], i);
    }
}

__device__ __forceinline__ int block_excl_scan256(int v, int* sh, int* total) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    int base = 0;
    for (int j = 0; j < wv; ++j) base += sh[j];
    *total = sh[0] + sh[1] + sh[2] + sh[3];
    return base + x - v;
}

__global__ __launch_bounds__(ASG_T) void vox_assign_kernel(int N, VoxGeo g, int max_voxels, VoxWs w, int* coors,
                                                           int* num_voxels) {
    __shared__ int sh[4];
    __shared__ int s_bid;
    __shared__ int s_prefix;
    const int tid = threadIdx.x;
    // blocks take the chunks in ticket order: a block waits only on blocks that started before it
    if (tid == 0) s_bid = (int)(atomicAdd(&w.misc[0], 1u) + 1u);   // the clean ticket word is all-ones
    __syncthreads();
    const int bid = s_bid;
    const int nb = (N + ASG_PTS - 1) / ASG_PTS;
    if (bid >= nb) return;   // a stale ticket word (never with a clean workspace): no out-of-range chunk
    const int i0 = bid * ASG_PTS + tid * ASG_PER;
    int lead[ASG_PER];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < ASG_PER; ++k) {
        const int i = i0 + k;
        const int s = i < N ? w.pslot[i] : -1;
        lead[k] = (s >= 0 && (uint32_t)s < w.cap && w.tfirst[s] == (uint32_t)i) ? s : -1;
        cnt += lead[k] >= 0;
    }
    int total;
    const int excl = block_excl_scan256(cnt, sh, &total);
    if (tid == 0) {
        int prefix = 0;
        if (bid == 0) {
            __hip_atomic_store(&w.st[0], ST_PREFIX | (unsigned long long)total, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&w.st[bid], ST_AGG | (unsigned long long)total, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        s_prefix = 0;
    }
    // look-back by the first wave: 64 predecessors per round trip (lane l reads block bid-1-l);
    // the window sums aggregates up to the nearest inclusive prefix, retried while any is missing
    if (bid > 0 && tid < 64) {
        long long acc = 0;
        int j0 = bid - 1, spins = 0;
        while (j0 >= 0) {
            const int j = j0 - tid;
            const unsigned long long v =
                j >= 0 ? __hip_atomic_load(&w.st[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) : ST_PREFIX;
            const bool is_pre = (v & ~ST_VAL) == ST_PREFIX;
            const unsigned long long pre_mask = __ballot(is_pre);
            const int stop = pre_mask ? __ffsll((long long)pre_mask) - 1 : 64;   // first lane holding a prefix
            const bool missing = tid <= stop && tid < 64 && v == ST_EMPTY;
            if (__any(missing)) {
                if (++spins > kSpinLimit) {
                    if (tid == 0) atomicExch(&w.misc[1], 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            long long part = (tid <= stop && j >= 0) ? (long long)(v & ST_VAL) : 0;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
            acc += part;
            if (stop < 64) break;
            j0 -= 64;
        }
        if (tid == 0) {
            __hip_atomic_store(&w.st[bid], ST_PREFIX | (unsigned long long)(acc + total), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
            s_prefix = (int)acc;
        }
    }
    __syncthreads();
    if (tid == 0) {
        const int prefix = s_prefix;
        if (bid == nb - 1) *num_voxels = min(prefix + total, max_voxels);
    }
    __syncthreads();
    int v = s_prefix + excl;
#pragma unroll
    for (int k = 0; k < ASG_PER; ++k) {
        const int s = lead[k];
        if (s < 0) continue;
        if (v < max_voxels) {
            const uint32_t key = w.tkey[s];
            const int cx = (int)(key % (uint32_t)g.grid[0]);
            const int cy = (int)((key / (uint32_t)g.grid[0]) % (uint32_t)g.grid[1]);
            const int cz = (int)(key / ((uint32_t)g.grid[0] * (uint32_t)g.grid[1]));
            coors[v * 3 + 0] = cz;
            coors[v * 3 + 1] = cy;
            coors[v * 3 + 2] = cx;
            w.vslot[v] = s;
        } else {
            // over the voxel budget: nobody gathers this voxel, clean its slot now
            w.tkey[s] = EMPTY;
            w.tfirst[s] = EMPTY;
            w.thead[s] = -1;
        }
        ++v;
    }
}

// One thread per kept voxel.  The list is re-walked for every kept slot (the
// next-smallest index each time): voxels hold few points at these densities,
// and no per-lane register array (divergent dynamic indexing) is needed.  The
// walk is bounded by N and every index is range-checked, so a corrupted
// workspace cannot send a load outside the buffers.
__global__ __launch_bounds__(256) void vox_gather_kernel(const float* __restrict__ pts, int N, int F, int nst,
                                                         VoxWs w, int max_points, int nfeat_mean, float* voxels,
                                                         int* num_points, float* means, int* num_voxels) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < nst) w.st[v] = ST_EMPTY;             // launch 2's look-back words, for the next call
    const int M = *num_voxels;
    if (v == 0) {
        w.misc[0] = EMPTY;                       // ticket
        if (w.misc[1] != EMPTY) {                // a look-back gave up: report M = -1
            w.misc[1] = EMPTY;
            *num_voxels = -1;
        }
    }
    if (v >= M) return;
    const int s = w.vslot[v];
    if (s < 0 || (uint32_t)s >= w.cap) return;
    const int head = w.thead[s];
    float* vox = voxels + (int64_t)v * max_points * F;
    float sum[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) sum[f] = 0.f;
    // one walk for the count and the two smallest indices (most voxels hold one or two points);
    // the third and later kept points re-walk for the next-smallest index
    int n = 0, m1 = 0x7fffffff, m2 = 0x7fffffff;
    {
        int steps = 0;
        for (int j = head; j >= 0 && j < N && steps < N; j = w.pnext[j], ++steps) {
            ++n;
            if (j < m1) {
                m2 = m1;
                m1 = j;
            } else if (j < m2) {
                m2 = j;
            }
        }
    }
    const int kept = min(n, max_points);
    int prev = -1;
    for (int r = 0; r < kept; ++r) {
        int best = r == 0 ? m1 : m2;
        if (r >= 2) {
            best = 0x7fffffff;
            int steps = 0;
            for (int j = head; j >= 0 && j < N && steps < N; j = w.pnext[j], ++steps)
                if (j > prev && j < best) best = j;
        }
        if (best >= N) break;                    // cannot happen on a consistent list
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
    for (int f = 0; f < nfeat_mean && f < 8; ++f)
        means[(int64_t)v * nfeat_mean + f] = kept ? sum[f] / (float)kept : 0.f;
    // leave the slot clean for the next call
    w.tkey[s] = EMPTY;
    w.tfirst[s] = EMPTY;
    w.thead[s] = -1;
}

int capacity_for(int N) {
    int P = 1024;
    while (P < N) P <<= 1;
    return P;
}

// layout of a workspace with point capacity P (a power of two >= 1024)
int64_t ws_layout(int P, char* base, VoxWs* w) {
    const int64_t cap = 2 * (int64_t)P;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
        char* p = base ? base + off : nullptr;
        off += ((bytes + 255) / 256) * 256;
        return p;
    };
    VoxWs v;
    v.P = P;
    v.cap = (uint32_t)cap;
    v.tkey = (uint32_t*)take(cap * 4);
    v.tfirst = (uint32_t*)take(cap * 4);
    v.thead = (int*)take(cap * 4);
    v.pslot = (int*)take((int64_t)P * 4);
    v.pnext = (int*)take((int64_t)P * 4);
    v.vslot = (int*)take((int64_t)P * 4);
    v.st = (unsigned long long*)take(((int64_t)P / ASG_PTS + 1) * 8);
    v.misc = (uint32_t*)take(64);
    if (w) *w = v;
    return off;
}

// the capacity of a workspace of `bytes` (the largest P whose layout fits)
int capacity_of(int64_t bytes) {
    int P = 0;
    for (int q = 1024; q <= (1 << 24) && ws_layout(q, nullptr, nullptr) <= bytes; q <<= 1) P = q;
    return P;
}

}  // namespace

extern "C" int64_t cmt_voxelize_workspace_bytes(int N, int max_voxels) {
    (void)max_voxels;
    return ws_layout(capacity_for(N > 0 ? N : 1), nullptr, nullptr);
}

extern "C" int cmt_voxelize_workspace_init(void* workspace, int64_t workspace_bytes, void* stream) {
    CMT_REQUIRE(workspace != nullptr && capacity_of(workspace_bytes) > 0, "cmt_voxelize_workspace_init: bad workspace");
    const hipError_t e = hipMemsetAsync(workspace, 0xff, (size_t)workspace_bytes, (hipStream_t)stream);
    if (e != hipSuccess) return cmt_fail((int)e, "cmt_voxelize_workspace_init: hipMemsetAsync failed");
    return 0;
}

extern "C" int cmt_voxelize(const float* points, int N, int F, const float* voxel_size3, const float* coors_range6,
                            const int* grid3, int max_points, int max_voxels, int nfeat_mean, float* voxels,
                            int* coors, int* num_points, float* means, int* num_voxels, void* workspace,
                            int64_t workspace_bytes, void* stream) {
    CMT_REQUIRE(voxel_size3 && coors_range6 && grid3, "cmt_voxelize: null geometry");
    CMT_REQUIRE(N >= 0 && F >= 3 && max_points > 0 && max_voxels > 0 && nfeat_mean <= F && nfeat_mean <= 8,
                "cmt_voxelize: bad sizes");
    CMT_REQUIRE((int64_t)grid3[0] * grid3[1] * grid3[2] < 0xffffffffLL, "cmt_voxelize: grid too large");
    CMT_REQUIRE(voxels && coors && num_points && means && num_voxels, "cmt_voxelize: null output");
    const int P = workspace ? capacity_of(workspace_bytes) : 0;
    if (workspace == nullptr || P < N || P == 0)
        return cmt_fail(CMT_EWORKSPACE, "cmt_voxelize: workspace too small (cmt_voxelize_workspace_bytes)");
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        (void)hipMemsetAsync(num_voxels, 0, sizeof(int), s);
        return cmt_check_launch("cmt_voxelize");
    }
    CMT_REQUIRE(points != nullptr, "cmt_voxelize: null points");
    VoxWs w;
    ws_layout(P, (char*)workspace, &w);
    VoxGeo g;
    for (int j = 0; j < 3; ++j) {
        g.vsize[j] = voxel_size3[j];
        g.rmin[j] = coors_range6[j];
        g.grid[j] = grid3[j];
    }
    const int nb_asg = cdiv(N, ASG_PTS);
    vox_bin_kernel<<<(unsigned)cdiv(N, BIN_PTS), 256, 0, s>>>(points, N, F, g, w);
    vox_assign_kernel<<<(unsigned)nb_asg, ASG_T, 0, s>>>(N, g, max_voxels, w, coors, num_voxels);
    // one thread per possible voxel (<= min(N, max_voxels)); also covers the look-back words
    const int ng = max(min(N, max_voxels), nb_asg);
    vox_gather_kernel<<<(unsigned)cdiv(ng, 256), 256, 0, s>>>(points, N, F, nb_asg, w, max_points, nfeat_mean,
                                                               voxels, num_points, means, num_voxels);
    return cmt_check_launch("cmt_voxelize");
}
