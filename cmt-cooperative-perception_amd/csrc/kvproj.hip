// Cross-attention K/V projection of ALL decoder layers in one launch (gfx950).
//
// Replaces, per layer, FlashMHA's packed in_proj on the memory side
// (attention.py:21-27 _in_projection_packed, petr_transformer.py:296-299
// key = key + key_pos): K_l = lowp(mem + pos) Wk_l^T + bk_l, V_l = lowp(mem) Wv_l^T + bv_l,
// written head-split [B][2L*8][Nk][32] for the attention kernel, plus the
// per-(64 keys, head) max squared key norm that bounds its softmax offset
// (cmt_gemm_args.plane_max2).
//
// Shape: M = B*Nk ~ 32k token rows, N = 2*L*256 = 3072, K = 256.  A general
// 128x128-tile GEMM re-reads both operands per tile: ~780 MB of L2->LDS
// traffic for 51 GFLOP, and one CU's load path moves only ~30-60 GB/s
// (MI355X_MICROARCH.md ldsdma-fill), so it ran at ~1/5 of MFMA peak.  Here a
// workgroup keeps ONE 128-row A tile resident (LDS -> VGPRs, read once) and
// sweeps half of the N columns (the K half with A2 = lowp(mem + pos), or the V
// half with A = lowp(mem)); each wave owns whole 32-column head planes, so
// its W fragments are private and come straight from L2 into VGPRs -- no W
// staging, no barriers in the main loop.  W is pre-packed once per weight
// version (fragment-major, 1 KB per plane and k-step), so every W load
// instruction is 1 KB contiguous.  Operand ingest per workgroup: 64 KB of A +
// 768 KB of W (L2-resident, 1.5 MB total).  Each finished plane (128 tokens x
// 64 B, contiguous in the head-split output) is transposed through the wave's
// LDS slice and leaves as 16-B non-temporal stores.
//
// MFMA 32x32x16 in the swapped form D[col][token] = W_frag x A_frag^T: lane
// (lr, lh) holds token lr and columns (r & 3) + 8 (r >> 2) + 4 lh of its
// 32-column plane, so a plane's row of 32 values is two lanes' 16 -- the
// squared-norm reduction is one permlane32 swap.
#include "cmt_common.h"

// kvproj_x3_kernel's schedule bits for dev experiments (dev/build_exp.sh -DCMT_KV_SCHED=n); the
// product build compiles schedule 0 only
#ifndef CMT_KV_SCHED
#define CMT_KV_SCHED 0
#endif

namespace {

constexpr int KP_BM = 128;            // token rows per workgroup
constexpr int KP_K = 256;             // reduction depth (embed dims)
constexpr int KP_KS = KP_K / 16;      // MFMA k-steps
constexpr int KP_MAXB = 2048;         // bias floats per column part held in LDS

typedef const __attribute__((address_space(1))) void* kp_gaddr_t;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* kp_laddr_t;
template <typename T> using frag_of = typename mfma_traits<T>::frag;

// two fp32 values rounded (RNE) into one dword of 16-bit values, x0 low (v_cvt_pk_f16_f32 for f16)
template <typename TC>
__device__ __forceinline__ uint32_t pack2(float x0, float x1) {
    typedef TC v2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{x0, x1}, v2));
}

// acc + the squares of the two 16-bit values packed in w (v_dot2_f32_f16 for f16)
template <typename TC>
__device__ __forceinline__ float sq2(uint32_t w, float acc) {
    if constexpr (std::is_same<TC, f16_t>::value) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 v = __builtin_bit_cast(h2, w);
        return __builtin_amdgcn_fdot2(v, v, acc, false);
    } else {
        const float x0 = (float)__builtin_bit_cast(TC, (uint16_t)(w & 0xffffu));
        const float x1 = (float)__builtin_bit_cast(TC, (uint16_t)(w >> 16));
        return acc + x0 * x0 + x1 * x1;
    }
}

// Batch stride of the head-split C in 16-bit elements: c_bstride when given (one
// layer's K/V planes written into a larger [B][planes][Nk][32] buffer), else the
// launch's own N/32 planes per batch element.
__host__ __device__ inline int64_t kv_c_bstride(const cmt_gemm_args& a) {
    return a.c_bstride ? a.c_bstride : (int64_t)(a.N >> 5) * a.rows_per_batch * 32;
}
// Bytes from C to the end of the last plane the launch writes.
__host__ __device__ inline int64_t kv_c_extent_bytes(const cmt_gemm_args& a) {
    const int64_t nb = a.M / a.rows_per_batch;
    return ((nb - 1) * kv_c_bstride(a) + (int64_t)(a.N >> 5) * a.rows_per_batch * 32) * 2;
}

// Whole 128-token tile per W fetch (8-wave form): the plane's W fragments
// serve all four 32-token tiles, so each workgroup fetches its columns' W
// once instead of once per 64-token half (768 KB instead of 1.5 MB per
// workgroup -- the per-CU L2 stream that bounded the two-half sweep).  A
// fragments come from the LDS tile per k-step (one ds_read_b128 per MFMA);
// the plane leaves through an 8 KB per-wave staging slice.
template <typename T, bool MAXQ>
__device__ __forceinline__ void kv_plane_full(const cmt_gemm_args& a, char* stg, const float* bw, const T* Wl,
                                              typename mfma_traits<T>::frag (&wf)[KP_KS], const char* arow, int j,
                                              int nxt, int plane, int m0, const uint32_t (&soff)[8],
                                              __amdgpu_buffer_rsrc_t crsrc, __amdgpu_buffer_rsrc_t prsrc, int lane) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    const int lr = lane & 31, lh = lane >> 5;
    const T* Wn = Wl + (int64_t)nxt * (KP_KS * 512);
    f32x16 acc[4];
    {
        f32x16 b16;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 b4 = *(const f32x4*)(bw + 32 * j + 8 * g + 4 * lh);
            b16[4 * g] = b4[0]; b16[4 * g + 1] = b4[1]; b16[4 * g + 2] = b4[2]; b16[4 * g + 3] = b4[3];
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = b16;
    }
#pragma unroll
    for (int ks = 0; ks < KP_KS; ++ks) {
        const int sw = ((2 * ks + lh) ^ (lr & 15)) << 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const frag_of<T> at = *(const frag_of<T>*)(arow + t * 32 * (KP_K * 2) + sw);
            acc[t] = mfma_traits<T>::mma(wf[ks], at, acc[t]);
        }
        wf[ks] = *(const frag_of<T>*)(Wn + ks * 512);   // plane `nxt` into the freed slot
    }
    float pm[2] = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int tok = 32 * t + lr;
        float ss = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const t4 v = t4{(T)acc[t][4 * g], (T)acc[t][4 * g + 1], (T)acc[t][4 * g + 2], (T)acc[t][4 * g + 3]};
            const int c0 = 8 * g + 4 * lh;
            *(t4*)(stg + tok * 64 + ((((c0 >> 3) ^ (tok >> 1)) & 3) << 4) + (c0 & 7) * 2) = v;
            if (MAXQ) {
#pragma unroll
                for (int e = 0; e < 4; ++e) ss += (float)v[e] * (float)v[e];
            }
        }
        if (MAXQ) {
            ss = pair_sum(m0 + tok < a.M ? ss : 0.f);
            pm[t >> 1] = (t & 1) ? fmaxf(pm[t >> 1], ss) : ss;
        }
    }
    if (MAXQ) {
#pragma unroll
        for (int gq = 0; gq < 2; ++gq) {
            float x = pm[gq];
#pragma unroll
            for (int off = 1; off < 32; off <<= 1) x = fmaxf(x, __shfl_xor(x, off));
            const int pm_planes = a.plane_max_cols >> 5;
            const int mg = m0 + 64 * gq;
            const uint32_t po = (lane == 0 && mg < a.M) ? (uint32_t)((((int64_t)(mg >> 6)) * pm_planes + plane) * 4)
                                                         : 0xffffffffu;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), prsrc, po, 0, 0);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t pl = (uint32_t)((int64_t)plane * a.rows_per_batch * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int tok = 16 * i + (lane >> 2), ch = lane & 3;
        const f32x4 v = *(const f32x4*)(stg + tok * 64 + (((ch ^ (tok >> 1)) & 3) << 4));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), crsrc,
                                              soff[i] == 0xffffffffu ? soff[i] : soff[i] + pl, 0, 2);
    }
}

template <typename T, bool MAXQ>
__device__ __forceinline__ void kv_sweep_full(const cmt_gemm_args& a, const char* lds, char* stg, const float* bw,
                                              const T* Wl, typename mfma_traits<T>::frag (&wa)[KP_KS], int nplanes,
                                              int plane0, int m0, int lane) {
    const int lr = lane & 31;
    const uint32_t cbytes = (uint32_t)kv_c_extent_bytes(a);
    const auto crsrc = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, cbytes, 0x00020000);
    const uint32_t pmbytes = MAXQ ? (uint32_t)(((a.M + 63) / 64) * (a.plane_max_cols >> 5) * 4) : 0u;
    const auto prsrc = __builtin_amdgcn_make_buffer_rsrc(MAXQ ? (void*)a.plane_max2 : a.C, 0, pmbytes, 0x00020000);
    const int rpb = a.rows_per_batch;
    const int64_t cbs = kv_c_bstride(a);
    uint32_t soff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = m0 + 16 * i + (lane >> 2);
        const int bb = m / rpb;
        const int64_t el = (int64_t)bb * cbs + (int64_t)(m - bb * rpb) * 32;
        soff[i] = m < a.M ? (uint32_t)((el + 8 * (lane & 3)) * 2) : 0xffffffffu;
    }
    const char* arow = lds + lr * (KP_K * 2);
    for (int j = 0; j < nplanes; ++j) {
        const int n1 = j + 1 < nplanes ? j + 1 : j;   // the last plane re-fetches itself (cached, unused)
        kv_plane_full<T, MAXQ>(a, stg, bw, Wl, wa, arow, j, n1, plane0 + j, m0, soff, crsrc, prsrc, lane);
    }
}

// 8 waves, two per SIMD (one's epilogue -- rounding, LDS staging, key-norm max,
// stores -- runs beside the other's MFMAs); A fragments are read from the LDS
// tile per k-step so a wave fits in 256 registers.
template <typename T>
__global__ __launch_bounds__(512, 1) void kvproj_kernel(cmt_gemm_args a, int parts) {
    typedef typename mfma_traits<T>::frag frag;
    constexpr int NW = 8, NTH = 64 * NW;
    constexpr int STG = 8192;   // per-wave store staging bytes
    // 64 KB A tile | NW x STG per-wave store staging | the part's bias (<= 8 KB)
    __shared__ __attribute__((aligned(16))) char lds[KP_BM * KP_K * 2 + NW * STG + KP_MAXB * 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // workgroup -> (row tile, column part); the parts of one row tile are
    // consecutive blocks (their A tiles differ only in A vs A2)
    const int rt = blockIdx.x / parts, part = blockIdx.x - rt * parts;
    const int m0 = rt * KP_BM;
    const int ncols = a.N / parts;                      // columns per part (multiple of 128)
    const int n_part = part * ncols;
    const bool sel_a2 = a.A2 != nullptr && n_part < a.a2_cols;
    const T* Ab = (const T*)(sel_a2 ? a.A2 : a.A);
    const int64_t lda = sel_a2 ? a.lda2 : a.lda;

    // ---- A tile -> LDS (16-B chunks XOR-swizzled by row & 15)
#pragma unroll
    for (int i = 0; i < KP_BM * KP_K * 2 / 16 / NTH; ++i) {
        const int piece = tid + NTH * i;
        const int r = piece >> 5;
        const int lc = (piece & 31) ^ (r & 15);
        const int src = min(m0 + r, a.M - 1);
        __builtin_amdgcn_global_load_lds((kp_gaddr_t)(Ab + (int64_t)src * lda + 8 * lc),
                                         (kp_laddr_t)(lds + piece * 16), 16, 0, 0);
    }
    // the part's bias -> LDS: the epilogue reads it with no vmcnt wait (a global
    // bias load there would drain the W prefetch and the stores before it, which
    // count on the same in-order counter)
    float* bsm = (float*)(lds + KP_BM * KP_K * 2 + NW * STG);
    for (int piece = tid; piece < (ncols >> 2); piece += NTH) {
        if (a.bias)
            __builtin_amdgcn_global_load_lds((kp_gaddr_t)(a.bias + n_part + 4 * piece), (kp_laddr_t)(bsm + 4 * piece),
                                             16, 0, 0);
        else
            *(f32x4*)(bsm + 4 * piece) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int planes_w = ncols / 32 / NW;               // head planes per wave
    const int plane0 = (n_part >> 5) + wave * planes_w;
    const T* W = (const T*)a.W;
    // W in the fragment-packed layout (cmt_hip.h cmt_kv_proj): plane p, k-step ks
    // is 1 KB contiguous, lane-major -- every W load instruction touches 8 lines
    const T* Wl = W + (int64_t)plane0 * (KP_KS * 512) + lane * 8;
    frag wa[KP_KS];   // the current plane; each slot refills with the next plane once used
#pragma unroll
    for (int ks = 0; ks < KP_KS; ++ks) wa[ks] = *(const frag*)(Wl + ks * 512);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_mem();

    char* stg = lds + KP_BM * KP_K * 2 + wave * STG;    // [128 tokens][32] 16-bit
    const float* bw = bsm + 32 * (plane0 - (n_part >> 5));

    // output stores: rows >= M (and non-writer lanes of the key-norm max) get an
    // out-of-range offset and the buffer range check drops them -- no branches
    const bool maxq = a.plane_max2 != nullptr && n_part < a.plane_max_cols;
    if (maxq) kv_sweep_full<T, true>(a, lds, stg, bw, Wl, wa, planes_w, plane0, m0, lane);
    else kv_sweep_full<T, false>(a, lds, stg, bw, Wl, wa, planes_w, plane0, m0, lane);
}

// ---------------------------------------------------------------------------
// Split form (CMT_F16P A / W: the 'ref' policy's fp32-accurate K/V):
// per k-step and 32-token tile three f16 MFMAs W_hi A_hi + W_hi A_lo + W_lo A_hi.
// The 128-token A tile is resident as its hi and lo planes (2 x 64 KB of
// LDS).  W (hi and lo, L2-resident: 3 MB for all layers) streams into a
// KV3_RING-deep register ring of k-steps, KV3_RING steps ahead across plane
// boundaries -- a whole plane's hi + lo fragments (128 registers) beside the
// accumulators and A fragments would not fit two waves per SIMD.  The bias
// comes from scalar loads (no LDS left), and each lane stores its token's
// 4-column pieces straight from the accumulators (8-byte stores; L2 merges
// the two lane halves' pieces of a 64-byte head row) -- no staging buffer.
// W_lo sits N * 256 elements after W_hi, both fragment-packed like
// cmt_kv_proj's W.  The A fragments are read one k-step ahead into a second
// register set (342.6 vs 347.2 us alone, 577.1 vs 576.1 frames/s in frame;
// SQ counters before it: MFMA pipe busy 44 % of SIMD cycles, 61 % of wave
// cycles issue-stalled -- profiles/r3_kvproj_sq_counters.json).
// ---------------------------------------------------------------------------
constexpr int KV3_RING = 4;

// Work units are (128-token tile, column part); the grid's first nfull workgroups take one unit
// each, the rest take HALF a unit (each wave the first or second half of its head planes), so the
// last round of a 3.45-round grid is 2 x 114 short units instead of 114 long ones beside 142 idle CUs.
template <typename TC, int SCHED>
__global__ __launch_bounds__(512, 1) void kvproj_x3_kernel(cmt_gemm_args a, int parts, int nfull) {
    // A tile hi plane | lo plane, each [128 tokens][256] f16 with 16-byte chunks XOR-swizzled by
    // row & 15, then the column part's bias (fp32)
    __shared__ __attribute__((aligned(16))) char lds[2 * KP_BM * KP_K * 2 + KP_MAXB * 4];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lr = lane & 31, lh = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = blockIdx.x;
    const int hx = bid - nfull;                                    // >= 0: a half unit
    const int unit = hx < 0 ? bid : nfull + (hx >> 1);
    const int rt = unit / parts, part = unit - rt * parts;
    const int m0 = rt * KP_BM;
    const int ncols = a.N / parts;
    const int n_part = part * ncols;
    const bool sel_a2 = a.A2 != nullptr && n_part < a.a2_cols;
    const pair_t* Ab = (const pair_t*)(sel_a2 ? a.A2 : a.A);
    const int64_t lda = sel_a2 ? a.lda2 : a.lda;   // 16-bit elements per pair row (hi 256 | lo 256)
#pragma unroll
    for (int i = 0; i < 2 * KP_BM * KP_K * 2 / 16 / 512; ++i) {
        const int piece = tid + 512 * i;
        const int plane_lo = piece >= KP_BM * 32;                 // first half: hi plane, second: lo plane
        const int pc = piece - plane_lo * KP_BM * 32;
        const int r = pc >> 5;
        const int lc = (pc & 31) ^ (r & 15);
        const int src = min(m0 + r, a.M - 1);
        __builtin_amdgcn_global_load_lds((kp_gaddr_t)(Ab + (int64_t)src * lda + plane_lo * KP_K + 8 * lc),
                                         (kp_laddr_t)(lds + piece * 16), 16, 0, 0);
    }
    const int planes_all = ncols / 32 / 8;                         // the wave's head planes of a whole unit
    const int h0 = planes_all >> 1;                                // a half unit: planes [0, h0) or [h0, all)
    const int planes_w = hx < 0 ? planes_all : (hx & 1) ? planes_all - h0 : h0;
    const int plane0 = (n_part >> 5) + wave * planes_all + (hx >= 0 && (hx & 1) ? h0 : 0);
    const pair_t* Wh = (const pair_t*)a.W + (int64_t)plane0 * (KP_KS * 512) + lane * 8;
    const pair_t* Wl = Wh + (int64_t)a.N * KP_K;
    pair8_t rh[KV3_RING], rl[KV3_RING];
#pragma unroll
    for (int ks = 0; ks < KV3_RING; ++ks) {
        rh[ks] = *(const pair8_t*)(Wh + ks * 512);
        rl[ks] = *(const pair8_t*)(Wl + ks * 512);
    }
    float* bsm = (float*)(lds + 2 * KP_BM * KP_K * 2);
    if constexpr (!(SCHED & 64))
        for (int i = tid; i < ncols; i += 512) bsm[i] = a.bias ? a.bias[n_part + i] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_mem();
    // head-split element offset of each tile's token row (plane 0)
    const int rpb = a.rows_per_batch;
    const int64_t cbs = kv_c_bstride(a);
    int64_t rbase[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int m = min(m0 + 32 * t + lr, a.M - 1);
        const int bb = m / rpb;
        rbase[t] = (int64_t)bb * cbs + (int64_t)(m - bb * rpb) * 32;
    }
    const char* lhi = lds;
    const char* llo = lds + KP_BM * KP_K * 2;
    const bool maxq = a.plane_max2 != nullptr && n_part < a.plane_max_cols;
    const int pm_planes = a.plane_max_cols >> 5;
    typedef TC t4 __attribute__((ext_vector_type(4)));
    // A fragments software-pipelined one k-step ahead (two register sets): k-step ks's MFMAs
    // run on the set read during k-step ks - 1 while the reads of ks + 1 are in flight; the
    // tile is the same for every plane, so the last k-step of a plane reads k-step 0 again
    pair8_t fa[2][4][2];
    auto read_a = [&](int ks, pair8_t (&f)[4][2]) {
        const int sw = ((2 * ks + lh) ^ (lr & 15)) << 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            f[t][0] = *(const pair8_t*)(lhi + (t * 32 + lr) * (KP_K * 2) + sw);
            f[t][1] = *(const pair8_t*)(llo + (t * 32 + lr) * (KP_K * 2) + sw);
        }
    };
    read_a(0, fa[0]);
    if constexpr (SCHED & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // SCHED bit 2: the younger half of the workgroup (waves 4-7) at priority 1 for the whole
    // loop (cdna_hip_programming.md T5, static form); bits 4 / 8 / 16 / 32: diagnostics only (no W
    // loads / no A fragment reads / no K-V stores / no bias loads: wrong results, for timing what
    // each costs)
    if constexpr (SCHED & 2)
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#ifdef CMT_KV_SLEEP
    // dev: the SIMD's second wave (waves 4-7) starts CMT_KV_SLEEP x 64 cycles late, so its plane
    // epilogues fall inside the partner's MFMA runs instead of beside the partner's own epilogues
    if (wave >= 4) __builtin_amdgcn_s_sleep(CMT_KV_SLEEP);
#endif
    for (int j = 0; j < planes_w; ++j) {
        const int plane = plane0 + j;
        f32x16 acc[4];
        if constexpr (!(SCHED & 64)) {
            // the bias from LDS (a global load here made the compiler drain the W ring, vmcnt(0),
            // at every plane): lane (lr, lh) holds columns 8 q + 4 lh + 0..3 of the plane
            const float* bp = bsm + plane * 32 - n_part + 4 * lh;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 b = (SCHED & 32) ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(bp + 8 * q);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t][4 * q + e] = b[e];
            }
        } else {
            const float* bp = a.bias + plane * 32;   // wave-uniform: scalar loads
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int c = (r & 3) + 8 * (r >> 2);
                const float b = (SCHED & 32) ? 0.f : a.bias ? (lh ? bp[c + 4] : bp[c]) : 0.f;
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t][r] = b;
            }
        }
        // the ring's next loads: the rest of this plane, then the next plane's first steps
        const int jn = j + 1 < planes_w ? j + 1 : j;   // past the last plane: re-fetch it (cached, unused)
#pragma unroll
        for (int ks = 0; ks < KP_KS; ++ks) {
            const int slot = ks % KV3_RING;
            if constexpr (!(SCHED & 8)) read_a((ks + 1) % KP_KS, fa[(ks + 1) & 1]);
            const pair8_t (&f)[4][2] = fa[(SCHED & 8) ? 0 : (ks & 1)];
            if constexpr (SCHED & 1) {
                // pass-major: each accumulator's three passes three MFMAs apart (no back-to-back
                // dependent MFMA of one wave)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rh[slot], f[t][1], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rl[slot], f[t][0], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rh[slot], f[t][0], acc[t], 0, 0, 0);
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rh[slot], f[t][0], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rh[slot], f[t][1], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(rl[slot], f[t][0], acc[t], 0, 0, 0);
                }
            }
            const int kn = ks + KV3_RING;
            const int64_t woff = kn < KP_KS ? (int64_t)j * (KP_KS * 512) + kn * 512
                                            : (int64_t)jn * (KP_KS * 512) + (kn - KP_KS) * 512;
            if constexpr (!(SCHED & 4)) {
                rh[slot] = *(const pair8_t*)(Wh + woff);
                rl[slot] = *(const pair8_t*)(Wl + woff);
            } else {
                asm volatile("" : "+v"(rh[slot]), "+v"(rl[slot]));
            }
            if constexpr ((SCHED & 13) == 1) {
                // the next k-step's 8 fragment reads one per MFMA gap from the top of the step (left
                // to itself the compiler issues them after 8 of the 12 MFMAs, and the next step's
                // first MFMA then waits on them), then the rest of the MFMAs, then the W loads
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
            }
            // each k-step's LDS fragment reads stay beside its MFMAs
            __builtin_amdgcn_sched_barrier(0);
        }
        TC* C = (TC*)a.C + (int64_t)plane * rpb * 32;
        float pm[2] = {0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int m = m0 + 32 * t + lr;
            float ss = 0.f;
            if constexpr (!(SCHED & 64)) {
                // lane (lr, lh) holds columns 8 g + 4 lh + 0..3 (g = 0..3) of token lr: the lane
                // pair swaps two 4-column groups (v_permlane32_swap) so that lh = 0 holds columns
                // 0..15 and lh = 1 columns 16..31, then stores them as two 16-byte pieces (half
                // the store instructions, twice the bytes each, of the 8-byte form below)
                // lane (lr, lh) packs its columns 8 g + 4 lh + 0..3 as X = groups 0, 1 and Y = groups
                // 2, 3 (two f16 per dword); one v_permlane32_swap per dword, X as the high half's
                // vdst and Y as the low half's vsrc, leaves lh = 0 with columns 0..15 and lh = 1
                // with 16..31 as (vdst, vsrc) dword pairs in the same order on both halves -- no
                // per-half selects -- stored as two 16-byte pieces
                uint32_t X[4], Y[4];
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const uint32_t w = pack2<TC>(acc[t][4 * g + 2 * e], acc[t][4 * g + 2 * e + 1]);
                        if (g < 2) X[2 * g + e] = w;
                        else Y[2 * (g - 2) + e] = w;
                    }
                if (maxq) {
#pragma unroll
                    for (int d = 0; d < 4; ++d) ss = sq2<TC>(Y[d], sq2<TC>(X[d], ss));
                }
                uint32_t f[4], s2[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    // v_permlane32_swap exchanges vdst of lanes 32..63 with vsrc of lanes 0..31
                    const auto r = __builtin_amdgcn_permlane32_swap(X[d], Y[d], false, false);
                    f[d] = r[0];
                    s2[d] = r[1];
                }
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 o0 = u4{f[0], f[1], s2[0], s2[1]};
                const u4 o1 = u4{f[2], f[3], s2[2], s2[3]};
                if constexpr (SCHED & 16) {
                    asm volatile("" ::"v"(o0), "v"(o1));
                } else if (m < a.M) {
                    // non-temporal (streaming) stores: 306-314 vs 320-327 us alone (profiles/r5_experiments.txt)
                    __builtin_nontemporal_store(o0, (u4*)(C + rbase[t] + 16 * lh));
                    __builtin_nontemporal_store(o1, (u4*)(C + rbase[t] + 16 * lh + 8));
                }
            } else {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const t4 v = t4{(TC)acc[t][4 * g], (TC)acc[t][4 * g + 1], (TC)acc[t][4 * g + 2],
                                    (TC)acc[t][4 * g + 3]};
                    if constexpr (SCHED & 16) asm volatile("" ::"v"(v));
                    else if (m < a.M) *(t4*)(C + rbase[t] + 8 * g + 4 * lh) = v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) ss += (float)v[e] * (float)v[e];
                }
            }
            ss = pair_sum(m < a.M ? ss : 0.f);
            pm[t >> 1] = (t & 1) ? fmaxf(pm[t >> 1], ss) : ss;
        }
        if (maxq) {
#pragma unroll
            for (int gq = 0; gq < 2; ++gq) {
                float x = pm[gq];
#pragma unroll
                for (int off = 1; off < 32; off <<= 1) x = fmaxf(x, __shfl_xor(x, off));
                const int mg = m0 + 64 * gq;
                if (lane == 0 && mg < a.M) a.plane_max2[(int64_t)(mg >> 6) * pm_planes + plane] = x;
            }
        }
    }
}

}  // namespace

extern "C" int cmt_kv_proj(const cmt_gemm_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_kv_proj: null args");
    const cmt_gemm_args& a = *ap;
    // column parts per 128-token tile: the K half (A2 = lowp(mem + pos)) and the V half (A)
    const int parts = a.A2 ? 2 : 1;
    CMT_REQUIRE(a.rows_per_batch > 0 && a.M % a.rows_per_batch == 0, "cmt_kv_proj: bad head-split rows");
    CMT_REQUIRE(a.c_bstride == 0 || (a.c_bstride % 32 == 0 &&
                                     a.c_bstride >= (int64_t)(a.N >> 5) * a.rows_per_batch * 32),
                "cmt_kv_proj: c_bstride must hold the launch's N/32 planes of rows_per_batch rows");
    if (a.w_dtype == CMT_F16P) {
        // split (fp32-accurate) form: f16 pair A / A2 rows, W_hi then W_lo fragment-packed, f16 / bf16 C
        CMT_REQUIRE(a.a_dtype == CMT_F16P && (a.c_dtype == CMT_F16 || a.c_dtype == CMT_BF16),
                    "cmt_kv_proj: split W needs pair A and an f16 / bf16 C");
        CMT_REQUIRE(a.A && a.W && a.C && a.M > 0 && a.K == KP_K && a.batch == 1 && a.a_mode == CMT_A_ROWS &&
                        a.c_mode == CMT_C_HEADSPLIT && a.R == nullptr && !a.relu && a.rows_per_batch > 0 &&
                        a.M % a.rows_per_batch == 0,
                    "cmt_kv_proj: row A, K = 256, head-split C, no residual / relu, batch 1");
        CMT_REQUIRE(a.N % (256 * parts) == 0 && a.N / parts <= KP_MAXB,
                    "cmt_kv_proj: N must be a multiple of 256 per column part, at most 2048 per part");
        CMT_REQUIRE(a.A2 == nullptr || (a.a2_mode == CMT_A2_SELECT && a.a2_cols * 2 == a.N),
                    "cmt_kv_proj: A2 selects the first half of the columns");
        CMT_REQUIRE(a.plane_max2 == nullptr || (a.plane_max_cols % (a.N / parts) == 0 && a.plane_max_cols <= a.N),
                    "cmt_kv_proj: plane_max_cols must be a multiple of the column part (N / parts) <= N");
        CMT_REQUIRE(a.lda % 8 == 0 && (a.A2 == nullptr || a.lda2 % 8 == 0) &&
                        ((uintptr_t)a.A | (uintptr_t)a.W | (uintptr_t)a.C | (uintptr_t)a.A2) % 16 == 0,
                    "cmt_kv_proj: 16-byte aligned operands");
        const int units = cdiv(a.M, KP_BM) * parts;
        // the units past the last full round of one workgroup per CU run as two half units (when a
        // wave has at least two head planes to share)
        const int ncu = cmt_cu_count();
        const int tail = (a.N / parts / 256 >= 2) ? units % ncu : 0;   // 287-296 vs 303-305 us alone (r5al)
        const int nfull = units - tail;
        const unsigned g3 = (unsigned)(nfull + 2 * tail);
        hipStream_t s3 = (hipStream_t)stream;
        if (a.c_dtype == CMT_F16) {
            kvproj_x3_kernel<f16_t, CMT_KV_SCHED><<<g3, 512, 0, s3>>>(a, parts, nfull);
        } else {
            kvproj_x3_kernel<bf16_t, 0><<<g3, 512, 0, s3>>>(a, parts, nfull);
        }
        return cmt_check_launch("cmt_kv_proj");
    }
    CMT_REQUIRE(a.w_dtype == CMT_BF16 || a.w_dtype == CMT_F16, "cmt_kv_proj: w_dtype must be f16 or bf16");
    CMT_REQUIRE(a.a_dtype == a.w_dtype && a.c_dtype == a.w_dtype, "cmt_kv_proj: A and C in the compute dtype");
    CMT_REQUIRE(a.A && a.W && a.C && a.M > 0 && a.K == KP_K && a.batch == 1, "cmt_kv_proj: needs A/W/C, K = 256");
    CMT_REQUIRE(a.a_mode == CMT_A_ROWS && a.c_mode == CMT_C_HEADSPLIT && a.R == nullptr && !a.relu,
                "cmt_kv_proj: row A, head-split C, no residual / relu");
    CMT_REQUIRE(a.rows_per_batch > 0 && a.M % a.rows_per_batch == 0, "cmt_kv_proj: bad head-split rows");
    CMT_REQUIRE(a.N % (256 * parts) == 0 && a.N / parts <= KP_MAXB,
                "cmt_kv_proj: N must be a multiple of 256 per column part, at most 2048 per part");
    CMT_REQUIRE(a.A2 == nullptr || (a.a2_mode == CMT_A2_SELECT && a.a2_cols * 2 == a.N && a.lda2 % 8 == 0),
                "cmt_kv_proj: A2 selects the first half of the columns");
    CMT_REQUIRE(a.plane_max2 == nullptr || (a.plane_max_cols % (a.N / parts) == 0 && a.plane_max_cols <= a.N),
                "cmt_kv_proj: plane_max_cols must be a multiple of the column part (N / parts) <= N");
    CMT_REQUIRE(kv_c_extent_bytes(a) < ((int64_t)1 << 32) - 1, "cmt_kv_proj: C must be < 4 GiB (32-bit offsets)");
    CMT_REQUIRE(a.lda % 8 == 0 && ((uintptr_t)a.A | (uintptr_t)a.W | (uintptr_t)a.C | (uintptr_t)a.A2 |
                                    (uintptr_t)a.bias) % 16 == 0, "cmt_kv_proj: 16-byte aligned operands");
    hipStream_t s = (hipStream_t)stream;
    const unsigned grid = (unsigned)(cdiv(a.M, KP_BM) * parts);
    if (a.w_dtype == CMT_BF16) kvproj_kernel<bf16_t><<<grid, 512, 0, s>>>(a, parts);
    else kvproj_kernel<f16_t><<<grid, 512, 0, s>>>(a, parts);
    return cmt_check_launch("cmt_kv_proj");
}
