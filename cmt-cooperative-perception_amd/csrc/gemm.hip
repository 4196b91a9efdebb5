// MFMA GEMM with fused prologue (pos-add, implicit conv gathers) and epilogue
// (bias, ReLU, residual, dtype cast, head-split scatter) for gfx950.
//
// C[m,n] = act(sum_k Aeff[m,k] * W[n,k] + bias[n]) + R[m,n]
//
// Block = 256 threads = 4 waves in a 2x2 grid; each wave owns a
// (BM/2)x(BN/2) sub-tile built from 32x32 MFMA tiles.  K is consumed in
// 32-deep steps staged through a double-buffered LDS image; the next step's
// global loads are issued before the current step's MFMAs (register staging,
// write-after-compute, one barrier per step).
//
// Low-precision path (f16/bf16): v_mfma_f32_32x32x16_{f16,bf16}; LDS image
// [row][32] with 16-byte chunks XOR-swizzled by (row>>2)&3 so the 16-lane
// groups of ds_read_b128 hit 16 distinct bank slots.
// Exact-f32 path: v_mfma_f32_32x32x2_f32 with the k index permuted as
// k = 16*(lane>>5) + t so each lane reads 16 contiguous floats; LDS rows are
// padded to 36 floats (conflict-free ds_read_b128).
#include "cmt_common.h"

#include <cstdlib>

// conv_halo_x3_kernel's variant bits for dev experiments (dev/build_exp.sh -DCMT_CONV_VAR=n); the
// product build compiles variant 0 only
#ifndef CMT_CONV_VAR
#define CMT_CONV_VAR 0
#endif

namespace {

constexpr int BK = 32;
constexpr int NT = 256;

struct RowInfo {         // per staged row: where the A row comes from
    int valid;           // row < M
    int img, y, x;       // CONV3X3
    int q;               // CONV1D3 position inside its segment
};

template <int AMODE>
__device__ __forceinline__ RowInfo make_row_info(const cmt_gemm_args& a, int row) {
    RowInfo ri;
    ri.valid = row < a.M;
    ri.img = ri.y = ri.x = ri.q = 0;
    if (AMODE == CMT_A_CONV3X3) {
        int hw = a.conv_h * a.conv_w;
        ri.img = row / hw;
        int p = row - ri.img * hw;
        ri.y = p / a.conv_w;
        ri.x = p - ri.y * a.conv_w;
    } else if (AMODE == CMT_A_CONV1D3) {
        ri.q = row % a.seg_len;
    }
    return ri;
}

// Returns the element offset of A[row][k0 .. k0+len) or -1 if the gathered row is padding.
template <int AMODE>
__device__ __forceinline__ int64_t a_offset(const cmt_gemm_args& a, const RowInfo& ri, int row, int k0) {
    if (!ri.valid) return -1;
    if (AMODE == CMT_A_ROWS) {
        return (int64_t)row * a.lda + k0;
    } else if (AMODE == CMT_A_CONV3X3) {
        int C = a.conv_c;
        int tap = k0 / C;
        int cin = k0 - tap * C;
        int yy = ri.y + tap / 3 - 1;
        int xx = ri.x + tap % 3 - 1;
        if (yy < 0 || yy >= a.conv_h || xx < 0 || xx >= a.conv_w) return -1;
        return (((int64_t)ri.img * a.conv_h + yy) * a.conv_w + xx) * a.lda + cin;
    } else {  // CONV1D3
        int C = a.K / 3;
        int tap = k0 / C;
        int c = k0 - tap * C;
        int qq = ri.q + tap - 1;
        if (qq < 0 || qq >= a.seg_len) return -1;
        return (int64_t)(row + tap - 1) * a.lda + c;
    }
}

__device__ __forceinline__ float load_elem(const void* p, int64_t idx, int dt) {
    if (dt == CMT_F32) return ((const float*)p)[idx];
    if (dt == CMT_F16) return (float)((const f16_t*)p)[idx];
    return (float)((const bf16_t*)p)[idx];
}

template <typename T>
__device__ __forceinline__ void store_out(void* C, int64_t idx, int dt, float v) {
    (void)sizeof(T);
    if (dt == CMT_F32) ((float*)C)[idx] = v;
    else if (dt == CMT_F16) ((f16_t*)C)[idx] = (f16_t)v;
    else ((bf16_t*)C)[idx] = (bf16_t)v;
}

template <int BM, int BN>
__device__ __forceinline__ void epilogue(const cmt_gemm_args& a, f32x16 (&acc)[BM / 64][BN / 64],
                                         int m0, int n0, int wm, int wn, int lane) {
    const int h = lane >> 5;
    const int col_l = lane & 31;
    const int z = blockIdx.z;
    const int esz = a.c_dtype == CMT_F32 ? 4 : 2;
    void* Cz = (char*)a.C + (int64_t)z * a.c_bstride * esz;
    const float* biasz = a.bias ? a.bias + (int64_t)z * a.bias_bstride : nullptr;
    const char* Rz = a.R ? (const char*)a.R + (int64_t)z * a.r_bstride * (a.r_dtype == CMT_F32 ? 4 : 2) : nullptr;
    // pass 1: bias, activation, residual (all loads before the first store --
    // vmcnt counts stores on CDNA4, so a load after a store would wait for it)
#pragma unroll
    for (int tn = 0; tn < BN / 64; ++tn) {
        const int col = n0 + wn * (BN / 2) + tn * 32 + col_l;
        const float bias = biasz ? biasz[col] : 0.f;
#pragma unroll
        for (int tm = 0; tm < BM / 64; ++tm) {
            const int row0 = m0 + wm * (BM / 2) + tm * 32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = min(row0 + (r & 3) + 8 * (r >> 2) + 4 * h, a.M - 1);
                float v = acc[tm][tn][r] + bias;
                if (a.relu) v = fmaxf(v, 0.f);
                if (Rz) v += load_elem(Rz, (int64_t)row * a.ldr + col, a.r_dtype);
                acc[tm][tn][r] = v;
            }
        }
    }
    // pass 2: stores
#pragma unroll
    for (int tn = 0; tn < BN / 64; ++tn) {
        const int col = n0 + wn * (BN / 2) + tn * 32 + col_l;
#pragma unroll
        for (int tm = 0; tm < BM / 64; ++tm) {
            // head-split addressing: one division per 32-row tile, the 32 rows
            // cross at most one batch boundary when rows_per_batch >= 32
            const int row0 = m0 + wm * (BM / 2) + tm * 32;
            const int rpb = a.rows_per_batch;
            int b0 = 0, rr0 = 0;
            if (a.c_mode != CMT_C_ROWS) {
                b0 = row0 / rpb;
                rr0 = row0 - b0 * rpb;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int off = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int row = row0 + off;
                if (row >= a.M) continue;
                int64_t idx;
                if (a.c_mode == CMT_C_ROWS) {
                    idx = (int64_t)row * a.ldc + col;
                } else {
                    int b = b0, rr = rr0 + off;
                    if (rpb >= 32) {
                        if (rr >= rpb) { rr -= rpb; ++b; }
                    } else {
                        b = row / rpb;
                        rr = row - b * rpb;
                    }
                    idx = (((int64_t)b * (a.N >> 5) + (col >> 5)) * rpb + rr) * 32 + (col & 31);
                }
                store_out<float>(Cz, idx, a.c_dtype, acc[tm][tn][r]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// f16 / bf16 compute
// ---------------------------------------------------------------------------
template <int CPR>
__device__ __forceinline__ int swz(int row, int c) {
    // 16-byte chunk permutation of an LDS row holding CPR chunks: the 16-lane
    // groups of ds_read_b128 (rows {0-3,12-15,20-27} / {4-11,16-19,28-31} at a
    // fixed chunk) land on 16 distinct bank slots for CPR = 4, 8, 16.
    return c ^ ((row / (16 / CPR)) & (CPR - 1));
}

template <typename CT, int BM, int BN, int LBK, int AMODE, bool A_F32>
__global__ __launch_bounds__(NT) void gemm_lowp_kernel(cmt_gemm_args a) {
    typedef typename mfma_traits<CT>::frag frag;
    constexpr int CPR = LBK / 8;               // 16-byte chunks per LDS row
    constexpr int ACH = BM * CPR / NT;         // A chunks staged per thread per k-step
    constexpr int BCH = BN * CPR / NT;
    static_assert(ACH >= 1 && BCH >= 1, "tile too small for the thread count");
    __shared__ __attribute__((aligned(16))) CT As[2][BM * LBK];
    __shared__ __attribute__((aligned(16))) CT Bs[2][BN * LBK];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * BM;
    const int z = blockIdx.z;

    const char* Ab = (const char*)a.A + (int64_t)z * a.a_bstride * (A_F32 ? 4 : 2);
    const CT* Wb = (const CT*)a.W + (int64_t)z * a.w_bstride;
    const bool use_a2 = (AMODE == CMT_A_ROWS) && a.A2 != nullptr && n0 < a.a2_cols;

    RowInfo ri[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) ri[i] = make_row_info<AMODE>(a, m0 + (tid + NT * i) / CPR);

    frag areg[ACH];
    frag breg[BCH];

    auto load_tiles = [&](int k0) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / CPR, c = idx % CPR;
            const int kk = k0 + c * 8;
            const int64_t off = a_offset<AMODE>(a, ri[i], m0 + row, kk);
            if (off < 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) areg[i][j] = (CT)0.f;
            } else if (A_F32) {
                const float* p = (const float*)Ab + off;
                f32x4 v0 = *(const f32x4*)p;
                f32x4 v1 = *(const f32x4*)(p + 4);
                if (use_a2) {
                    const float* p2 = (const float*)a.A2 + (int64_t)(m0 + row) * a.lda2 + kk;
                    v0 += *(const f32x4*)p2;
                    v1 += *(const f32x4*)(p2 + 4);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    areg[i][j] = (CT)v0[j];
                    areg[i][j + 4] = (CT)v1[j];
                }
            } else {
                areg[i] = *(const frag*)((const CT*)Ab + off);
            }
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / CPR, c = idx % CPR;
            breg[i] = *(const frag*)(Wb + (int64_t)(n0 + row) * a.ldw + k0 + c * 8);
        }
    };
    auto store_tiles = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / CPR, c = idx % CPR;
            *(frag*)(&As[buf][row * LBK + 8 * swz<CPR>(row, c)]) = areg[i];
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / CPR, c = idx % CPR;
            *(frag*)(&Bs[buf][row * LBK + 8 * swz<CPR>(row, c)]) = breg[i];
        }
    };

    f32x16 acc[BM / 64][BN / 64];
#pragma unroll
    for (int i = 0; i < BM / 64; ++i)
#pragma unroll
        for (int j = 0; j < BN / 64; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = a.K / LBK;
    load_tiles(0);
    store_tiles(0);
    __syncthreads();
    const int lr = lane & 31;
    const int lh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_tiles((kt + 1) * LBK);
#pragma unroll
        for (int ks = 0; ks < LBK / 16; ++ks) {
            frag af[BM / 64], bfr[BN / 64];
#pragma unroll
            for (int tm = 0; tm < BM / 64; ++tm) {
                const int row = wm * (BM / 2) + tm * 32 + lr;
                af[tm] = *(const frag*)(&As[cur][row * LBK + 8 * swz<CPR>(row, 2 * ks + lh)]);
            }
#pragma unroll
            for (int tn = 0; tn < BN / 64; ++tn) {
                const int row = wn * (BN / 2) + tn * 32 + lr;
                bfr[tn] = *(const frag*)(&Bs[cur][row * LBK + 8 * swz<CPR>(row, 2 * ks + lh)]);
            }
#pragma unroll
            for (int tm = 0; tm < BM / 64; ++tm)
#pragma unroll
                for (int tn = 0; tn < BN / 64; ++tn)
                    acc[tm][tn] = mfma_traits<CT>::mma(af[tm], bfr[tn], acc[tm][tn]);
        }
        if (kt + 1 < nk) store_tiles(cur ^ 1);
        __syncthreads();
    }
    epilogue<BM, BN>(a, acc, m0, n0, wm, wn, lane);
}

// ---------------------------------------------------------------------------
// exact f32 compute (v_mfma_f32_32x32x2_f32)
// ---------------------------------------------------------------------------
constexpr int LDF = 36;  // padded LDS row (floats)

template <int BM, int BN, int AMODE>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(cmt_gemm_args a) {
    constexpr int ACH = BM / 32;  // float4 chunks per thread
    constexpr int BCH = BN / 32;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDF];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDF];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * BM;
    const int z = blockIdx.z;

    const float* Ab = (const float*)a.A + (int64_t)z * a.a_bstride;
    const float* Wb = (const float*)a.W + (int64_t)z * a.w_bstride;
    const bool use_a2 = (AMODE == CMT_A_ROWS) && a.A2 != nullptr && n0 < a.a2_cols;

    RowInfo ri[ACH];
    int arow[ACH], achunk[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        int idx = tid + NT * i;
        arow[i] = idx >> 3;
        achunk[i] = idx & 7;
        ri[i] = make_row_info<AMODE>(a, m0 + arow[i]);
    }
    f32x4 areg[ACH], breg[BCH];

    auto load_tiles = [&](int k0) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int kk = k0 + achunk[i] * 4;
            int64_t off = a_offset<AMODE>(a, ri[i], m0 + arow[i], kk);
            if (off < 0) {
                areg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
                areg[i] = *(const f32x4*)(Ab + off);
                if (use_a2) areg[i] += *(const f32x4*)((const float*)a.A2 + (int64_t)(m0 + arow[i]) * a.lda2 + kk);
            }
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            int idx = tid + NT * i;
            int row = idx >> 3, c = idx & 7;
            breg[i] = *(const f32x4*)(Wb + (int64_t)(n0 + row) * a.ldw + k0 + c * 4);
        }
    };
    auto store_tiles = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) *(f32x4*)(&As[buf][arow[i] * LDF + achunk[i] * 4]) = areg[i];
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            int idx = tid + NT * i;
            *(f32x4*)(&Bs[buf][(idx >> 3) * LDF + (idx & 7) * 4]) = breg[i];
        }
    };

    f32x16 acc[BM / 64][BN / 64];
#pragma unroll
    for (int i = 0; i < BM / 64; ++i)
#pragma unroll
        for (int j = 0; j < BN / 64; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = a.K / BK;
    load_tiles(0);
    store_tiles(0);
    __syncthreads();
    const int lr = lane & 31;
    const int lh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_tiles((kt + 1) * BK);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            f32x4 af[BM / 64], bfr[BN / 64];
#pragma unroll
            for (int tm = 0; tm < BM / 64; ++tm)
                af[tm] = *(const f32x4*)(&As[cur][(wm * (BM / 2) + tm * 32 + lr) * LDF + 16 * lh + 4 * kc]);
#pragma unroll
            for (int tn = 0; tn < BN / 64; ++tn)
                bfr[tn] = *(const f32x4*)(&Bs[cur][(wn * (BN / 2) + tn * 32 + lr) * LDF + 16 * lh + 4 * kc]);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int tm = 0; tm < BM / 64; ++tm)
#pragma unroll
                    for (int tn = 0; tn < BN / 64; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm][t], bfr[tn][t], acc[tm][tn], 0, 0, 0);
        }
        if (kt + 1 < nk) store_tiles(cur ^ 1);
        __syncthreads();
    }
    epilogue<BM, BN>(a, acc, m0, n0, wm, wn, lane);
}


// ---------------------------------------------------------------------------
// LDS-DMA path (A already in the compute dtype).
//
// Tiles are copied HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging):
// one wave-instruction moves 8 rows x 128 B (64 k of one stage) into a
// lane-linear LDS image; the 16-byte chunk permutation (row>>1)&7 is applied
// to the SOURCE address and undone on the ds_read_b128 side (guide rule 21),
// so the fragment reads are bank-conflict free.  S stages are kept in flight
// with counted vmcnt waits and one raw s_barrier per k-step.  Gathered A rows
// (3x3 / 1D-3 convolution taps outside the map) read a zero page.
//
// The MFMA is issued as C^T = W . A^T (W rows on the A operand), so each lane
// ends with 4 consecutive output columns of one row: 16-byte (fp32) / 8-byte
// stores, 4 per 32x32 tile instead of 16 scalar ones.
//
// Workgroups are numbered XCD-aware: the round-robin dispatch order is
// remapped so one XCD walks a contiguous band of M tiles with every N tile,
// and the band's A rows and all of W stay in that XCD's L2.
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(64))) char g_zero_page[256];

typedef const __attribute__((address_space(1))) void* gaddr_t;
typedef __attribute__((address_space(3))) void* laddr_t;

__device__ __forceinline__ void glds16(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds((gaddr_t)src, (laddr_t)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

template <int PER, int S>
__device__ __forceinline__ void wait_tiles(int inflight) {
    if (S > 3 && inflight >= 3) wait_vm_lgkm<(S > 3 ? 3 * PER : 0)>();
    else if (S > 2 && inflight == 2) wait_vm_lgkm<(S > 2 ? 2 * PER : 0)>();
    else if (inflight == 1) wait_vm_lgkm<PER>();
    else wait_vm_lgkm<0>();
}

template <typename CT>
__device__ __forceinline__ void store4(void* C, int64_t idx, int dt, f32x4 v) {
    if (dt == CMT_F32) {
        *(f32x4*)((float*)C + idx) = v;
    } else if (dt == CMT_F16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 h = {(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3]};
        *(h4*)((f16_t*)C + idx) = h;
    } else {
        typedef __bf16 b4 __attribute__((ext_vector_type(4)));
        b4 h = {(bf16_t)v[0], (bf16_t)v[1], (bf16_t)v[2], (bf16_t)v[3]};
        *(b4*)((bf16_t*)C + idx) = h;
    }
}

// lo_off: element distance of a CMT_F16P row's lo half (its logical width)
__device__ __forceinline__ f32x4 load4(const void* p, int64_t idx, int dt, int lo_off = 0) {
    if (dt == CMT_F32) return *(const f32x4*)((const float*)p + idx);
    if (dt == CMT_F16P) {
        typedef pair_t b4 __attribute__((ext_vector_type(4)));
        const b4 h = *(const b4*)((const pair_t*)p + idx);
        const b4 l = *(const b4*)((const pair_t*)p + idx + lo_off);
        return f32x4{(float)h[0] + (float)l[0], (float)h[1] + (float)l[1], (float)h[2] + (float)l[2],
                     (float)h[3] + (float)l[3]};
    }
    if (dt == CMT_F16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 h = *(const h4*)((const f16_t*)p + idx);
        return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    }
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    b4 h = *(const b4*)((const bf16_t*)p + idx);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}

// Main loop of the LDS-DMA GEMM for one BM x BN output tile (4 waves in a
// WM x (4/WM) grid; each wave owns (BM/WM) x (BN*WM/4) as TM x TN 32x32 MFMA
// tiles).  Accumulators are in the swapped C^T layout: lane = output row.
//
// X3 (A and W both CMT_F16P, cmt_hip.h): every stage carries four tiles --
// A_hi, A_lo, W_hi, W_lo of the same 64 k -- and each k step runs the three
// products A_hi W_hi + A_lo W_hi + A_hi W_lo on them, so one staged byte feeds
// 3/2 MFMAs instead of one (a stage per product re-streams A_hi and W_hi) and
// the k loop is K / 64 steps long, not 3K / 64.  The A row's lo half starts at
// its logical width (K for rows, the channel count for the implicit convs),
// W's at K.
template <typename CT, int BM, int BN, int S, int AMODE, int WM, bool X3 = false>
struct DmaTile {
    static constexpr int KS = 64;                          // k per stage: one 128-byte LDS row per tile row
    static constexpr int NPL = X3 ? 2 : 1;                 // planes per operand (hi, lo)
    static constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = NPL * (A_BYTES + B_BYTES);
    static constexpr int APER = BM / 32, BPER = BN / 32;   // 256 lanes x 16 B = 32 rows per block-wide copy
    static constexpr int PER = NPL * (APER + BPER);        // glds per thread per stage
    static constexpr int WN = 4 / WM;
    static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static constexpr int SMEM = S * STAGE;
    static_assert(TM >= 1 && TN >= 1 && APER >= 1, "tile too small");

    // k steps kt0 .. kt0 + nk - 1 (of 64) of the logical K; nk < 0: all of them
    static __device__ __forceinline__ void run(const cmt_gemm_args& a, char* smem, int m0, int n0, int z,
                                               f32x16 (&acc)[TM][TN], int kt0 = 0, int nk = -1) {
        typedef typename mfma_traits<CT>::frag frag;
        const int tid = threadIdx.x;
        const int lane = tid & 63;
        const int wave = tid >> 6;
        const int wm = wave / WN, wn = wave % WN;

        const bool sel_a2 = AMODE == CMT_A_ROWS && a.A2 != nullptr && n0 < a.a2_cols;
        const CT* Ab = (const CT*)(sel_a2 ? a.A2 : a.A) + (int64_t)z * a.a_bstride;
        const int64_t lda = sel_a2 ? a.lda2 : a.lda;
        const CT* Wb = (const CT*)a.W + (int64_t)z * a.w_bstride;

        // per-thread source rows: copy i of this wave covers tile rows (4i + wave)*8 + lane/8
        const int ch = lane & 7;
        const CT* asrc[APER];
        RowInfo ri[APER];
        int acs[APER];
#pragma unroll
        for (int i = 0; i < APER; ++i) {
            const int row = (4 * i + wave) * 8 + (lane >> 3);
            acs[i] = (ch ^ ((row >> 1) & 7)) * 8;
            const int m = m0 + row;
            ri[i] = make_row_info<AMODE>(a, m);
            asrc[i] = Ab + (int64_t)min(m, a.M - 1) * lda + acs[i];
        }
        const CT* bsrc[BPER];
#pragma unroll
        for (int i = 0; i < BPER; ++i) {
            const int row = (4 * i + wave) * 8 + (lane >> 3);
            bsrc[i] = Wb + (int64_t)(n0 + row) * a.ldw + (ch ^ ((row >> 1) & 7)) * 8;
        }

        // implicit convs (3x3, 1D k = 3): the stages arrive in increasing k order and a tap spans
        // (tap width) / 64 stages, so each row's gathered offset is recomputed once per tap
        // (9 or 3 times per tile), not per stage (no integer division in the k loop)
        const int tapw = AMODE == CMT_A_CONV3X3 ? a.conv_c : (AMODE == CMT_A_CONV1D3 ? a.K / 3 : a.K);
        const int ntaps = AMODE == CMT_A_CONV3X3 ? 9 : (AMODE == CMT_A_CONV1D3 ? 3 : 1);
        (void)ntaps;
        const int a_lo = AMODE == CMT_A_ROWS ? a.K : tapw;    // element offset of an A row's lo half
        int ctap = -1, ccin = 0;
        int64_t toff[APER];
        auto issue = [&](int buf, int kt) {
            char* sb = smem + buf * STAGE;
            int ka, kw;   // A / W column of this stage's first k
            if constexpr (AMODE != CMT_A_ROWS) {
                // the same per-tap cache for the 1D k = 3 conv (taps of K / 3 columns)
                if (ctap < 0) {
                    const int k0 = kt * KS;
                    ctap = k0 / tapw;
                    ccin = k0 - ctap * tapw;
#pragma unroll
                    for (int i = 0; i < APER; ++i)
                        toff[i] = a_offset<AMODE>(a, ri[i], m0 + (4 * i + wave) * 8 + (lane >> 3), ctap * tapw);
                } else if ((ccin += KS) == tapw) {
                    ccin = 0;
                    ++ctap;
#pragma unroll
                    for (int i = 0; i < APER; ++i)
                        toff[i] = a_offset<AMODE>(a, ri[i], m0 + (4 * i + wave) * 8 + (lane >> 3), ctap * tapw);
                }
                ka = ccin;
                kw = ctap * tapw + ccin;
            } else {
                ka = kw = kt * KS;
            }
#pragma unroll
            for (int i = 0; i < APER; ++i) {
                const CT* src;
                if (AMODE == CMT_A_ROWS)
                    src = asrc[i] + ka;
                else
                    src = toff[i] < 0 ? nullptr : (const CT*)Ab + toff[i] + ka + acs[i];
                glds16(src ? (const void*)src : (const void*)g_zero_page, sb + (4 * i + wave) * 1024);
                if constexpr (X3)
                    glds16(src ? (const void*)(src + a_lo) : (const void*)g_zero_page,
                           sb + A_BYTES + (4 * i + wave) * 1024);
            }
#pragma unroll
            for (int i = 0; i < BPER; ++i) {
                glds16(bsrc[i] + kw, sb + NPL * A_BYTES + (4 * i + wave) * 1024);
                if constexpr (X3) glds16(bsrc[i] + kw + a.K, sb + NPL * A_BYTES + B_BYTES + (4 * i + wave) * 1024);
            }
        };

#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

        if (nk < 0) nk = a.K / KS;
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s < nk) issue(s, kt0 + s);

        const int lr = lane & 31;
        const int lh = lane >> 5;
        for (int kt = 0; kt < nk; ++kt) {
            const int last = min(nk - 1, kt == 0 ? S - 1 : kt + S - 2);
            wait_tiles<PER, S>(last - kt);
            barrier_mem();
            // every wave is past its reads of stage kt-1: refill that buffer
            if (kt >= 1 && kt + S - 1 < nk) issue((kt - 1) % S, kt0 + kt + S - 1);
            const char* As = smem + (kt % S) * STAGE;
            const char* Bs = As + NPL * A_BYTES;
#pragma unroll
            for (int ks = 0; ks < KS / 16; ++ks) {
                frag af[TM], bfr[TN];
                const int kc = 2 * ks + lh;
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    const int r = wm * (BM / WM) + tm * 32 + lr;
                    af[tm] = *(const frag*)(As + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4));
                }
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const int r = wn * (BN / WN) + tn * 32 + lr;
                    bfr[tn] = *(const frag*)(Bs + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4));
                }
                if constexpr (X3) {
                    frag al[TM], bl[TN];
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm) {
                        const int r = wm * (BM / WM) + tm * 32 + lr;
                        al[tm] = *(const frag*)(As + A_BYTES + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4));
                    }
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) {
                        const int r = wn * (BN / WN) + tn * 32 + lr;
                        bl[tn] = *(const frag*)(Bs + B_BYTES + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4));
                    }
                    // the two small products first, then the hi product, per accumulator
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<CT>::mma(bfr[tn], al[tm], acc[tm][tn]);
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<CT>::mma(bl[tn], af[tm], acc[tm][tn]);
                }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<CT>::mma(bfr[tn], af[tm], acc[tm][tn]);
            }
        }
    }
};

// XCD-aware tile order (bijective remap of the round-robin dispatch): one XCD
// walks a contiguous band of M tiles with every N tile.
__device__ __forceinline__ void xcd_tile(int tiles_m, int tiles_n, int batch, int& z, int& mt, int& nt) {
    const int nwg = tiles_m * tiles_n * batch;
    const int orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int per_z = tiles_m * tiles_n;
    z = wg / per_z;
    const int rem = wg - z * per_z;
    mt = rem / tiles_n;
    nt = rem - mt * tiles_n;
}

template <typename CT, int BM, int BN, int S, int AMODE, bool X3 = false>
__global__ __launch_bounds__(NT) void gemm_dma_kernel(cmt_gemm_args a, int tiles_m, int tiles_n) {
    typedef DmaTile<CT, BM, BN, S, AMODE, 2, X3> Tile;
    constexpr int TM = Tile::TM, TN = Tile::TN;
    __shared__ __attribute__((aligned(16))) char smem[Tile::SMEM];
    int z, mt, nt;
    // split-K (batch 1): grid z enumerates the K parts
    const int ksp = a.k_splits > 1 ? a.k_splits : 1;
    xcd_tile(tiles_m, tiles_n, a.batch * ksp, z, mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    f32x16 acc[TM][TN];
    const int part = ksp > 1 ? z : 0;
    if (ksp > 1) z = 0;
    const int nkp = a.K / Tile::KS / ksp;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 31;
    const int lh = lane >> 5;
    const int esz = a.c_dtype == CMT_F32 ? 4 : 2;
    char* Cz = (char*)a.C + ((int64_t)z * a.c_bstride + part * a.c_split_stride) * esz;
    const float* biasz = a.bias && part == 0 ? a.bias + (int64_t)z * a.bias_bstride : nullptr;
    const char* Rz = a.R && part == 0 ? (const char*)a.R + (int64_t)z * a.r_bstride * (a.r_dtype == CMT_F32 ? 4 : 2)
                                      : nullptr;
    // bias and residual are read BEFORE the k loop: issued ahead of the first LDS-DMA stage they
    // complete with it (vmcnt is in order), instead of costing the epilogue one more memory round
    // trip -- the decoder's 900-row GEMMs are latency-bound (the split-K out-projections and fc2
    // carry the residual in part 0)
    f32x4 bv[TN][4], rv[TM][TN][4];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * (BN / 2) + tn * 32 + 8 * g + 4 * lh;
            bv[tn][g] = biasz ? *(const f32x4*)(biasz + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    if (Rz) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = min(m0 + wm * (BM / 2) + tm * 32 + lr, a.M - 1);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    rv[tm][tn][g] = load4(Rz, (int64_t)m * a.ldr + n0 + wn * (BN / 2) + tn * 32 + 8 * g + 4 * lh,
                                          a.r_dtype, a.N);
        }
    }
    Tile::run(a, smem, m0, n0, z, acc, part * nkp, nkp);

    // ---- epilogue: lane = output row, 4 consecutive columns per register group.
    // X3 with a.range_flag: the f16-pair range guard of x3_epilogue on the pre-activation values
    bool bad = false;
    if (Rz) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 r = rv[tm][tn][g];
                    // bias + relu come first; keep R apart only when relu is on
                    if (a.relu) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float v = acc[tm][tn][4 * g + j] + bv[tn][g][j];
                            if constexpr (X3) bad |= f16_unrepresentable(v);
                            acc[tm][tn][4 * g + j] = fmaxf(v, 0.f) + r[j];
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            acc[tm][tn][4 * g + j] += bv[tn][g][j] + r[j];
                            if constexpr (X3) bad |= f16_unrepresentable(acc[tm][tn][4 * g + j]);
                        }
                    }
                }
        }
    } else {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float v = acc[tm][tn][4 * g + j] + bv[tn][g][j];
                        if constexpr (X3) bad |= f16_unrepresentable(v);
                        acc[tm][tn][4 * g + j] = a.relu ? fmaxf(v, 0.f) : v;
                    }
    }
    if constexpr (X3) raise_range_flag(a.range_flag, bad);
    // ---- stores staged through LDS: the swapped layout leaves each lane 4
    // columns of one row (8/16-byte pieces at a row stride); the tile is
    // written to LDS (16-byte chunks XOR-swizzled by row) and read back so
    // every wave instruction stores 1 KB of contiguous memory (head-split:
    // 16 rows x 64 B of one head; rows: whole row segments).
    // A CMT_F16P C is staged and stored twice: the hi halves, then the lo
    // halves N columns further (rows) or 32 elements further (head split).
    const int npass = a.c_dtype == CMT_F16P ? 2 : 1;
    for (int pass = 0; pass < npass; ++pass) {
        barrier_mem();                                       // every wave is done with the staging ring
        const int cpr = BN * esz / 16;                       // 16-byte chunks per tile row (power of two)
        const int cpe = 16 / esz;                            // elements per chunk
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int row = wm * (BM / 2) + tm * 32 + lr;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c0 = wn * (BN / 2) + tn * 32 + 8 * g + 4 * lh;     // first of 4 columns
                    const int ch = c0 / cpe;
                    char* dst = smem + row * (BN * esz) + ((ch ^ (row & (cpr - 1))) << 4) + (c0 % cpe) * esz;
                    f32x4 v = {acc[tm][tn][4 * g], acc[tm][tn][4 * g + 1], acc[tm][tn][4 * g + 2],
                               acc[tm][tn][4 * g + 3]};
                    if (pass) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] -= (float)(pair_t)v[j];   // lo = f16(x - hi)
                    }
                    store4<CT>(dst, 0, a.c_dtype == CMT_F16P ? CMT_F16 : a.c_dtype, v);
                }
        }
        barrier_mem();
        const bool headsplit = a.c_mode != CMT_C_ROWS;
        const int lcpr = esz == 4 ? __builtin_ctz(BN / 4) : __builtin_ctz(BN / 8);   // log2 chunks per row
        const int lcph = esz == 4 ? 3 : 2;                   // log2 chunks per 32-column head slice
        constexpr int LBM = __builtin_ctz(BM);
        // batch of the tile's first row; a tile spans at most two batches when rows_per_batch >= BM
        const int rpb = headsplit ? a.rows_per_batch : 1;
        const int b0 = headsplit ? m0 / rpb : 0;
        const int rr0 = m0 - b0 * rpb;
        // head-plane max of squared row norms (cmt_gemm_args.plane_max2, 16-bit C):
        // with 4 chunks per 32-column head row one iteration of the loop below
        // covers one head plane x 64 rows -- one entry
        if (headsplit && a.plane_max2 != nullptr && esz == 2) {
            constexpr int PITERS = BM * BN / 8 / NT;         // 16-byte chunks of the 16-bit tile per thread
            float* red = (float*)(smem + BM * BN * 2);       // [iteration][wave], after the staged tile
#pragma unroll
            for (int it = 0; it < PITERS; ++it) {
                const int q = threadIdx.x + it * NT;
                const int h = q >> (LBM + 2);
                const int rem = q & ((BM << 2) - 1);
                const int row = rem >> 2;
                const int c = (h << 2) + (rem & 3);
                const f32x4 v = *(const f32x4*)(smem + row * (BN * 2) + ((c ^ (row & ((1 << lcpr) - 1))) << 4));
                float ss = 0.f;
                if (m0 + row < a.M && n0 + c * 8 < a.plane_max_cols) {
                    if (a.c_dtype == CMT_BF16) {
                        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 w = __builtin_bit_cast(u32x4, v);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float lo = __uint_as_float(w[j] << 16), hi = __uint_as_float(w[j] & 0xffff0000u);
                            ss += lo * lo + hi * hi;
                        }
                    } else {
                        const f16x8 hv = __builtin_bit_cast(f16x8, v);
#pragma unroll
                        for (int j = 0; j < 8; ++j) ss += (float)hv[j] * (float)hv[j];
                    }
                }
                ss += __shfl_xor(ss, 1);                     // the 4 chunks of one head row
                ss += __shfl_xor(ss, 2);
#pragma unroll
                for (int off = 4; off < 64; off <<= 1) ss = fmaxf(ss, __shfl_xor(ss, off));
                if ((threadIdx.x & 63) == 0) red[it * 4 + (threadIdx.x >> 6)] = ss;
            }
            barrier_mem();
            if ((int)threadIdx.x < PITERS) {
                const int itx = threadIdx.x;
                const float mx = fmaxf(fmaxf(red[itx * 4], red[itx * 4 + 1]), fmaxf(red[itx * 4 + 2], red[itx * 4 + 3]));
                const int q0 = itx * NT;
                const int plane = (n0 >> 5) + (q0 >> (LBM + 2));
                const int row0 = (q0 & ((BM << 2) - 1)) >> 2;
                if (plane * 32 < a.plane_max_cols)
                    a.plane_max2[(int64_t)((m0 + row0) >> 6) * (a.plane_max_cols >> 5) + plane] = mx;
            }
        }
#pragma unroll 4
        for (int q = threadIdx.x; q < (BM << lcpr); q += NT) {
            int row, c;
            if (headsplit) {                                 // head-major, then row, then chunk: contiguous in memory
                const int h = q >> (LBM + lcph);
                const int rem = q & ((BM << lcph) - 1);
                row = rem >> lcph;
                c = (h << lcph) + (rem & ((1 << lcph) - 1));
            } else {
                row = q >> lcpr;
                c = q & ((1 << lcpr) - 1);
            }
            const int m = m0 + row;
            if (m >= a.M) continue;
            const f32x4 v = *(const f32x4*)(smem + row * (BN * esz) + ((c ^ (row & ((1 << lcpr) - 1))) << 4));
            const int n = n0 + c * cpe;
            int64_t idx;
            if (headsplit) {
                int bb = b0, rr = rr0 + row;
                if (rpb >= BM) {
                    if (rr >= rpb) { rr -= rpb; ++bb; }
                } else {
                    bb = m / rpb;
                    rr = m - bb * rpb;
                }
                // a CMT_F16P C: 64 elements per (head, row) -- the hi row, then the lo row
                idx = a.c_dtype == CMT_F16P
                          ? (((int64_t)bb * (a.N >> 5) + (n >> 5)) * rpb + rr) * 64 + (pass ? 32 : 0) + (n & 31)
                          : (((int64_t)bb * (a.N >> 5) + (n >> 5)) * rpb + rr) * 32 + (n & 31);
            } else {
                idx = (int64_t)m * a.ldc + n + (pass ? a.N : 0);
            }
            *(f32x4*)(Cz + idx * esz) = v;                   // 16 bytes: 4 fp32 or 8 f16/bf16 values
        }

    }
}

// Epilogue of the 8-wave split tiles (gemm_x3_kernel, conv_halo_x3_kernel), row-mode C:
// bias / relu / residual loads first, then the tile staged through LDS (the ring is
// free) and stored as whole row segments (a CMT_F16P C in two passes, hi then lo).
template <int BM, int TM, int TN, int WNW, int NTX>
__device__ __forceinline__ void x3_epilogue(const cmt_gemm_args& a, f32x16 (&acc)[TM][TN], char* smem, int m0, int n0,
                                            int z, int wm, int wn) {
    constexpr int BN = 128;
    const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
    const int esz = a.c_dtype == CMT_F32 ? 4 : 2;
    char* Cz = (char*)a.C + (int64_t)z * a.c_bstride * esz;
    const float* biasz = a.bias ? a.bias + (int64_t)z * a.bias_bstride : nullptr;
    const char* Rz = a.R ? (const char*)a.R + (int64_t)z * a.r_bstride * (a.r_dtype == CMT_F32 ? 4 : 2) : nullptr;
    // range guard (a.range_flag): a pre-activation value outside the f16 pair format means a
    // non-finite or too large input element reached this tile (0 x inf is NaN, so every output
    // of its 3x3 neighbourhood shows it), or the output itself cannot be carried as a pair
    bool bad = false;
    f32x4 bv[TN][4];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * (BN / WNW) + tn * 32 + 8 * g + 4 * lh;
            bv[tn][g] = biasz ? *(const f32x4*)(biasz + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int m = min(m0 + wm * 64 + tm * 32 + lr, a.M - 1);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = n0 + wn * (BN / WNW) + tn * 32 + 8 * g + 4 * lh;
                const f32x4 r = Rz ? load4(Rz, (int64_t)m * a.ldr + n, a.r_dtype, a.N) : f32x4{0.f, 0.f, 0.f, 0.f};
                if (a.relu) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float t = acc[tm][tn][4 * g + j] + bv[tn][g][j];
                        bad |= f16_unrepresentable(t);
                        acc[tm][tn][4 * g + j] = fmaxf(t, 0.f) + r[j];
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[tm][tn][4 * g + j] += bv[tn][g][j] + r[j];
                        bad |= f16_unrepresentable(acc[tm][tn][4 * g + j]);
                    }
                }
            }
    }
    const int npass = a.c_dtype == CMT_F16P ? 2 : 1;
    const int cpr = BN * esz / 16;                            // 16-byte chunks per tile row
    const int cpe = 16 / esz;                                 // elements per chunk
    const int lcpr = esz == 4 ? 5 : 4;                        // log2(cpr) for BN = 128
    // CONV3X3_NCHW with A2 (cmt_hip.h): a second output out + A2[m] at C + c_split_stride
    const bool two = a.a_mode == CMT_A_CONV3X3_NCHW && a.A2 != nullptr;
    for (int out = 0; out < (two ? 2 : 1); ++out) {
    if (out == 1) {
        Cz += a.c_split_stride * esz;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = min(m0 + wm * 64 + tm * 32 + lr, a.M - 1);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = n0 + wn * (BN / WNW) + tn * 32 + 8 * g + 4 * lh;
                    const f32x4 pv = *(const f32x4*)((const float*)a.A2 + (int64_t)m * a.lda2 + n);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[tm][tn][4 * g + j] += pv[j];
                        bad |= f16_unrepresentable(acc[tm][tn][4 * g + j]);
                    }
                }
        }
        raise_range_flag(a.range_flag, bad);
    }
    if (!two) raise_range_flag(a.range_flag, bad);
    for (int pass = 0; pass < npass; ++pass) {
        barrier_mem();                                        // every wave is done with the ring / last pass
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int row = wm * 64 + tm * 32 + lr;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c0 = wn * (BN / WNW) + tn * 32 + 8 * g + 4 * lh;
                    const int c = c0 / cpe;
                    char* dst = smem + row * (BN * esz) + ((c ^ (row & (cpr - 1))) << 4) + (c0 % cpe) * esz;
                    f32x4 v = {acc[tm][tn][4 * g], acc[tm][tn][4 * g + 1], acc[tm][tn][4 * g + 2],
                               acc[tm][tn][4 * g + 3]};
                    if (pass) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] -= (float)(pair_t)v[j];   // lo = f16(x - hi)
                    }
                    store4<pair_t>(dst, 0, a.c_dtype == CMT_F16P ? CMT_F16 : a.c_dtype, v);
                }
        }
        barrier_mem();
#pragma unroll 4
        for (int q = tid; q < (BM << lcpr); q += NTX) {
            const int row = q >> lcpr, c = q & (cpr - 1);
            const int m = m0 + row;
            if (m >= a.M) continue;
            const f32x4 v = *(const f32x4*)(smem + row * (BN * esz) + ((c ^ (row & (cpr - 1))) << 4));
            const int64_t idx = (int64_t)m * a.ldc + n0 + c * cpe + (pass ? a.N : 0);
            *(f32x4*)(Cz + idx * esz) = v;
        }
    }
    }
}

// ---------------------------------------------------------------------------
// Split (CMT_F16P) GEMM for the large problems of the 'ref' policy (shared_conv,
// the BEV / RV position MLPs): BM x 128 tiles (BM 256 or 128), 8 waves, 32-deep
// k stages in an S-slot LDS-DMA ring.
//
// Each stage carries A_hi, A_lo, W_hi, W_lo of 32 k (64-byte LDS rows; 16-byte
// chunks XOR-swizzled by (row >> 2) & 3 on the source address, so the 16-lane
// groups of ds_read_b128 hit 16 distinct bank slots) and each 16-k step runs the
// three products W_hi A_lo + W_lo A_hi + W_hi A_hi in the order of the 128 x 128
// DmaTile<..., X3> -- the same fp32 accumulation sequence, so the two kernels
// give bit-identical outputs.  Against that tile (2 stages of 64 k, 4 waves, one
// wave per SIMD) a BM = 256 tile stages 1.33x the MFMA work per byte and keeps
// 2 stages in flight behind the one being read (the 64 KB fills of the 2-stage
// ring were the pace: ~36 GB/s per CU against 88 for the MFMA rate).
// Row-mode C only (fp32, f16 / bf16 or pair), bias / ReLU / residual, batch.
// ---------------------------------------------------------------------------
template <int BM, int AMODE>
struct X3Tile {
    static constexpr int BN = 128, KS = 32, ROWB = KS * 2, NTX = 512;
    static constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
    static constexpr int STAGE = 2 * (A_BYTES + B_BYTES);
    static constexpr int S = BM == 256 ? 3 : 4;
    static constexpr int SMEM = S * STAGE;
    static constexpr int APER = A_BYTES / 1024 / 8, BPER = B_BYTES / 1024 / 8;   // wave copies per plane
    static constexpr int PER = 2 * (APER + BPER);                               // glds per thread per stage
    static constexpr int WMW = BM / 64, WNW = 8 / WMW;                          // wave grid
    static constexpr int TM = 2, TN = BN / WNW / 32;
    static_assert(APER >= 1 && BPER >= 1 && TN >= 1, "x3 tile");
    static_assert(SMEM >= BM * BN * 4 && SMEM <= 160 * 1024, "x3 LDS");
};

template <int BM, int AMODE>
__global__ __launch_bounds__(512) void gemm_x3_kernel(cmt_gemm_args a, int tiles_m, int tiles_n) {
    typedef X3Tile<BM, AMODE> T;
    typedef pair8_t frag;
    constexpr int BN = T::BN, KS = T::KS, S = T::S, TM = T::TM, TN = T::TN, PER = T::PER;
    __shared__ __attribute__((aligned(16))) char smem[T::SMEM];
    int z, mt, nt;
    xcd_tile(tiles_m, tiles_n, a.batch, z, mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WNW, wn = wave % T::WNW;
    const int lr = lane & 31, lh = lane >> 5;

    const pair_t* Ab = (const pair_t*)a.A + (int64_t)z * a.a_bstride;
    const pair_t* Wb = (const pair_t*)a.W + (int64_t)z * a.w_bstride;
    // copy i of this wave: tile rows (8 i + wave) * 16 + lane / 4, 16-byte chunk lane & 3
    const int ch = lane & 3;
    const pair_t* asrc[T::APER];
    RowInfo ri[T::APER];
    int acs[T::APER];
#pragma unroll
    for (int i = 0; i < T::APER; ++i) {
        const int row = (8 * i + wave) * 16 + (lane >> 2);
        acs[i] = (ch ^ ((row >> 2) & 3)) * 8;
        const int m = m0 + row;
        ri[i] = make_row_info<AMODE>(a, m);
        asrc[i] = Ab + (int64_t)min(m, a.M - 1) * a.lda + acs[i];
    }
    const pair_t* bsrc[T::BPER];
#pragma unroll
    for (int i = 0; i < T::BPER; ++i) {
        const int row = (8 * i + wave) * 16 + (lane >> 2);
        bsrc[i] = Wb + (int64_t)(n0 + row) * a.ldw + (ch ^ ((row >> 2) & 3)) * 8;
    }
    const int tapw = AMODE == CMT_A_CONV3X3 ? a.conv_c : (AMODE == CMT_A_CONV1D3 ? a.K / 3 : a.K);
    const int a_lo = AMODE == CMT_A_ROWS ? a.K : tapw;     // element offset of an A row's lo half
    int ctap = -1, ccin = 0;
    int64_t toff[T::APER];
    auto issue = [&](int buf, int kt) {
        char* sb = smem + buf * T::STAGE;
        int ka, kw;
        if constexpr (AMODE != CMT_A_ROWS) {
            // a tap spans tapw / 32 stages: gathered row offsets once per tap
            if (ctap < 0) {
                const int k0 = kt * KS;
                ctap = k0 / tapw;
                ccin = k0 - ctap * tapw;
#pragma unroll
                for (int i = 0; i < T::APER; ++i)
                    toff[i] = a_offset<AMODE>(a, ri[i], m0 + (8 * i + wave) * 16 + (lane >> 2), ctap * tapw);
            } else if ((ccin += KS) == tapw) {
                ccin = 0;
                ++ctap;
#pragma unroll
                for (int i = 0; i < T::APER; ++i)
                    toff[i] = a_offset<AMODE>(a, ri[i], m0 + (8 * i + wave) * 16 + (lane >> 2), ctap * tapw);
            }
            ka = ccin;
            kw = ctap * tapw + ccin;
        } else {
            ka = kw = kt * KS;
        }
#pragma unroll
        for (int i = 0; i < T::APER; ++i) {
            const pair_t* src;
            if (AMODE == CMT_A_ROWS) src = asrc[i] + ka;
            else src = toff[i] < 0 ? nullptr : Ab + toff[i] + ka + acs[i];
            glds16(src ? (const void*)src : (const void*)g_zero_page, sb + (8 * i + wave) * 1024);
            glds16(src ? (const void*)(src + a_lo) : (const void*)g_zero_page, sb + T::A_BYTES + (8 * i + wave) * 1024);
        }
#pragma unroll
        for (int i = 0; i < T::BPER; ++i) {
            glds16(bsrc[i] + kw, sb + 2 * T::A_BYTES + (8 * i + wave) * 1024);
            glds16(bsrc[i] + kw + a.K, sb + 2 * T::A_BYTES + T::B_BYTES + (8 * i + wave) * 1024);
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = a.K / KS;
#pragma unroll
    for (int st = 0; st < S; ++st)
        if (st < nk) issue(st, st);
    for (int kt = 0; kt < nk; ++kt) {
        const int last = min(nk - 1, kt == 0 ? S - 1 : kt + S - 2);
        wait_tiles<PER, S>(last - kt);
        barrier_mem();
        // every wave is past its reads of stage kt-1: refill that slot
        if (kt >= 1 && kt + S - 1 < nk) issue((kt - 1) % S, kt + S - 1);
        const char* As = smem + (kt % S) * T::STAGE;
        const char* Bs = As + 2 * T::A_BYTES;
#pragma unroll
        for (int ks = 0; ks < KS / 16; ++ks) {
            const int kc = 2 * ks + lh;
            frag af[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int r = wm * 64 + tm * 32 + lr;
                const int o = r * T::ROWB + ((kc ^ ((r >> 2) & 3)) << 4);
                af[tm] = *(const frag*)(As + o);
                al[tm] = *(const frag*)(As + T::A_BYTES + o);
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int r = wn * (BN / T::WNW) + tn * 32 + lr;
                const int o = r * T::ROWB + ((kc ^ ((r >> 2) & 3)) << 4);
                bh[tn] = *(const frag*)(Bs + o);
                bl[tn] = *(const frag*)(Bs + T::B_BYTES + o);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<pair_t>::mma(bh[tn], al[tm], acc[tm][tn]);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<pair_t>::mma(bl[tn], af[tm], acc[tm][tn]);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_traits<pair_t>::mma(bh[tn], af[tm], acc[tm][tn]);
        }
    }

    x3_epilogue<BM, TM, TN, T::WNW, T::NTX>(a, acc, smem, m0, n0, z, wm, wn);
}

template <int BM>
int launch_x3(const cmt_gemm_args& a, hipStream_t s) {
    const int tm = cdiv(a.M, BM), tn = a.N / 128;
    const unsigned nwg = (unsigned)((int64_t)tm * tn * a.batch);
    if (a.a_mode == CMT_A_CONV3X3) gemm_x3_kernel<BM, CMT_A_CONV3X3><<<nwg, 512, 0, s>>>(a, tm, tn);
    else gemm_x3_kernel<BM, CMT_A_ROWS><<<nwg, 512, 0, s>>>(a, tm, tn);
    return cmt_check_launch("cmt_gemm");
}

// ---------------------------------------------------------------------------
// shared_conv at the reference's numerics, straight from the NCHW fp32 map
// (CMT_A_CONV3X3_NCHW, W CMT_F16P; cmt_head.py:280-287, 481).
//
// The 3x3 implicit GEMM re-stages every input pixel once per tap when the A
// tile is gathered per (tap, channel chunk) (gemm_x3_kernel<CONV3X3>: 9 x 32 KB
// of A per 32 channels of a 256-pixel tile).  Here a tile of BM = 256
// consecutive pixels of one image reads, per chunk of 16 input channels, the
// pixel HALO it needs for all nine taps -- pixels p0 - W - 1 .. p0 + 256 + W,
// zero outside the image -- from the NCHW map (each channel's run is
// contiguous: one coalesced scalar load per channel and lane), splits it into
// f16 hi / lo in registers and writes it to LDS once as 64-byte pixel rows (hi
// 16 | lo 16, 16-byte chunks XOR-swizzled by hsw(row)).  The nine taps'
// A fragments are then ds_reads of that halo at a per-tap row shift (W x dy +
// dx); a lane whose pixel sits on the left / right image edge zeroes its
// fragment for dx = -1 / +1 (the row-wrapped neighbour is padding).  W is
// staged per (chunk, kernel row) -- 3 taps x 128 rows x 64 bytes -- through an
// S-slot LDS-DMA ring (one barrier per three taps).  Per 16 channels the LDS
// fill is ~40 KB halo + 72 KB W against
// 9 x 24 KB, and the NCHW -> pair-rows layout pass disappears.
//
// The halo loads of chunk c + 1 go out at tap 0 of chunk c (after that step's
// W issue) into registers and are converted after tap 8; vmcnt completes in
// issue order, so each W wait counts the halo loads issued after it (the
// compiler's own wait for the halo registers trails 8 W stages).
// 8 waves in a 4 x 2 grid of 64 x 64 sub-tiles, the three products per tap in
// gemm_x3_kernel's order; epilogue x3_epilogue (bias, ReLU, pair / fp32 rows).
// ---------------------------------------------------------------------------
struct HaloConv {
    static constexpr int BM = 256, BN = 128, CK = 16, NTX = 512;
    static constexpr int WMAX = 180;                          // widest map row supported (the 0.075 m BEV grid)
    static constexpr int NHMAX = BM + 2 * WMAX + 2;           // halo pixels per tile
    static constexpr int ROWB = 64;                           // hi 16 | lo 16 f16 per row
    static constexpr int HALO = (NHMAX * ROWB + 1023) / 1024 * 1024;
    static constexpr int WTAP = BN * ROWB;                    // one (chunk, tap) of W: 8 KB
    static constexpr int WSLOT = 3 * WTAP;                    // one step = one kernel row (3 taps)
    static constexpr int S = 3;                               // W ring slots
    static constexpr int SMEM = 2 * HALO + S * WSLOT;
    static constexpr int UPT = (2 * NHMAX + 15 + NTX - 1) / NTX;   // (pixel, channel octet) units per thread
    static constexpr int WNW = 2, TM = 2, TN = 2;
    static_assert(SMEM <= 160 * 1024 && SMEM >= BM * BN * 4, "halo conv LDS");
    static_assert(WTAP == NTX * 16, "one 16-byte DMA per thread per tap of a W slot");
};

// halo row swizzle of conv_halo_x3_kernel (see its unit setup)
__device__ __forceinline__ int hsw(int h) { return ((h >> 2) + 2 * ((h >> 1) & 1)) & 3; }

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// VAR bits: 1 = the younger half of the workgroup (waves 4-7) at priority 1 for the whole loop
// (cdna_hip_programming.md T5, static form); 2 = s_setprio(1) around every tap's MFMA cluster;
// 16 = the halo loads as inline asm, waited for by a counted vmcnt of our own: hipcc's own wait
// for a VGPR-destination load beside the W ring's LDS-DMA is vmcnt(0) (cdna_hip_programming.md
// 'Three .s-level traps' (b)), which drained the W ring at the end of every chunk;
// 4 / 8 = diagnostics only (no halo loads / no W refills: wrong results, for timing those streams).
// X3 = false (round 6): one MFMA pass in the compute dtype E (f16 / bf16: the 'fp16' / 'bf16' policies'
// shared_conv, W [N][K] in E) on the same halo / W layouts -- the lo halves are neither stored nor read
template <int VAR, typename E = pair_t, bool X3 = true>
__global__ __launch_bounds__(512) void conv_halo_x3_kernel(cmt_gemm_args a, int tiles_m, int tiles_n) {
    typedef HaloConv T;
    typedef typename mfma_traits<E>::frag frag;
    constexpr bool AH = (VAR & 16) != 0;
    constexpr int BM = T::BM, S = T::S, TM = T::TM, TN = T::TN, UPT = T::UPT;
    constexpr int HLOADS = UPT * 8;                           // halo loads per thread per chunk
    __shared__ __attribute__((aligned(16))) char smem[T::SMEM];
    int z, mt, nt;
    xcd_tile(tiles_m, tiles_n, a.batch, z, mt, nt);
    const int m0 = mt * BM, n0 = nt * T::BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / T::WNW, wn = wave % T::WNW;
    const int lr = lane & 31, lh = lane >> 5;
    const int Wd = a.conv_w, HW = a.conv_h * a.conv_w, Cin = a.conv_c;
    const int NH = BM + 2 * Wd + 2;                           // halo pixels of this launch
    const int hs = m0 - Wd - 1;                               // image pixel of halo row 0
    const float* X = (const float*)a.A + (int64_t)z * a.a_bstride;
    const pair_t* Wb = (const pair_t*)a.W;

    // halo units of this thread: (halo row h, channel octet o); lanes walk consecutive rows (coalesced
    // loads), octet 1's rows start at a 16-aligned unit.  Halo row h's 16-byte chunks are XOR-swizzled
    // by hsw(h) = ((h >> 2) + 2 ((h >> 1) & 1)) & 3: every 8-lane group of a ds_write_b128 (banks mod 32,
    // two 64-byte rows per bank row) then stores 8 aligned consecutive rows on 8 distinct slots, and the
    // 16-lane groups of the tap-shifted ds_read_b128 stay conflict-free at any shift.  (The former
    // (h >> 2) & 3 put rows h and h + 2 on one slot: 2-way on every halo store, ~2.5 M extra LDS
    // cycles per launch, profiles/r5b_convh_pmc_summary.json; permuting the lanes instead cost more
    // in the halo loads than it saved, r6b.)
    const int NHA = (NH + 15) & ~15;
    int u_src[UPT], u_lds[UPT];
    bool u_ok[UPT], u_on[UPT];
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        const int u = tid + i * T::NTX;
        const int o = u >= NHA ? 1 : 0;
        const int h = u - o * NHA;
        const int p = hs + h;
        u_on[i] = h < NH && u < NHA + NH;                     // a unit of this tile at all
        u_ok[i] = u_on[i] && p >= 0 && p < HW;                // inside the image (else zeros)
        u_src[i] = 8 * o * HW + p;
        u_lds[i] = h * T::ROWB + ((o ^ hsw(h)) << 4);         // hi chunk; the lo chunk is (2 + o) ^ hsw
    }
    float hv[UPT][8];
    auto load_halo = [&](int c) {
        const float* Xc = X + (int64_t)c * T::CK * HW;
#pragma unroll
        for (int i = 0; i < UPT; ++i) {
            // every wave issues all HLOADS loads (the vmcnt waits count them), with no
            // condition on the loaded value (a select would wait for it): padding units
            // read the zero page
            const float* src = u_ok[i] ? Xc + u_src[i] : (const float*)g_zero_page;
            const int es = u_ok[i] ? HW : 0;
            if constexpr (VAR & 4) {
#pragma unroll
                for (int e = 0; e < 8; ++e) hv[i][e] = (float)(es + e) * 1e-3f;
            } else if constexpr (AH) {
                // SGPR base (the chunk's channel block) + a 32-bit VGPR byte offset per load;
                // padding units load pixel 0 of the channel and are zeroed after the wait
                uint32_t vo = (uint32_t)(u_ok[i] ? u_src[i] : 0) * 4u;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    asm volatile("global_load_dword %0, %1, %2" : "=v"(hv[i][e]) : "v"(vo), "s"(Xc) : "memory");
                    vo += (uint32_t)HW * 4u;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) hv[i][e] = src[e * es];
            }
        }
    };
    auto store_halo = [&](int buf, auto first) {
        char* hb = smem + buf * T::HALO;
        if constexpr (AH && !(VAR & 4)) {
            // the halo loads went out at the chunk's first step; two W stages (3 DMAs each) since
            // (none before chunk 0's, in the prologue): wait for the loads, naming every
            // destination so nothing reads them before
            asm volatile("s_waitcnt vmcnt(%24)"
                         : "+v"(hv[0][0]), "+v"(hv[0][1]), "+v"(hv[0][2]), "+v"(hv[0][3]), "+v"(hv[0][4]),
                           "+v"(hv[0][5]), "+v"(hv[0][6]), "+v"(hv[0][7]), "+v"(hv[1][0]), "+v"(hv[1][1]),
                           "+v"(hv[1][2]), "+v"(hv[1][3]), "+v"(hv[1][4]), "+v"(hv[1][5]), "+v"(hv[1][6]),
                           "+v"(hv[1][7]), "+v"(hv[2][0]), "+v"(hv[2][1]), "+v"(hv[2][2]), "+v"(hv[2][3]),
                           "+v"(hv[2][4]), "+v"(hv[2][5]), "+v"(hv[2][6]), "+v"(hv[2][7])
                         : "n"(decltype(first)::value ? 0 : 6)
                         : "memory");
            static_assert(!AH || UPT == 3, "the wait statement names three units");
        } else {
            // pin the halo registers here: without this the split arithmetic below (no memory
            // dependence) is hoisted right behind the loads and waits for them there
#pragma unroll
            for (int i = 0; i < UPT; ++i)
                asm volatile("" : "+v"(hv[i][0]), "+v"(hv[i][1]), "+v"(hv[i][2]), "+v"(hv[i][3]), "+v"(hv[i][4]),
                             "+v"(hv[i][5]), "+v"(hv[i][6]), "+v"(hv[i][7]));
        }
#pragma unroll
        for (int i = 0; i < UPT; ++i) {
            if (!u_on[i]) continue;
            frag hi;
            pair8_t lo;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = AH && !u_ok[i] ? 0.f : hv[i][e];
                hi[e] = (E)x;
                if constexpr (X3) lo[e] = (pair_t)(x - (float)hi[e]);
            }
            *(frag*)(hb + u_lds[i]) = hi;
            if constexpr (X3) *(pair8_t*)(hb + (u_lds[i] ^ (2 << 4))) = lo;   // (2 + o) ^ sw == (o ^ sw) ^ 2
        }
    };

    // W slot fill: LDS byte tid * 16 of the slot = row tid / 4, physical chunk tid % 4
    const int wrow = tid >> 2, wlc = (tid & 3) ^ ((wrow >> 2) & 3);
    // (one pass: the lo chunks of a slot row take the hi channels again -- never read)
    const pair_t* wsrc = Wb + (int64_t)(n0 + wrow) * a.ldw + (X3 ? (wlc >> 1) * a.K : 0) + (wlc & 1) * 8;
    const int nchunks = Cin / T::CK, G = nchunks * 3;
    auto issue_w = [&](int g) {   // step g = (chunk g / 3, kernel row g % 3): its three taps
        const int c = g / 3, dy = g - 3 * (g / 3);
        char* slot = smem + 2 * T::HALO + (g % S) * T::WSLOT + wave * 1024;
        if constexpr (VAR & 8) {
            if (g >= S) return;
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) glds16(wsrc + (3 * dy + dx) * Cin + c * T::CK, slot + dx * T::WTAP);
    };

    // per-lane fragment geometry: tile rows of the two 32-row sub-tiles, their edge flags
    int arow[TM];
    bool edl[TM], edr[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        arow[tm] = wm * 64 + tm * 32 + lr;
        const int x = (m0 + arow[tm]) % Wd;
        edl[tm] = x == 0;
        edr[tm] = x == Wd - 1;
    }
    int woff[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        const int r = wn * 64 + tn * 32 + lr;
        woff[tn] = r * T::ROWB + ((lh ^ ((r >> 2) & 3)) << 4);
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // prologue: chunk 0's halo, W of steps 0 .. S-1
    load_halo(0);
    store_halo(0, std::true_type{});
#pragma unroll
    for (int g = 0; g < S; ++g) issue_w(g);

    // Every step (one kernel row: three taps) issues exactly one W stage (past the last step:
    // a dummy refill of a slot no later step reads) and the first step of every chunk the next
    // chunk's halo loads (the last chunk: its own again, converted into the idle buffer), so
    // the issue stream is the same for every chunk and each wait below counts the ops issued
    // after W(g) exactly.
    constexpr int WOPS = 3;                                   // DMAs per thread per W stage
    if constexpr (VAR & 1)
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
    for (int c = 0; c < nchunks; ++c) {
        const char* Hs = smem + (c & 1) * T::HALO;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int g = 3 * c + dy;
            // VMEM ops issued after W(g): S - 2 later stages (S - 1 at step 0), plus the halo
            // loads of the chunk's first step for its second and third
            if (dy >= 1) vm_wait<(S - 2) * WOPS + HLOADS>();
            else if (c == 0) vm_wait<(S - 1) * WOPS>();
            else vm_wait<(S - 2) * WOPS>();
            barrier_mem();
            if (g >= 1) issue_w(g + S - 1 < G ? g + S - 1 : g - 1);
            if (dy == 0) load_halo(c + 1 < nchunks ? c + 1 : c);

            const char* Ws = smem + 2 * T::HALO + (g % S) * T::WSLOT;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const int tsh = dy * Wd + dx;                 // halo row of (pixel, tap) - tile row
                frag af[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    const int hr = arow[tm] + tsh;
                    const int base = hr * T::ROWB, sw = hsw(hr);
                    af[tm] = *(const frag*)(Hs + base + ((lh ^ sw) << 4));
                    if constexpr (X3) al[tm] = *(const frag*)(Hs + base + (((2 + lh) ^ sw) << 4));
                    if ((dx == 0 && edl[tm]) || (dx == 2 && edr[tm])) {
                        af[tm] = frag{};
                        if constexpr (X3) al[tm] = frag{};
                    }
                }
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    bh[tn] = *(const frag*)(Ws + dx * T::WTAP + woff[tn]);
                    if constexpr (X3) bl[tn] = *(const frag*)(Ws + dx * T::WTAP + (woff[tn] ^ (2 << 4)));
                }
                if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(1);
                if constexpr (X3) {
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn)
                            acc[tm][tn] = mfma_traits<E>::mma(bh[tn], al[tm], acc[tm][tn]);
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn)
                            acc[tm][tn] = mfma_traits<E>::mma(bl[tn], af[tm], acc[tm][tn]);
                }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[tm][tn] = mfma_traits<E>::mma(bh[tn], af[tm], acc[tm][tn]);
                if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(0);
            }
        }
        // chunk c + 1's halo into the other buffer (its last readers, chunk c - 1's taps, are
        // all past this chunk's first barrier); the next step's barrier publishes it
        store_halo((c + 1) & 1, std::false_type{});
    }
    // the dummy W refills and the last halo loads are still in flight: drain them before
    // the epilogue reuses the LDS
    vm_wait<0>();
    x3_epilogue<BM, TM, TN, T::WNW, T::NTX>(a, acc, smem, m0, n0, z, wm, wn);
}

int launch_conv_halo(const cmt_gemm_args& a, hipStream_t s) {
    const int tm = cdiv(a.conv_h * a.conv_w, HaloConv::BM), tn = a.N / HaloConv::BN;
    const unsigned nwg = (unsigned)((int64_t)tm * tn * a.batch);
    if (a.w_dtype == CMT_F16P) conv_halo_x3_kernel<CMT_CONV_VAR><<<nwg, HaloConv::NTX, 0, s>>>(a, tm, tn);
    else if (a.w_dtype == CMT_F16) conv_halo_x3_kernel<0, f16_t, false><<<nwg, HaloConv::NTX, 0, s>>>(a, tm, tn);
    else conv_halo_x3_kernel<0, bf16_t, false><<<nwg, HaloConv::NTX, 0, s>>>(a, tm, tn);
    return cmt_check_launch("cmt_gemm");
}

// ---------------------------------------------------------------------------
// GEMM + residual + LayerNorm, fused (cmt_gemm_ln).  One workgroup owns 32
// full output rows (BN = N = 256): waves 1 x 4, each wave 32 rows x 64
// columns.  The epilogue adds bias and R, reduces each row's mean / variance
// across the two lane halves (permlane32_swap) and the 4 waves (a slot after
// the staging ring in the same LDS array), then writes what cmt_layernorm_ex
// would: Y, lowp(y), lowp(y + P) and the second LN (post_norm) Y2.
// ---------------------------------------------------------------------------
template <typename CT, int S, bool X3 = false>
__global__ __launch_bounds__(NT) void gemm_ln_kernel(cmt_gemm_args a, cmt_ln_args ln) {
    typedef DmaTile<CT, 32, 256, S, CMT_A_ROWS, 1, X3> Tile;
    static_assert(Tile::TM == 1 && Tile::TN == 2, "32 x 256 tile, 1 x 4 waves");
    __shared__ __attribute__((aligned(16))) char smem[Tile::SMEM + 2 * 4 * 32 * 4];
    float* red = (float*)(smem + Tile::SMEM);       // [2][4 waves][32 rows]
    const int m0 = blockIdx.x * 32;
    f32x16 acc[1][2];
    Tile::run(a, smem, m0, 0, 0, acc);

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int lr = lane & 31;
    const int lh = lane >> 5;
    const int m = m0 + lr;
    const int mc = min(m, a.M - 1);
    constexpr int C = 256;
    // column of value group t = (tn, g): wave*64 + tn*32 + 8g + 4lh -> 8 groups of 4 per lane
    auto col = [&](int t) { return wave * 64 + (t >> 2) * 32 + 8 * (t & 3) + 4 * lh; };

    // ---- every load first (vmcnt counts stores too)
    f32x4 v[8], bw[8], bb[8], pv[8], yo[8], w2[8], b2[8], y2o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int n = col(t);
        v[t] = f32x4{acc[0][t >> 2][4 * (t & 3)], acc[0][t >> 2][4 * (t & 3) + 1], acc[0][t >> 2][4 * (t & 3) + 2],
                     acc[0][t >> 2][4 * (t & 3) + 3]};
        if (a.bias) v[t] += *(const f32x4*)(a.bias + n);
        if (a.R) v[t] += load4(a.R, (int64_t)mc * a.ldr + n, a.r_dtype);
        bw[t] = *(const f32x4*)(ln.W + n);
        bb[t] = *(const f32x4*)(ln.B + n);
        if (ln.Yp) pv[t] = *(const f32x4*)(ln.P + (int64_t)mc * ln.ldp + n);
        if (ln.Y && (ln.flags & CMT_LN_MAX_INTO)) yo[t] = *(const f32x4*)(ln.Y + (int64_t)mc * ln.ldy + n);
        if (ln.Y2) {
            w2[t] = *(const f32x4*)(ln.W2 + n);
            b2[t] = *(const f32x4*)(ln.B2 + n);
            if (ln.flags2 & CMT_LN_MAX_INTO) y2o[t] = *(const f32x4*)(ln.Y2 + (int64_t)mc * ln.ldy2 + n);
        }
    }
    // row reduction: 32 values per lane -> lane pair -> 4 waves
    auto row_sum = [&](float x, int slot) {
        x = pair_sum(x);
        if (lh == 0) red[(slot * 4 + wave) * 32 + lr] = x;
        barrier_mem();
        return red[(slot * 4 + 0) * 32 + lr] + red[(slot * 4 + 1) * 32 + lr] + red[(slot * 4 + 2) * 32 + lr] +
               red[(slot * 4 + 3) * 32 + lr];
    };
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) sum += v[t][0] + v[t][1] + v[t][2] + v[t][3];
    const float mean = row_sum(sum, 0) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float d = v[t][j] - mean;
            ss += d * d;
        }
    const float rstd = rsqrtf(row_sum(ss, 1) / (float)C + ln.eps);
    f32x4 y[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) y[t][j] = (v[t][j] - mean) * rstd * bw[t][j] + bb[t][j];
    // second LN (post_norm) statistics on the first LN's raw output
    f32x4 y2[8];
    if (ln.Y2) {
        barrier_mem();   // slots reused
        float s2 = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) s2 += y[t][0] + y[t][1] + y[t][2] + y[t][3];
        const float mean2 = row_sum(s2, 0) / (float)C;
        float q2 = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float d = y[t][j] - mean2;
                q2 += d * d;
            }
        const float rstd2 = rsqrtf(row_sum(q2, 1) / (float)C + ln.eps);
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float o = (y[t][j] - mean2) * rstd2 * w2[t][j] + b2[t][j];
                if (ln.flags2 & CMT_LN_NAN_TO_NUM) o = nan_to_num(o);
                if (ln.flags2 & CMT_LN_MAX_INTO) o = fmaxf(o, y2o[t][j]);
                y2[t][j] = o;
            }
    }
    if (m >= a.M) return;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int n = col(t);
        f32x4 o = y[t];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (ln.flags & CMT_LN_NAN_TO_NUM) o[j] = nan_to_num(o[j]);
            if (ln.flags & CMT_LN_MAX_INTO) o[j] = fmaxf(o[j], yo[t][j]);
        }
        if (ln.Y) *(f32x4*)(ln.Y + (int64_t)m * ln.ldy + n) = o;
        if constexpr (X3) {   // CMT_F16P rows: hi at n, lo at C + n
            if (ln.Yl) store_pair4((pair_t*)ln.Yl + (int64_t)m * ln.ldyl, C, n, o);
            if (ln.Yp) store_pair4((pair_t*)ln.Yp + (int64_t)m * ln.ldyp, C, n, o + pv[t]);
        } else {
            if (ln.Yl) store4<CT>(ln.Yl, (int64_t)m * ln.ldyl + n, ln.lowp_dtype, o);
            if (ln.Yp) store4<CT>(ln.Yp, (int64_t)m * ln.ldyp + n, ln.lowp_dtype, o + pv[t]);
        }
        if (ln.Y2) *(f32x4*)(ln.Y2 + (int64_t)m * ln.ldy2 + n) = y2[t];
    }
}

template <int BM, int BN, int S, int AMODE>
int launch_dma_mode(const cmt_gemm_args& a, hipStream_t s) {
    const int tm = cdiv(a.M, BM), tn = a.N / BN;
    const int64_t nwg = (int64_t)tm * tn * a.batch * (a.k_splits > 1 ? a.k_splits : 1);
    // the pair stages carry four tiles: 128 x 128 keeps 2 of them (128 KB), the others 3 or 2
    constexpr int SP = BM * BN >= 128 * 128 ? 2 : (BM * BN >= 128 * 64 ? 2 : 3);
    if (a.w_dtype == CMT_F16P) gemm_dma_kernel<pair_t, BM, BN, SP, AMODE, true><<<(unsigned)nwg, NT, 0, s>>>(a, tm, tn);
    else if (a.w_dtype == CMT_BF16) gemm_dma_kernel<bf16_t, BM, BN, S, AMODE><<<(unsigned)nwg, NT, 0, s>>>(a, tm, tn);
    else gemm_dma_kernel<f16_t, BM, BN, S, AMODE><<<(unsigned)nwg, NT, 0, s>>>(a, tm, tn);
    return cmt_check_launch("cmt_gemm");
}

template <int BM, int BN, int S>
int launch_dma(const cmt_gemm_args& a, hipStream_t s) {
    switch (a.a_mode) {
        case CMT_A_ROWS: return launch_dma_mode<BM, BN, S, CMT_A_ROWS>(a, s);
        case CMT_A_CONV3X3: return launch_dma_mode<BM, BN, S, CMT_A_CONV3X3>(a, s);
        default: return launch_dma_mode<BM, BN, S, CMT_A_CONV1D3>(a, s);
    }
}

template <int BM, int BN, int LBK, int AMODE>
void launch_lowp(const cmt_gemm_args& a, dim3 grid, hipStream_t s) {
    if constexpr (AMODE == CMT_A_CONV3X3) {
        // the conv gather reads NHWC rows already in the compute dtype
        if (a.w_dtype == CMT_BF16) gemm_lowp_kernel<bf16_t, BM, BN, LBK, AMODE, false><<<grid, NT, 0, s>>>(a);
        else gemm_lowp_kernel<f16_t, BM, BN, LBK, AMODE, false><<<grid, NT, 0, s>>>(a);
    } else {
        if (a.w_dtype == CMT_BF16) {
            if (a.a_dtype == CMT_F32) gemm_lowp_kernel<bf16_t, BM, BN, LBK, AMODE, true><<<grid, NT, 0, s>>>(a);
            else gemm_lowp_kernel<bf16_t, BM, BN, LBK, AMODE, false><<<grid, NT, 0, s>>>(a);
        } else {
            if (a.a_dtype == CMT_F32) gemm_lowp_kernel<f16_t, BM, BN, LBK, AMODE, true><<<grid, NT, 0, s>>>(a);
            else gemm_lowp_kernel<f16_t, BM, BN, LBK, AMODE, false><<<grid, NT, 0, s>>>(a);
        }
    }
}

template <int BM, int BN, int AMODE>
int launch_mode(const cmt_gemm_args& a, hipStream_t s) {
    dim3 grid(a.N / BN, cdiv(a.M, BM), a.batch);
    if (a.w_dtype == CMT_F32) {
        gemm_f32_kernel<BM, BN, AMODE><<<grid, NT, 0, s>>>(a);
    } else {
        // deepest K step that divides K (and, for the gathered modes, the per-tap channel count)
        const int kdiv = AMODE == CMT_A_CONV3X3 ? a.conv_c : (AMODE == CMT_A_CONV1D3 ? a.K / 3 : a.K);
        if (BM == 64 && kdiv % 128 == 0) launch_lowp<BM, BN, 128, AMODE>(a, grid, s);
        else if (kdiv % 64 == 0) launch_lowp<BM, BN, 64, AMODE>(a, grid, s);
        else launch_lowp<BM, BN, 32, AMODE>(a, grid, s);
    }
    return cmt_check_launch("cmt_gemm");
}

template <int BM, int BN>
int launch_tiles(const cmt_gemm_args& a, hipStream_t s) {
    switch (a.a_mode) {
        case CMT_A_ROWS: return launch_mode<BM, BN, CMT_A_ROWS>(a, s);
        case CMT_A_CONV3X3: return launch_mode<BM, BN, CMT_A_CONV3X3>(a, s);
        default: return launch_mode<BM, BN, CMT_A_CONV1D3>(a, s);
    }
}

}  // namespace

extern "C" int cmt_gemm_ln(const cmt_gemm_args* gp, const cmt_ln_args* lp, void* stream) {
    CMT_REQUIRE(gp != nullptr && lp != nullptr, "cmt_gemm_ln: null args");
    const cmt_gemm_args& a = *gp;
    const cmt_ln_args& l = *lp;
    CMT_REQUIRE(a.M > 0 && a.N == 256 && l.C == 256 && a.K % 64 == 0 && a.batch == 1,
                "cmt_gemm_ln: needs N == C == 256, K % 64 == 0, batch 1");
    CMT_REQUIRE(a.A && a.W && (a.w_dtype == CMT_F16 || a.w_dtype == CMT_BF16 || a.w_dtype == CMT_F16P) &&
                    a.a_dtype == a.w_dtype, "cmt_gemm_ln: A and W in the f16/bf16 compute dtype or both CMT_F16P");
    CMT_REQUIRE(a.w_dtype != CMT_F16P || a.R == nullptr || a.r_dtype == CMT_F32, "cmt_gemm_ln: split R must be fp32");
    CMT_REQUIRE(a.a_mode == CMT_A_ROWS && a.A2 == nullptr && a.c_mode == CMT_C_ROWS && !a.relu,
                "cmt_gemm_ln: plain row GEMM (no A2, no head split, no relu)");
    CMT_REQUIRE(a.lda % 8 == 0 && a.ldw % 8 == 0 && (a.R == nullptr || a.ldr % 4 == 0) &&
                (a.r_dtype == CMT_F32 || a.r_dtype == a.w_dtype), "cmt_gemm_ln: bad A/W/R strides or R dtype");
    CMT_REQUIRE(l.W && l.B && (l.Y || l.Yl || l.Yp || l.Y2) && (l.Yp == nullptr || l.P) &&
                (l.Y2 == nullptr || (l.W2 && l.B2)), "cmt_gemm_ln: bad LN outputs");
    CMT_REQUIRE((l.Yl == nullptr && l.Yp == nullptr) || l.lowp_dtype == a.w_dtype,
                "cmt_gemm_ln: lowp outputs must use the compute dtype");
    CMT_REQUIRE(l.ldy % 4 == 0 && l.ldyl % 4 == 0 && l.ldyp % 4 == 0 && l.ldp % 4 == 0 && l.ldy2 % 4 == 0,
                "cmt_gemm_ln: LN strides must be multiples of 4");
    hipStream_t s = (hipStream_t)stream;
    const unsigned grid = (unsigned)cdiv(a.M, 32);
    // split pairs: four tiles per stage (A_hi, A_lo, W_hi, W_lo: 72 KB), 2 stages
    if (a.w_dtype == CMT_F16P) gemm_ln_kernel<pair_t, 2, true><<<grid, NT, 0, s>>>(a, l);
    else if (a.w_dtype == CMT_BF16) gemm_ln_kernel<bf16_t, 3><<<grid, NT, 0, s>>>(a, l);
    else gemm_ln_kernel<f16_t, 3><<<grid, NT, 0, s>>>(a, l);
    return cmt_check_launch("cmt_gemm_ln");
}

// the row-mode / 3x3-conv split GEMMs gemm_x3_kernel covers
static bool x3_eligible(const cmt_gemm_args& a) {
    const int kdiv = a.a_mode == CMT_A_CONV3X3 ? a.conv_c : a.K;
    return (a.a_mode == CMT_A_ROWS || a.a_mode == CMT_A_CONV3X3) && a.A2 == nullptr && a.c_mode == CMT_C_ROWS &&
           a.k_splits <= 1 && a.plane_max2 == nullptr && a.N % 128 == 0 && kdiv % 32 == 0 && a.K % 32 == 0;
}

extern "C" int cmt_gemm(const cmt_gemm_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_gemm: null args");
    const cmt_gemm_args& a = *ap;
    CMT_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.batch > 0, "cmt_gemm: empty problem");
    CMT_REQUIRE(a.N % 64 == 0, "cmt_gemm: N must be a multiple of 64");
    CMT_REQUIRE(a.A && a.W && a.C, "cmt_gemm: null A/W/C");
    if (a.a_mode == CMT_A_CONV3X3_NCHW) {
        CMT_REQUIRE(a.a_dtype == CMT_F32 &&
                        ((a.w_dtype == CMT_F16P && (a.c_dtype == CMT_F16P || a.c_dtype == CMT_F32)) ||
                         ((a.w_dtype == CMT_F16 || a.w_dtype == CMT_BF16) &&
                          (a.c_dtype == a.w_dtype || a.c_dtype == CMT_F32))) &&
                        a.c_mode == CMT_C_ROWS && a.k_splits <= 1 && a.plane_max2 == nullptr,
                    "cmt_gemm: the NCHW conv3x3 takes fp32 A and CMT_F16P W (fp32 / CMT_F16P row C) or f16 / "
                    "bf16 W (one pass; fp32 or W-dtype row C), no split-K / plane_max2");
        CMT_REQUIRE(a.A2 == nullptr || (a.lda2 % 4 == 0 && ((uintptr_t)a.A2 & 15) == 0),
                    "cmt_gemm: NCHW conv3x3 second-output rows A2: fp32, lda2 % 4 == 0, 16-byte aligned");
        CMT_REQUIRE(a.conv_c % 16 == 0 && a.K == 9 * a.conv_c && a.conv_h > 0 && a.conv_w > 0 &&
                        a.conv_w <= HaloConv::WMAX && a.M == a.conv_h * a.conv_w && a.N % 128 == 0,
                    "cmt_gemm: bad NCHW conv3x3 geometry (C_in % 16, K = 9 C_in, width <= 180, M = h * w, "
                    "N % 128)");
        CMT_REQUIRE(a.ldw % 8 == 0 && a.ldc % 8 == 0 && (a.R == nullptr || a.ldr % 4 == 0) && a.bias_bstride % 4 == 0 &&
                        a.r_dtype != CMT_F16P,
                    "cmt_gemm: NCHW conv3x3 strides (ldw, ldc % 8; ldr, bias_bstride % 4; fp32 / f16 R)");
        return launch_conv_halo(a, (hipStream_t)stream);
    }
    CMT_REQUIRE(a.K % BK == 0, "cmt_gemm: K must be a multiple of 32");
    CMT_REQUIRE(a.w_dtype == CMT_F32 || a.w_dtype == CMT_F16 || a.w_dtype == CMT_BF16 || a.w_dtype == CMT_F16P,
                "cmt_gemm: bad w_dtype");
    CMT_REQUIRE(a.w_dtype != CMT_F16P || a.a_dtype == CMT_F16P, "cmt_gemm: split (CMT_F16P) W needs CMT_F16P A");
    CMT_REQUIRE(a.k_splits <= 1 ||
                    (a.w_dtype != CMT_F32 && a.a_dtype == a.w_dtype && a.a_mode == CMT_A_ROWS &&
                     a.c_mode == CMT_C_ROWS && a.c_dtype == CMT_F32 && a.batch == 1 && !a.relu &&
                     a.plane_max2 == nullptr && a.k_splits <= 64 && (a.K / 64) % a.k_splits == 0 &&
                     a.c_split_stride >= (int64_t)(a.M - 1) * a.ldc + a.N),
                "cmt_gemm: split-K needs compute-dtype row A, fp32 row C, batch 1, no relu / plane_max2, "
                "K / 64 divisible by k_splits and non-overlapping parts");
    CMT_REQUIRE(a.a_dtype == CMT_F32 || a.a_dtype == a.w_dtype, "cmt_gemm: A must be f32 or the compute dtype");
    CMT_REQUIRE(a.a_mode != CMT_A_CONV3X3 || a.a_dtype == a.w_dtype,
                "cmt_gemm: the conv3x3 gather needs A in the compute dtype");
    CMT_REQUIRE(a.c_dtype == CMT_F32 || a.c_dtype == CMT_F16 || a.c_dtype == CMT_BF16 || a.c_dtype == CMT_F16P,
                "cmt_gemm: bad c_dtype");
    CMT_REQUIRE(a.lda % 8 == 0 && a.ldw % 8 == 0, "cmt_gemm: lda/ldw must be multiples of 8 elements");
    CMT_REQUIRE(a.r_dtype == CMT_F32 || a.r_dtype == a.w_dtype, "cmt_gemm: R must be f32 or the compute dtype");
    CMT_REQUIRE((a.c_dtype != CMT_F16P && a.r_dtype != CMT_F16P) || a.w_dtype == CMT_F16P,
                "cmt_gemm: CMT_F16P C / R belong to the split GEMM");
    CMT_REQUIRE(a.A2 == nullptr || (a.a_mode == CMT_A_ROWS && a.a2_cols % 128 == 0),
                "cmt_gemm: A2 needs row mode and 128-aligned a2_cols");
    CMT_REQUIRE(a.A2 == nullptr || a.a2_mode == CMT_A2_SELECT || (a.a_dtype == CMT_F32 && a.lda2 % 4 == 0),
                "cmt_gemm: A2 add mode needs f32 A");
    CMT_REQUIRE(a.A2 == nullptr || a.a2_mode == CMT_A2_ADD || (a.a_dtype == a.w_dtype && a.a_dtype != CMT_F32 &&
                                                               a.lda2 % 8 == 0),
                "cmt_gemm: A2 select mode needs A in the f16/bf16 compute dtype");
    if (a.a_mode == CMT_A_CONV3X3)
        CMT_REQUIRE(a.conv_c % BK == 0 && a.K == 9 * a.conv_c && a.conv_h > 0 && a.conv_w > 0 &&
                    a.M % (a.conv_h * a.conv_w) == 0, "cmt_gemm: bad conv3x3 geometry");
    if (a.a_mode == CMT_A_CONV1D3)
        CMT_REQUIRE(a.K % 3 == 0 && (a.K / 3) % BK == 0 && a.seg_len > 0 && a.M % a.seg_len == 0,
                    "cmt_gemm: bad conv1d3 geometry");
    if (a.c_mode == CMT_C_HEADSPLIT)
        CMT_REQUIRE(a.rows_per_batch > 0 && a.M % a.rows_per_batch == 0, "cmt_gemm: bad head-split rows");
    if (a.plane_max2 != nullptr)
        CMT_REQUIRE(a.c_mode == CMT_C_HEADSPLIT && (a.c_dtype == CMT_F16 || a.c_dtype == CMT_BF16) &&
                    a.w_dtype != CMT_F32 && a.a_dtype == a.w_dtype && a.plane_max_cols % 32 == 0 &&
                    a.plane_max_cols <= a.N,
                    "cmt_gemm: plane_max2 needs a head-split 16-bit C, compute-dtype A and plane_max_cols % 32 == 0");
    hipStream_t s = (hipStream_t)stream;
    if (a.w_dtype == CMT_F16P && x3_eligible(a)) {
        // split GEMMs whose 256-row grid covers most CUs (tools/bench_kernels.py --only split, against
        // the 128 x 128 DMA tile: shared_conv 265 -> 249 us, RV fc1 76 -> 59, RV fc2 76 -> 64, BEV fc2
        // 42 -> 34, RV query fc1 33 -> 20; 128 x 128 x3 tiles everywhere: 280, 65, 69, 37, 22);
        // fusion frame 539 -> 559 frames/s alternating on one box
        const int64_t t256 = (int64_t)(a.N / 128) * cdiv(a.M, 256) * a.batch;
        if (t256 >= 160) return launch_x3<256>(a, s);
    }
    if (a.w_dtype != CMT_F32 && a.a_dtype == a.w_dtype) {
        // LDS-DMA path: 64-deep k stages
        const int kdiv = a.a_mode == CMT_A_CONV3X3 ? a.conv_c : (a.a_mode == CMT_A_CONV1D3 ? a.K / 3 : a.K);
        CMT_REQUIRE(kdiv % 64 == 0, "cmt_gemm: compute-dtype A needs K (per tap) % 64 == 0");
        CMT_REQUIRE(a.ldc % 4 == 0 && (a.R == nullptr || a.ldr % 4 == 0) && a.bias_bstride % 4 == 0,
                    "cmt_gemm: ldc/ldr/bias_bstride must be multiples of 4");
        const int64_t big_tiles = (int64_t)(a.N / 128) * cdiv(a.M, 128) * a.batch;
        // 128 x 128 tiles from ~1.9 workgroups per CU up (480 tiles: a lower threshold made the RV
        // query MLP's fc1 faster alone -- 9.9 vs 12.4 us at 344 tiles -- but the bf16 frame slower,
        // 919 vs 927 frames/s, beside the conv on the second stream), 2 LDS stages
        if (a.N % 128 == 0 && big_tiles >= 480) return launch_dma<128, 128, 2>(a, s);
        // long-K problems a 128x128 grid fills less than twice over (the RV embedding's second
        // GEMM, M = 24 000, N = 256, K = 1024: 376 tiles): still 128 x 128 with 2 stages when N
        // allows (26.7 us vs 30.0 us on 128 x 64 x 3 stages, 36.3 on 128 x 128 x 3), else
        // 128 x 64 tiles (3/4 of the 64 x 64 tiles' operand bytes per output)
        const int64_t mid_tiles = (int64_t)(a.N / 64) * cdiv(a.M, 128) * a.batch;
        if (kdiv >= 512 && a.a_mode == CMT_A_ROWS && mid_tiles >= 480) {
            if (a.N % 128 == 0) return launch_dma<128, 128, 2>(a, s);
            return launch_dma<128, 64, 3>(a, s);
        }
        return launch_dma<64, 64, 4>(a, s);
    }
    // Tile choice: 128x128 when the grid still fills the chip, else 64x64.
    const int64_t big_tiles = (int64_t)(a.N / 128) * cdiv(a.M, 128) * a.batch;
    if (a.N % 128 == 0 && big_tiles >= 384) return launch_tiles<128, 128>(a, s);
    return launch_tiles<64, 64>(a, s);
}
