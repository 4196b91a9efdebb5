// Row-block chains of the decoder layer's query side (gfx950).
//
// A workgroup owns 32 complete query rows (all C = 256 columns) and runs a
// short chain of 256 x 256 (K = 256) sub-GEMMs whose operands stay in LDS, with
// the post-norm decoder layer's bias / residual / LayerNorm epilogues in between
// (petr_transformer.py:374-487, operation_order self_attn, norm, cross_attn,
// norm, ffn, norm; mmcv FFN add_identity; LN eps from the module):
//
//   kind 0, chain A (after self-attention), 1 workgroup per row block:
//       out_proj + bias + residual -> norms[0] -> Y -> lowp(Y + query_pos) -> cross-attn Q projection
//   kind 1, chain B1 (after cross-attention), 4 workgroups per row block (g = FFN quarter):
//       out_proj + bias + residual -> norms[1] -> o -> fc1 rows [256g, 256g+256) + ReLU
//       -> fc2 K block g -> fp32 partial WS[g] (g = 0 adds fc2.bias + o, the FFN residual)
//   kind 2, chain B2, 3 workgroups per row block (1 on the last layer; g = Q|K|V block):
//       sum of the 4 partials -> norms[2] -> Y (next query); g = 0: post_norm -> OUT
//       -> next layer's self-attn in_proj block g (Q|K read lowp(Y + pos), V reads lowp(Y))
//
// Why split B: every workgroup streams its sub-GEMMs' weights through LDS, and
// one CU's LDS-DMA stream moves only ~30-90 GB/s (MI355X_MICROARCH.md
// ldsdma-fill), so a 900-row layer is bound by weight bytes per workgroup, not
// by MFMA.  One-workgroup chain B (12 sub-GEMMs, 1.5 MB per workgroup on 29
// CUs) took 54 us; B1 + B2 stream 384 KB / 128 KB per workgroup on 116 / 87.
//
// Every weight reaches LDS as a stream of 16 KB stages (256 weight rows x 32 k)
// through a ring of NSTG slots by LDS-DMA; the stream runs across sub-GEMM
// boundaries.  MFMA 32x32x16 in the swapped form (lane = query row), so a row's
// LayerNorm reduces over registers, the lane pair and the 8 waves.  All global
// stores happen after the last stage and all ordinary global loads before the
// first, so no counted LDS-DMA wait is ever drained early.
//
// Eight waves per workgroup (two per SIMD), each owning 32 output columns (one
// 32x32 MFMA tile) of every sub-GEMM: the weight fragments a wave holds in
// registers halve, and the workgroup keeps twice as many loads in flight --
// each workgroup is bound by how fast one CU pulls its 128-384 KB of weights
// and row data from L2, not by its MFMAs.
#include "cmt_common.h"

#include <cstdio>
#include <cstdlib>

namespace {

constexpr int RB = 32;                         // query rows per workgroup
constexpr int CE = 256;                        // embed dims
constexpr int NWV = 8;                         // waves
constexpr int NTC = 64 * NWV;                  // threads
constexpr int VPL = CE / NWV / 2;              // values per lane of a row (its 32-column tile, lane pair)
constexpr int KSTG = 32;                       // k per weight stage
constexpr int NSTG = 6;                        // weight ring depth
constexpr int STG_BYTES = CE * KSTG * 2;       // 16 KB
constexpr int SUB_STAGES = CE / KSTG;          // 8 stages per sub-GEMM
constexpr int ACT_BYTES = RB * CE * 2;         // 16 KB operand image [32][256] 16-bit
constexpr int OFF_ACT_A = NSTG * STG_BYTES;    // 96 KB
constexpr int OFF_ACT_B = OFF_ACT_A + ACT_BYTES;
constexpr int OFF_PRM = OFF_ACT_B + ACT_BYTES; // fp32 parameter block
constexpr int PRM_A = 1024, PRM_B = 3840;      // floats (cmt_hip.h cmt_chain_args.prm)
constexpr int OFF_RED = OFF_PRM + PRM_B * 4;
constexpr int LDS_TOTAL = OFF_RED + 2 * NWV * RB * 4;
constexpr int DMA_PER_STAGE = STG_BYTES / 16 / NTC;   // 16-byte LDS-DMA pieces per thread per stage

typedef const __attribute__((address_space(1))) void* rc_gaddr_t;
typedef __attribute__((address_space(3))) void* rc_laddr_t;

// counted LDS-DMA wait + every outstanding LDS access of this wave (the
// barrier that follows hands LDS writes to the other waves)
template <int N>
__device__ __forceinline__ void rc_wait() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

template <typename T>
struct Eng {
    typedef typename mfma_traits<T>::frag frag;
    char* lds;
    int tid, lane, wave, lr, lh;
    int issued, consumed, nstages;
    const T *w0, *w1, *w2;   // weights of sub-GEMMs 0, 1, 2 ([256 rows][K], leading dims below)
    int ld0, ld1, ld2;

    __device__ __forceinline__ const T* sub_base(int sub, int& ld) const {
        if (sub == 0) { ld = ld0; return w0; }
        if (sub == 1) { ld = ld1; return w1; }
        ld = ld2;
        return w2;
    }

    __device__ __forceinline__ void issue() {
        if (issued >= nstages) return;
        const int sub = issued / SUB_STAGES, kc = issued % SUB_STAGES;
        int ld;
        const T* W = sub_base(sub, ld);
        char* dst = lds + (issued % NSTG) * STG_BYTES;
#pragma unroll
        for (int i = 0; i < DMA_PER_STAGE; ++i) {
            const int piece = tid + NTC * i;
            const int n = piece >> 2;
            const int lc = (piece & 3) ^ ((n >> 2) & 3);
            __builtin_amdgcn_global_load_lds((rc_gaddr_t)(W + (int64_t)n * ld + kc * KSTG + 8 * lc),
                                             (rc_laddr_t)(dst + piece * 16), 16, 0, 0);
        }
        ++issued;
    }

    // stage `consumed` landed for every wave; then refill the slot of stage consumed-1
    __device__ __forceinline__ void acquire() {
        const int ahead = issued - consumed - 1;   // stages issued after the one needed now
        static_assert(NSTG - 2 == 4, "wait ladder covers 0..4 stages");
        if (ahead >= 4) rc_wait<4 * DMA_PER_STAGE>();
        else if (ahead == 3) rc_wait<3 * DMA_PER_STAGE>();
        else if (ahead == 2) rc_wait<2 * DMA_PER_STAGE>();
        else if (ahead == 1) rc_wait<DMA_PER_STAGE>();
        else rc_wait<0>();
        barrier_mem();
        issue();
    }

    // one stage: acc += W[wave*32 + i][k] * A[row][k] (swapped: lane = row)
    __device__ __forceinline__ void mma_stage(const char* A, f32x16& acc) {
        const char* Wt = lds + (consumed % NSTG) * STG_BYTES;
        const int kc = consumed % SUB_STAGES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const frag af = *(const frag*)(A + lr * (CE * 2) + (((kc * 4 + 2 * ks + lh) ^ (lr & 15)) << 4));
            const int n = wave * 32 + lr;
            const frag wf = *(const frag*)(Wt + n * (KSTG * 2) + (((2 * ks + lh) ^ ((n >> 2) & 3)) << 4));
            acc = mfma_traits<T>::mma(wf, af, acc);
        }
        ++consumed;
    }

    __device__ __forceinline__ void sub_gemm(const char* A, f32x16& acc, bool zero) {
        if (zero) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        }
        for (int kc = 0; kc < SUB_STAGES; ++kc) {
            acquire();
            mma_stage(A, acc);
        }
    }

    // chain B2's single sub-GEMM: each wave owns weight rows [64 wave, 64 wave + 64) of its
    // in_proj block, so its fragments come from global memory straight into registers (all
    // issued in the prologue) instead of through the LDS-DMA ring, whose per-CU landing
    // cadence (~0.6 us per 16 KB stage) bounded the kernel.  Wn is fragment-major
    // (cmt_hip.h cmt_chain_args.Wn): every load instruction reads 1 KB contiguous.
    __device__ __forceinline__ void load_wregs(const T* Wp, int g, frag (&wr)[SUB_STAGES][2]) const {
        // fragment-major layout (cmt_hip.h): wave w4 of the 4-wave geometry, n-tile nt, i.e. weight rows
        // 64 w4 + 32 nt -- this wave's 32 rows for wave = 2 w4 + nt
        const int w4 = wave >> 1, nt = wave & 1;
        const T* base = Wp + (int64_t)((g * 4 + w4) * SUB_STAGES) * 4 * 512 + lane * 8;
#pragma unroll
        for (int kc = 0; kc < SUB_STAGES; ++kc)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) wr[kc][ks] = *(const frag*)(base + ((kc * 2 + ks) * 2 + nt) * 512);
    }

    __device__ __forceinline__ void sub_gemm_regs(const char* A, const frag (&wr)[SUB_STAGES][2], f32x16& acc) const {
        // the operand image was written by all the waves (put_act)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_mem();
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int kc = 0; kc < SUB_STAGES; ++kc)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const frag af = *(const frag*)(A + lr * (CE * 2) + (((kc * 4 + 2 * ks + lh) ^ (lr & 15)) << 4));
                acc = mfma_traits<T>::mma(wr[kc][ks], af, acc);
            }
    }

    // column of this lane's value r (4 consecutive per group r >> 2) in its wave's 32-column tile
    __device__ __forceinline__ int col(int r) const { return wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh; }

    __device__ __forceinline__ const float* prm() const { return (const float*)(lds + OFF_PRM); }

    // sum over the row's 256 columns (this lane's 16, the lane pair, the 8 waves); slots alternate
    __device__ __forceinline__ float row_sum(float x, int slot) {
        x = pair_sum(x);
        float* red = (float*)(lds + OFF_RED);
        if (lh == 0) red[(slot * NWV + wave) * RB + lr] = x;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_mem();
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += red[(slot * NWV + w) * RB + lr];
        return t;
    }

    // in-place LayerNorm (nn.LayerNorm: biased variance) with weight / bias at parameter offsets
    __device__ __forceinline__ void layernorm(float (&v)[VPL], int w_off, int b_off, float eps) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < VPL; ++i) s += v[i];
        const float mean = row_sum(s, 0) * (1.f / CE);
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            const float d = v[i] - mean;
            q += d * d;
        }
        const float rstd = rsqrtf(row_sum(q, 1) * (1.f / CE) + eps);
        const float* pw = prm() + w_off;
        const float* pb = prm() + b_off;
#pragma unroll
        for (int r = 0; r < VPL; ++r) {
            const int c = col(r);
            v[r] = (v[r] - mean) * rstd * pw[c] + pb[c];
        }
    }

    // this lane's values of its row into an operand image [32][256] (16-B chunks XOR row & 15)
    __device__ __forceinline__ void put_act(char* act, const float (&v)[VPL]) {
        typedef T t4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int c0 = col(4 * g);
            const t4 x = {(T)v[4 * g], (T)v[4 * g + 1], (T)v[4 * g + 2], (T)v[4 * g + 3]};
            *(t4*)(act + lr * (CE * 2) + (((c0 >> 3) ^ (lr & 15)) << 4) + (c0 & 7) * 2) = x;
        }
    }
};

// this lane's VPL fp32 values of `row` (columns of Eng::col) from a [rows][256] fp32 matrix
__device__ __forceinline__ void load_row(const float* M, int row, int wave, int lh, float (&v)[VPL]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 x = *(const f32x4*)(M + (int64_t)row * CE + wave * 32 + 8 * g + 4 * lh);
        v[4 * g] = x[0];
        v[4 * g + 1] = x[1];
        v[4 * g + 2] = x[2];
        v[4 * g + 3] = x[3];
    }
}

__device__ __forceinline__ void store_row(float* M, int row, int wave, int lh, const float (&v)[VPL]) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
        *(f32x4*)(M + (int64_t)row * CE + wave * 32 + 8 * g + 4 * lh) =
            f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
}

// The B1 -> B2 partials workspace is private to the chains, so it is kept in
// the lanes' own order: per (plane, row block, wave, 16-byte group j) one
// contiguous 1 KB slab, lane-major.  Every wave instruction then moves 1 KB
// of consecutive bytes (8 cache lines) instead of 32-byte pieces of 32 rows
// (32 lines), which is what bounded chain B2 (~9 us for one workgroup).
__device__ __forceinline__ void load_tile(const float* M, int rb, int wave, int lane, float (&v)[VPL]) {
    const float* p = M + (int64_t)rb * RB * CE + wave * (VPL * 64) + lane * 4;
#pragma unroll
    for (int j = 0; j < VPL / 4; ++j) {
        const f32x4 x = *(const f32x4*)(p + j * 256);
        v[4 * j] = x[0];
        v[4 * j + 1] = x[1];
        v[4 * j + 2] = x[2];
        v[4 * j + 3] = x[3];
    }
}

__device__ __forceinline__ void store_tile(float* M, int rb, int wave, int lane, const float (&v)[VPL]) {
    float* p = M + (int64_t)rb * RB * CE + wave * (VPL * 64) + lane * 4;
#pragma unroll
    for (int j = 0; j < VPL / 4; ++j)
        *(f32x4*)(p + j * 256) = f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
}

// KIND is compile-time: each chain kind gets its own register allocation (chain A's two
// register-streamed weight sets would otherwise be live in every kind's code)
template <typename T, int KIND>
__global__ __launch_bounds__(NTC, 1) void chain_kernel(cmt_chain_args a) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) char lds[LDS_TOTAL];
    Eng<T> e;
    e.lds = lds;
    e.tid = threadIdx.x;
    e.lane = threadIdx.x & 63;
    e.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e.lr = e.lane & 31;
    e.lh = e.lane >> 5;
    e.issued = e.consumed = 0;
    constexpr int kind = KIND;
    const bool has_next = a.Wn != nullptr;
    // workgroup -> (row block, part g)
    const int parts = kind == 0 ? 1 : kind == 1 ? 4 : (has_next ? 3 : 1);
    const int rb = blockIdx.x / parts, g = blockIdx.x - rb * parts;
    const T* Wo = (const T*)a.Wo;
    const bool wo_regs = kind == 0 && a.wo_frag;   // chain A with fragment-major Wo: no LDS weight ring
    if (kind == 0) {
        e.w0 = Wo; e.ld0 = CE;
        e.w1 = nullptr; e.ld1 = CE;        // the Q projection streams into registers (fragment-major W1)
        e.nstages = wo_regs ? 0 : SUB_STAGES;
    } else if (kind == 1) {
        e.w0 = Wo; e.ld0 = CE;
        e.w1 = (const T*)a.W1 + (int64_t)g * CE * CE; e.ld1 = CE;       // fc1 rows [256g, 256g + 256)
        e.w2 = nullptr; e.ld2 = 4 * CE;    // fc2 K block g streams into registers (fragment-major W2)
        e.nstages = 2 * SUB_STAGES;
    } else {
        e.w0 = Wo; e.ld0 = CE;             // unused: B2's in_proj block streams into registers
        e.nstages = 0;
    }
    const int m0 = rb * RB;
    const int row = min(m0 + e.lr, a.rows - 1);
    const bool row_ok = m0 + e.lr < a.rows;
    char* actA = lds + OFF_ACT_A;
    char* actB = lds + OFF_ACT_B;
    float* ws = (float*)a.WS;
    const int64_t plane = (int64_t)((a.rows + RB - 1) / RB) * RB * CE;   // one partial in tile order

    // ---- prologue: every ordinary load and the first LDS-DMAs, then one full wait
    float res[VPL], qp[VPL], oold[VPL];
    if (kind == 2) {
        // the FFN output + residual: sum of the four B1 partials
        float t[VPL];
        load_tile(ws, rb, e.wave, e.lane, res);
#pragma unroll
        for (int p = 1; p < 4; ++p) {
            load_tile(ws + p * plane, rb, e.wave, e.lane, t);
#pragma unroll
            for (int i = 0; i < VPL; ++i) res[i] += t[i];
        }
    } else if (a.R) {
        load_row(a.R, row, e.wave, e.lh, res);
    } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) res[i] = 0.f;
    }
    const bool need_p = kind == 0 || (kind == 2 && has_next && g < 2);
    if (need_p) {
        load_row(a.P, row, e.wave, e.lh, qp);
    } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) qp[i] = 0.f;
    }
    const bool max_into = kind == 2 && g == 0 && (a.out_flags & CMT_LN_MAX_INTO);
    if (max_into) {
        load_row(a.OUT, row, e.wave, e.lh, oold);
    } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) oold[i] = 0.f;
    }
    if (kind != 2) {
        // attention output rows -> actA (32 rows x 32 chunks, swizzled)
#pragma unroll
        for (int i = 0; i < ACT_BYTES / 16 / NTC; ++i) {
            const int piece = e.tid + NTC * i;
            const int r = piece >> 5;
            const int lc = (piece & 31) ^ (r & 15);
            const int src_row = min(m0 + r, a.rows - 1);
            __builtin_amdgcn_global_load_lds((rc_gaddr_t)((const T*)a.X + (int64_t)src_row * CE + 8 * lc),
                                             (rc_laddr_t)(actA + piece * 16), 16, 0, 0);
        }
    }
    const int nprm = kind == 0 ? PRM_A : PRM_B;
    for (int piece = e.tid; piece < (nprm >> 2); piece += NTC)
        __builtin_amdgcn_global_load_lds((rc_gaddr_t)(a.prm + 4 * piece), (rc_laddr_t)(lds + OFF_PRM + piece * 16),
                                         16, 0, 0);
#pragma unroll
    for (int s = 0; s < NSTG - 1; ++s) e.issue();
    typename Eng<T>::frag wr[SUB_STAGES][2];
    typename Eng<T>::frag wr0[kind == 0 ? SUB_STAGES : 1][2];
    if constexpr (kind == 0) {
        if (wo_regs) e.load_wregs(Wo, 0, wr0);
    }
    if (kind == 2 && has_next) e.load_wregs((const T*)a.Wn, g, wr);
    if (kind == 0) e.load_wregs((const T*)a.W1, 0, wr);
    if (kind == 1) e.load_wregs((const T*)a.W2, g, wr);
    // first use of the ordinary loads: everything issued so far has landed after this
    asm volatile("" ::"v"(res[0]), "v"(res[VPL - 1]), "v"(qp[0]), "v"(qp[VPL - 1]), "v"(oold[0]),
                 "v"(oold[VPL - 1]));
    rc_wait<0>();
    barrier_mem();

    f32x16 acc;
    float v[VPL];
    const float eps = a.eps;
    if (kind == 0) {
        // ---------------- chain A
        if constexpr (kind == 0) {
            if (wo_regs) e.sub_gemm_regs(actA, wr0, acc);              // out_proj (register weights)
            else e.sub_gemm(actA, acc, true);                          // out_proj (LDS weight ring)
        }
        {
            const float* bo = e.prm();
#pragma unroll
            for (int r = 0; r < VPL; ++r) v[r] = acc[r] + bo[e.col(r)] + res[r];
        }
        e.layernorm(v, 256, 512, eps);                                 // norms[0]
        float y[VPL];
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            y[i] = v[i];
            v[i] += qp[i];
        }
        e.put_act(actB, v);                                            // lowp(y + query_pos)
        e.sub_gemm_regs(actB, wr, acc);                                // cross-attn Q projection
        const float* bq = e.prm() + 768;
        t4 qo[4];
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const int c0 = e.col(4 * gg);
            qo[gg] = t4{(T)(acc[4 * gg] + bq[c0]), (T)(acc[4 * gg + 1] + bq[c0 + 1]), (T)(acc[4 * gg + 2] + bq[c0 + 2]),
                        (T)(acc[4 * gg + 3] + bq[c0 + 3])};
        }
        if (row_ok) {
            store_row(a.Y, row, e.wave, e.lh, y);
            const int b = row / a.Nq, rr = row - b * a.Nq;
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int c0 = e.col(4 * gg);
                *(t4*)((T*)a.Q + (((int64_t)b * 8 + (c0 >> 5)) * a.Nq + rr) * 32 + (c0 & 31)) = qo[gg];
            }
        }
        return;
    }

    if (kind == 1) {
        // ---------------- chain B1: out_proj + norms[1], then FFN quarter g
        e.sub_gemm(actA, acc, true);                                   // out_proj
        {
            const float* bo = e.prm();
#pragma unroll
            for (int r = 0; r < VPL; ++r) v[r] = acc[r] + bo[e.col(r)] + res[r];
        }
        e.layernorm(v, 256, 512, eps);                                 // norms[1] -> o (FFN residual)
        e.put_act(actB, v);                                            // lowp(o): fc1 operand
        e.sub_gemm(actB, acc, true);                                   // fc1 rows [256g, 256g + 256)
        {
            const float* b1 = e.prm() + 768 + 256 * g;
            float h[VPL];
#pragma unroll
            for (int r = 0; r < VPL; ++r) h[r] = fmaxf(acc[r] + b1[e.col(r)], 0.f);
            e.put_act(actA, h);                                        // hidden quarter g = fc2 K block g
        }
        e.sub_gemm_regs(actA, wr, acc);                                // fc2 partial over K block g
        const float* b2 = e.prm() + 1792;
#pragma unroll
        for (int r = 0; r < VPL; ++r) {
            float x = acc[r];
            if (g == 0) x += b2[e.col(r)] + v[r];
            v[r] = x;
        }
        store_tile(ws + g * plane, rb, e.wave, e.lane, v);             // whole row block (clamped rows too)
        return;
    }

    // ---------------- chain B2: norms[2] (+ post_norm), next layer's in_proj block g
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = res[i];
    e.layernorm(v, 2048, 2304, eps);                                   // norms[2] -> next query
    float y[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) y[i] = v[i];
    if (g == 0) {
        e.layernorm(v, 2560, 2816, eps);                               // post_norm -> layer output
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            float x = v[i];
            if (a.out_flags & CMT_LN_NAN_TO_NUM) x = nan_to_num(x);
            if (max_into) x = fmaxf(x, oold[i]);
            v[i] = x;
        }
    }
    t4 qo[4];
    if (has_next) {
        float u[VPL];
#pragma unroll
        for (int i = 0; i < VPL; ++i) u[i] = y[i] + qp[i];             // qp = 0 for the V block
        e.put_act(actA, u);                                            // lowp(y + pos) (Q|K) / lowp(y) (V)
        e.sub_gemm_regs(actA, wr, acc);
        const float* bqkv = e.prm() + 3072 + g * CE;
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const int c0 = e.col(4 * gg);
            qo[gg] = t4{(T)(acc[4 * gg] + bqkv[c0]), (T)(acc[4 * gg + 1] + bqkv[c0 + 1]),
                        (T)(acc[4 * gg + 2] + bqkv[c0 + 2]), (T)(acc[4 * gg + 3] + bqkv[c0 + 3])};
        }
    }
    if (row_ok) {
        if (g == 0) {
            store_row(a.Y, row, e.wave, e.lh, y);
            store_row(a.OUT, row, e.wave, e.lh, v);
            if (a.OUT16) {
#pragma unroll
                for (int gg = 0; gg < 4; ++gg)
                    *(t4*)((T*)a.OUT16 + (int64_t)row * CE + e.col(4 * gg)) =
                        t4{(T)v[4 * gg], (T)v[4 * gg + 1], (T)v[4 * gg + 2], (T)v[4 * gg + 3]};
            }
        }
        if (has_next) {
            const int b = row / a.Nq, rr = row - b * a.Nq;
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int c0 = g * CE + e.col(4 * gg);
                *(t4*)((T*)a.Q + (((int64_t)b * 24 + (c0 >> 5)) * a.Nq + rr) * 32 + (c0 & 31)) = qo[gg];
            }
        }
    }
}

}  // namespace

int cmt_chain_x3(const cmt_chain_args& a, hipStream_t s);   // rowchain_x3.hip

extern "C" int cmt_chain(const cmt_chain_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_chain: null args");
    const cmt_chain_args& a = *ap;
    CMT_REQUIRE(a.kind >= 0 && a.kind <= 2, "cmt_chain: kind must be 0 (A), 1 (B1) or 2 (B2)");
    CMT_REQUIRE(a.rows > 0 && a.Nq > 0 && a.rows % a.Nq == 0, "cmt_chain: rows must be B * Nq");
    CMT_REQUIRE(a.dtype == CMT_F16 || a.dtype == CMT_BF16 || a.dtype == CMT_F16P,
                "cmt_chain: dtype must be f16, bf16 or the f16 pair (CMT_F16P)");
    CMT_REQUIRE(a.prm && a.Y, "cmt_chain: null pointer");
    if (a.kind == 0) CMT_REQUIRE(a.X && a.P && a.Wo && a.W1 && a.Q, "cmt_chain: chain A needs X, P, Wo, W1, Q");
    if (a.kind == 1)
        CMT_REQUIRE((a.X || a.xpart) && a.Wo && a.W1 && a.W2 && a.WS,
                    "cmt_chain: chain B1 needs X (or xpart), Wo, W1, W2, WS");
    CMT_REQUIRE(a.xpart == nullptr || a.dtype == CMT_F16P, "cmt_chain: xpart is a split-chain (CMT_F16P) input");
    if (a.kind == 2) {
        CMT_REQUIRE(a.WS && a.OUT, "cmt_chain: chain B2 needs WS and OUT");
        CMT_REQUIRE(a.Wn == nullptr || (a.P && a.Q), "cmt_chain: chain B2 with Wn needs P and Q");
    } else {
        CMT_REQUIRE(a.OUT16 == nullptr, "cmt_chain: OUT16 is a chain B2 output");
    }
    CMT_REQUIRE(((uintptr_t)a.X | (uintptr_t)a.prm | (uintptr_t)a.Wo | (uintptr_t)a.W1 | (uintptr_t)a.W2 |
                 (uintptr_t)a.Wn | (uintptr_t)a.P | (uintptr_t)a.Y | (uintptr_t)a.R | (uintptr_t)a.OUT |
                 (uintptr_t)a.WS | (uintptr_t)a.Q) % 16 == 0 && (uintptr_t)a.OUT16 % 8 == 0,
                "cmt_chain: buffers must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    if (a.dtype == CMT_F16P) return cmt_chain_x3(a, s);   // rowchain_x3.hip
    const int parts = a.kind == 0 ? 1 : a.kind == 1 ? 4 : (a.Wn ? 3 : 1);
    const unsigned grid = (unsigned)(cdiv(a.rows, RB) * parts);
#define CHAIN_LAUNCH(T)                                                    \
    do {                                                                   \
        if (a.kind == 0) chain_kernel<T, 0><<<grid, NTC, 0, s>>>(a);       \
        else if (a.kind == 1) chain_kernel<T, 1><<<grid, NTC, 0, s>>>(a);  \
        else chain_kernel<T, 2><<<grid, NTC, 0, s>>>(a);                   \
    } while (0)
    if (a.dtype == CMT_BF16) CHAIN_LAUNCH(bf16_t);
    else CHAIN_LAUNCH(f16_t);
#undef CHAIN_LAUNCH
    return cmt_check_launch("cmt_chain");
}
