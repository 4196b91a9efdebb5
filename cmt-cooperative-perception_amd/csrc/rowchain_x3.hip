// Row-block chains of the decoder layer's query side at the reference's
// numerics ('ref' policy, CMT_F16P operands): the split-f16 form of
// rowchain.hip (cmt_chain with dtype CMT_F16P).
//
// A workgroup owns 32 complete query rows and runs the same chains as the f16
// / bf16 kernels (petr_transformer.py:374-487, post-norm order self_attn,
// norm, cross_attn, norm, ffn, norm; mmcv FFN add_identity):
//
//   kind 0, chain A, 1 workgroup per row block:
//       self-attn out_proj + bias + residual -> norms[0] -> Y -> (Y + query_pos) -> cross-attn Q
//   kind 1, chain B1, 4 workgroups per row block (g = FFN quarter):
//       cross-attn out_proj + bias + residual -> norms[1] -> o -> fc1 rows [256g, 256g+256) + ReLU
//       -> fc2 K block g -> fp32 partial WS[g] (g = 0 adds fc2.bias + o)
//   kind 2, chain B2, 3 workgroups per row block (1 on the last layer; g = Q|K|V block):
//       sum of the 4 partials -> norms[2] -> Y; g = 0: post_norm -> OUT (+ its pair copy OUT16)
//       -> next layer's self-attn in_proj block g (Q|K read Y + pos, V reads Y), head-split pairs
//
// Every GEMM operand is an f16 pair (cmt_hip.h CMT_F16P) and every product the
// three f16 MFMA passes hi*hi + lo*hi + hi*lo with fp32 accumulation, as the
// separate split GEMMs compute them.  The activations stay in LDS as pair
// images (hi plane, lo plane: [32 rows][256], 16-byte chunks XOR-swizzled by
// row & 15).  The weights never touch LDS: each of the 8 waves owns 32 output
// columns of every 256-wide sub-GEMM and streams its fragments (hi and lo,
// fragment-major packs: 1 KB contiguous per load instruction) from L2 straight
// into a WRING-deep register ring (a whole sub-GEMM) that runs across sub-GEMM boundaries --
// with pairs the per-workgroup weight bytes double, and the f16 kernels'
// LDS-DMA ring would hold two stages in what LDS is left.  All loads are
// ordinary compiler-visible loads (its waitcnt pass counts them exactly).
// MFMA 32x32x16 in the swapped form (lane = query row), so a row's LayerNorm
// reduces over registers, the lane pair and the 8 waves.
#include "cmt_common.h"

#ifdef CMT_STAMPS
// diagnostic build only (make OUT=../lib_stamps HIPFLAGS+=-DCMT_STAMPS): shader-clock stamps of
// wave 0 of the first 16 workgroups of the last launch of each chain kind, read back by
// cmt_debug_chain_stamps (dev/chain_stamps.py)
__device__ unsigned long long g_chain_stamps[3][16][16];
#define STAMP(K, i)                                                                            \
    do {                                                                                      \
        if (blockIdx.x < 16 && threadIdx.x == 0) g_chain_stamps[K][blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
extern "C" int cmt_debug_chain_stamps(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chain_stamps), sizeof(g_chain_stamps));
}
#else
#define STAMP(K, i) do { } while (0)
#endif

namespace {

constexpr int RB = 32;                    // query rows per workgroup
constexpr int CE = 256;                   // embed dims
constexpr int NWV = 8;                    // waves
constexpr int NTC = 64 * NWV;             // threads
constexpr int VPL = CE / NWV / 2;         // values per lane of a row (16)
constexpr int KS = CE / 16;               // MFMA k-steps per sub-GEMM
constexpr int WRING_DEFAULT = 16;         // k-steps of weight fragments in flight per wave (a whole
                                          // sub-GEMM: one sub-GEMM ahead)
constexpr int PLANE = RB * CE * 2;        // one f16 image [32][256]: 16 KB
constexpr int ACT = 2 * PLANE;            // a pair image: hi plane, lo plane
constexpr int OFF_A = 0, OFF_B = ACT;
constexpr int OFF_PRM = 2 * ACT;
constexpr int PRM_A = 1024, PRM_B = 3840; // floats (cmt_hip.h cmt_chain_args.prm)
constexpr int OFF_RED = OFF_PRM + PRM_B * 4;
constexpr int LDS_TOTAL = OFF_RED + 2 * NWV * RB * 4;

// column of lane value r in wave w's 32-column tile
__device__ __forceinline__ int xcol(int wave, int lh, int r) { return wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh; }

// Weight stream of one wave: up to 3 sub-GEMMs, each a fragment-major pair pack (the Wn layout,
// cmt_hip.h: hi pack then lo pack, lo_off elements apart) of which this wave reads block g.
template <int NSUB, int WRING>
struct WStream {
    const pair_t* base[NSUB];   // this wave's first fragment (hi) of each sub-GEMM
    int64_t lo_off[NSUB];
    int nt;                     // this wave's 32-row half of its 64-row weight group
    pair8_t rh[WRING], rl[WRING];

    __device__ __forceinline__ void load(int step) {   // step = sub * KS + k-step (compile-time after unroll)
        if (step >= NSUB * KS) return;
        const int sub = step / KS, kk = step % KS;
        const pair_t* p = base[sub] + (kk * 2 + nt) * 512;
        rh[step % WRING] = *(const pair8_t*)p;
        rl[step % WRING] = *(const pair8_t*)(p + lo_off[sub]);
    }
};

struct Ctx {
    char* lds;
    int lane, wave, lr, lh;

    __device__ __forceinline__ int col(int r) const { return xcol(wave, lh, r); }
    __device__ __forceinline__ const float* prm() const { return (const float*)(lds + OFF_PRM); }

    // sum over the row's 256 columns (this lane's 16, the lane pair, the 8 waves); slots alternate
    __device__ __forceinline__ float row_sum(float x, int slot) const {
        x = pair_sum(x);
        float* red = (float*)(lds + OFF_RED);
        if (lh == 0) red[(slot * NWV + wave) * RB + lr] = x;
        barrier_mem();
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += red[(slot * NWV + w) * RB + lr];
        return t;
    }

    // nn.LayerNorm (biased variance), weight / bias at parameter offsets
    __device__ __forceinline__ void layernorm(float (&v)[VPL], int w_off, int b_off, float eps) const {
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

    // this lane's values of its row into a pair image (hi plane, lo plane)
    __device__ __forceinline__ void put_act(char* act, const float (&v)[VPL]) const {
        typedef pair_t p4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int c0 = col(4 * g);
            p4 h, l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float x = v[4 * g + j];
                h[j] = (pair_t)x;
                l[j] = (pair_t)(x - (float)h[j]);
            }
            const int off = lr * (CE * 2) + (((c0 >> 3) ^ (lr & 15)) << 4) + (c0 & 7) * 2;
            *(p4*)(act + off) = h;
            *(p4*)(act + PLANE + off) = l;
        }
    }

    // acc = act . W^T of sub-GEMM SUB over K = 256: three f16 passes per k-step; the stream's
    // ring slot of each step refills with the step WRING ahead (into the next sub-GEMM too)
    template <int SUB, int NSUB, int WRING>
    __device__ __forceinline__ void sub_gemm(const char* act, WStream<NSUB, WRING>& ws, f32x16& acc) const {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const int step = SUB * KS + kk;
            const int off = lr * (CE * 2) + (((2 * kk + lh) ^ (lr & 15)) << 4);
            const pair8_t ah = *(const pair8_t*)(act + off);
            const pair8_t al = *(const pair8_t*)(act + PLANE + off);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ws.rh[step % WRING], al, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ws.rl[step % WRING], ah, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ws.rh[step % WRING], ah, acc, 0, 0, 0);
            ws.load(step + WRING);
        }
    }
};

// this lane's VPL fp32 values of `row` (columns xcol) from a [rows][256] fp32 matrix
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

// the B1 -> B2 partials in the lanes' own order (rowchain.hip's private layout)
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

// this wave's first fragment (hi) in a fragment-major pack of a [256 G][256] matrix, block g
__device__ __forceinline__ const pair_t* frag_base(const void* W, int g, int wave, int lane) {
    return (const pair_t*)W + (int64_t)((g * 4 + (wave >> 1)) * 8) * 4 * 512 + lane * 8;
}

// XP (chain B1, ABI 19): the attention output is not read as X but combined here from the
// cross-attention's XS split partials (cmt_attn_fwd with CMT_ATTN_KEEP_PARTIALS; attn_combine_kernel's
// arithmetic in its order, explicit fmas in both), each of the 4 workgroups of a row block
// combining its 32 rows itself -- no combine launch, no pair-row round trip through HBM.
constexpr int XS = 8;

template <int KIND, int WRING, bool XP = false>
__global__ __launch_bounds__(NTC, 1) void chain_x3_kernel(cmt_chain_args a) {
    static_assert(!XP || KIND == 1, "split partials feed chain B1 only");
    __shared__ __attribute__((aligned(16))) char lds[LDS_TOTAL];
    Ctx e;
    e.lds = lds;
    STAMP(KIND, 0);
    const int tid = threadIdx.x;
    e.lane = tid & 63;
    e.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    e.lr = e.lane & 31;
    e.lh = e.lane >> 5;
    const bool has_next = a.Wn != nullptr;
    constexpr int NSUB = KIND == 0 ? 2 : KIND == 1 ? 3 : 1;
    const int parts = KIND == 0 ? 1 : KIND == 1 ? 4 : (has_next ? 3 : 1);
    const int rb = blockIdx.x / parts, g = blockIdx.x - rb * parts;
    const int m0 = rb * RB;
    const int row = min(m0 + e.lr, a.rows - 1);
    const bool row_ok = m0 + e.lr < a.rows;
    char* actA = lds + OFF_A;
    char* actB = lds + OFF_B;
    float* ws = a.WS;
    const int64_t plane = (int64_t)((a.rows + RB - 1) / RB) * RB * CE;   // one partial in tile order

    // ---- the weight stream of this wave (fragment-major pair packs, hi then lo)
    WStream<NSUB, WRING> wst;
    wst.nt = e.wave & 1;
    if constexpr (KIND == 0) {
        wst.base[0] = frag_base(a.Wo, 0, e.wave, e.lane);   // self-attn out_proj
        wst.base[1] = frag_base(a.W1, 0, e.wave, e.lane);   // cross-attn Q projection
        wst.lo_off[0] = wst.lo_off[1] = (int64_t)CE * CE;
    } else if constexpr (KIND == 1) {
        wst.base[0] = frag_base(a.Wo, 0, e.wave, e.lane);   // cross-attn out_proj
        wst.base[1] = frag_base(a.W1, g, e.wave, e.lane);   // fc1 rows [256g, 256g + 256)
        wst.base[2] = frag_base(a.W2, g, e.wave, e.lane);   // fc2 K block g
        wst.lo_off[0] = (int64_t)CE * CE;
        wst.lo_off[1] = wst.lo_off[2] = (int64_t)4 * CE * CE;
    } else {
        wst.base[0] = frag_base(has_next ? a.Wn : a.prm, g, e.wave, e.lane);   // next in_proj block g
        wst.lo_off[0] = (int64_t)3 * CE * CE;
    }
    const bool gemm = KIND != 2 || has_next;

    // ---- prologue loads, in the order their values are needed (vmcnt counts in issue order: a
    // wait for a value loaded after the weight ring's first WRING steps would wait for those
    // too -- the stamps showed ~6 700 cycles to the first barrier that way): the attention output
    // rows and the parameter block (-> LDS), B2's partials / query_pos / old output, then the
    // weight ring, then the LDS writes and the values first used after the first sub-GEMM
    f32x4 xv[4];
    if constexpr (KIND != 2 && !XP) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {                      // 2048 16-byte pieces: hi then lo planes
            const int piece = tid + NTC * i;
            const int pl = piece >> 10, pc = piece & 1023;
            const int r = pc >> 5, ch = pc & 31;
            const int src_row = min(m0 + r, a.rows - 1);
            xv[i] = *(const f32x4*)((const pair_t*)a.X + (int64_t)src_row * (2 * CE) + pl * CE + 8 * ch);
        }
    }
    constexpr int NPRM4 = (KIND == 0 ? PRM_A : PRM_B) / 4;
    constexpr int PRM_IT = (NPRM4 + NTC - 1) / NTC;
    f32x4 pv[PRM_IT];
#pragma unroll
    for (int i = 0; i < PRM_IT; ++i) {
        const int piece = tid + NTC * i;
        if (piece < NPRM4) pv[i] = *(const f32x4*)(a.prm + 4 * piece);
    }
    float res[VPL], qp[VPL], oold[VPL];
    const bool need_p = KIND == 0 || (KIND == 2 && has_next && g < 2);
    const bool max_into = KIND == 2 && g == 0 && (a.out_flags & CMT_LN_MAX_INTO);
    if constexpr (KIND == 2) {
        float t[3][VPL];
        load_tile(ws, rb, e.wave, e.lane, res);
#pragma unroll
        for (int p = 1; p < 4; ++p) load_tile(ws + p * plane, rb, e.wave, e.lane, t[p - 1]);
#pragma unroll
        for (int p = 1; p < 4; ++p)
#pragma unroll
            for (int i = 0; i < VPL; ++i) res[i] += t[p - 1][i];
        if (need_p) {
            load_row(a.P, row, e.wave, e.lh, qp);
        } else {
#pragma unroll
            for (int i = 0; i < VPL; ++i) qp[i] = 0.f;
        }
        if (max_into) {
            load_row(a.OUT, row, e.wave, e.lh, oold);
        } else {
#pragma unroll
            for (int i = 0; i < VPL; ++i) oold[i] = 0.f;
        }
    }
    if (gemm) {
#pragma unroll
        for (int s = 0; s < WRING; ++s) wst.load(s);
    }
    if constexpr (XP) {
        // the split combine (attn_combine_kernel<XS>), rounded to f16 per xround, as pair chunks:
        // pieces (row r, 8-column chunk ch) tid and tid + 512, one at a time behind the weight
        // ring's loads; their XS partial rows of 8 values, offsets and sums from the workspace
        // layout of cmt_attn_fwd (O [XS][B][8][Nq][32], then M, then L)
        const int64_t prow = (int64_t)(a.rows / a.Nq) * 8 * a.Nq;   // partial rows per split
        const float* Op = a.xpart;
        const float* Mp = Op + XS * prow * 32;
        const float* Lp = Mp + XS * prow;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int piece = tid + NTC * i;
            const int r = piece >> 5, ch = piece & 31;
            const int src_row = min(m0 + r, a.rows - 1);
            const int b = src_row / a.Nq, q = src_row - b * a.Nq;
            const int64_t bhq = ((int64_t)b * 8 + (ch >> 2)) * a.Nq + q;
            f32x4 po[XS][2];
            float pm[XS], pls[XS];
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                const float* o = Op + (s * prow + bhq) * 32 + 8 * (ch & 3);
                po[s][0] = *(const f32x4*)o;
                po[s][1] = *(const f32x4*)(o + 4);
                pm[s] = Mp[s * prow + bhq];
                pls[s] = Lp[s * prow + bhq];
            }
            float M = -__builtin_inff();
#pragma unroll
            for (int s = 0; s < XS; ++s) M = pls[s] > 0.f ? fmaxf(M, pm[s]) : M;
            f32x4 n0 = {0.f, 0.f, 0.f, 0.f}, n1 = {0.f, 0.f, 0.f, 0.f};
            float den = 0.f;
#pragma unroll
            for (int s = 0; s < XS; ++s) {
                const float w = pls[s] > 0.f ? __builtin_amdgcn_exp2f(pm[s] - M) : 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    n0[j] = __builtin_fmaf(w, po[s][0][j], n0[j]);
                    n1[j] = __builtin_fmaf(w, po[s][1][j], n1[j]);
                }
                den = __builtin_fmaf(w, pls[s], den);
            }
            const float inv = 1.f / den;
            pair8_t h, l;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float x = (j < 4 ? n0[j] : n1[j - 4]) * inv;
                if (a.xround) x = (float)(f16_t)x;
                h[j] = (pair_t)x;
                l[j] = (pair_t)(x - (float)h[j]);
            }
            const int off = r * (CE * 2) + ((ch ^ (r & 15)) << 4);
            *(pair8_t*)(actA + off) = h;
            *(pair8_t*)(actA + PLANE + off) = l;
        }
    }
    if constexpr (KIND != 2 && !XP) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = tid + NTC * i;
            const int pl = piece >> 10, pc = piece & 1023;
            const int r = pc >> 5, ch = pc & 31;
            *(f32x4*)(actA + pl * PLANE + r * (CE * 2) + ((ch ^ (r & 15)) << 4)) = xv[i];
        }
    }
#pragma unroll
    for (int i = 0; i < PRM_IT; ++i) {
        const int piece = tid + NTC * i;
        if (piece < NPRM4) *(f32x4*)(lds + OFF_PRM + piece * 16) = pv[i];
    }
    if constexpr (KIND != 2) {
        if (a.R) {
            load_row(a.R, row, e.wave, e.lh, res);
        } else {
#pragma unroll
            for (int i = 0; i < VPL; ++i) res[i] = 0.f;
        }
        if (need_p) {
            load_row(a.P, row, e.wave, e.lh, qp);
        } else {
#pragma unroll
            for (int i = 0; i < VPL; ++i) qp[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < VPL; ++i) oold[i] = 0.f;
    }
    STAMP(KIND, 1);
    barrier_mem();   // actA and the parameter block written by every wave
    STAMP(KIND, 2);

    f32x16 acc;
    float v[VPL];
    const float eps = a.eps;
    typedef f16_t h4 __attribute__((ext_vector_type(4)));
    typedef pair_t p4 __attribute__((ext_vector_type(4)));
    if constexpr (KIND == 0) {
        // ---------------- chain A
        e.sub_gemm<0>(actA, wst, acc);                                  // self-attn out_proj
        STAMP(0, 3);
        {
            const float* bo = e.prm();
#pragma unroll
            for (int r = 0; r < VPL; ++r) v[r] = acc[r] + bo[e.col(r)] + res[r];
        }
        e.layernorm(v, 256, 512, eps);                                  // norms[0]
        STAMP(0, 4);
        float u[VPL];
#pragma unroll
        for (int i = 0; i < VPL; ++i) u[i] = v[i] + qp[i];
        e.put_act(actB, u);                                             // (y + query_pos) pairs
        barrier_mem();
        STAMP(0, 5);
        e.sub_gemm<1>(actB, wst, acc);                                  // cross-attn Q projection
        STAMP(0, 6);
        const float* bq = e.prm() + 768;
        h4 qo[4];
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const int c0 = e.col(4 * gg);
            qo[gg] = h4{(f16_t)(acc[4 * gg] + bq[c0]), (f16_t)(acc[4 * gg + 1] + bq[c0 + 1]),
                        (f16_t)(acc[4 * gg + 2] + bq[c0 + 2]), (f16_t)(acc[4 * gg + 3] + bq[c0 + 3])};
        }
        if (row_ok) {
            store_row(a.Y, row, e.wave, e.lh, v);
            const int b = row / a.Nq, rr = row - b * a.Nq;
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int c0 = e.col(4 * gg);
                *(h4*)((f16_t*)a.Q + (((int64_t)b * 8 + (c0 >> 5)) * a.Nq + rr) * 32 + (c0 & 31)) = qo[gg];
            }
        }
        STAMP(0, 7);
        return;
    }
    if constexpr (KIND == 1) {
        // ---------------- chain B1: out_proj + norms[1], then FFN quarter g
        e.sub_gemm<0>(actA, wst, acc);                                  // cross-attn out_proj
        STAMP(1, 3);
        {
            const float* bo = e.prm();
#pragma unroll
            for (int r = 0; r < VPL; ++r) v[r] = acc[r] + bo[e.col(r)] + res[r];
        }
        e.layernorm(v, 256, 512, eps);                                  // norms[1] -> o (FFN residual)
        STAMP(1, 4);
        e.put_act(actB, v);                                             // fc1 operand
        barrier_mem();
        STAMP(1, 5);
        e.sub_gemm<1>(actB, wst, acc);                                  // fc1 rows [256g, 256g + 256)
        STAMP(1, 6);
        {
            const float* b1 = e.prm() + 768 + 256 * g;
            float h[VPL];
#pragma unroll
            for (int r = 0; r < VPL; ++r) h[r] = fmaxf(acc[r] + b1[e.col(r)], 0.f);
            e.put_act(actA, h);                                         // hidden quarter g = fc2 K block g
        }
        barrier_mem();
        STAMP(1, 7);
        e.sub_gemm<2>(actA, wst, acc);                                  // fc2 partial over K block g
        STAMP(1, 8);
        const float* b2 = e.prm() + 1792;
#pragma unroll
        for (int r = 0; r < VPL; ++r) {
            float x = acc[r];
            if (g == 0) x += b2[e.col(r)] + v[r];
            v[r] = x;
        }
        store_tile(ws + g * plane, rb, e.wave, e.lane, v);              // whole row block (clamped rows too)
        STAMP(1, 9);
        return;
    }
    // ---------------- chain B2: norms[2] (+ post_norm), next layer's in_proj block g
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = res[i];
    e.layernorm(v, 2048, 2304, eps);                                    // norms[2] -> next query
    STAMP(2, 3);
    float y[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) y[i] = v[i];
    if (g == 0) {
        e.layernorm(v, 2560, 2816, eps);                                // post_norm -> layer output
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            float x = v[i];
            if (a.out_flags & CMT_LN_NAN_TO_NUM) x = nan_to_num(x);
            if (max_into) x = fmaxf(x, oold[i]);
            v[i] = x;
        }
    }
    if (has_next) {
        float u[VPL];
#pragma unroll
        for (int i = 0; i < VPL; ++i) u[i] = y[i] + qp[i];              // qp = 0 for the V block
        STAMP(2, 4);
        e.put_act(actA, u);                                             // (y + pos) (Q|K) / y (V) pairs
        barrier_mem();
        STAMP(2, 5);
        e.sub_gemm<0>(actA, wst, acc);
        STAMP(2, 6);
    }
    if (row_ok) {
        if (g == 0) {
            store_row(a.Y, row, e.wave, e.lh, y);
            store_row(a.OUT, row, e.wave, e.lh, v);
            if (a.OUT16) {   // the layer output again as pair rows (the task-head GEMM operand)
#pragma unroll
                for (int gg = 0; gg < 4; ++gg)
                    store_pair4((pair_t*)a.OUT16 + (int64_t)row * (2 * CE), CE, e.col(4 * gg),
                                f32x4{v[4 * gg], v[4 * gg + 1], v[4 * gg + 2], v[4 * gg + 3]});
            }
        }
        if (has_next) {
            // head-split pairs [B][24][Nq][64]: per (plane, row) the 32 hi values, then the 32 lo
            const float* bqkv = e.prm() + 3072 + g * CE;
            const int b = row / a.Nq, rr = row - b * a.Nq;
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int c0 = e.col(4 * gg), cc = g * CE + c0;
                p4 h, l;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float x = acc[4 * gg + j] + bqkv[c0 + j];
                    h[j] = (pair_t)x;
                    l[j] = (pair_t)(x - (float)h[j]);
                }
                pair_t* dst = (pair_t*)a.Q + (((int64_t)b * 24 + (cc >> 5)) * a.Nq + rr) * 64 + (cc & 31);
                *(p4*)dst = h;
                *(p4*)(dst + 32) = l;
            }
        }
    }
    STAMP(2, 7);
}

}  // namespace

// cmt_chain with dtype CMT_F16P (capi/rowchain.hip routes here)
int cmt_chain_x3(const cmt_chain_args& a, hipStream_t s) {
    CMT_REQUIRE(a.kind != 0 || a.wo_frag, "cmt_chain: the split chains take fragment-major pair weights (wo_frag)");
    CMT_REQUIRE(a.xpart == nullptr || (a.kind == 1 && a.xsplits == XS && a.Nq > 0 && a.rows % a.Nq == 0 &&
                                       (uintptr_t)a.xpart % 16 == 0),
                "cmt_chain: xpart (split partials) feeds chain B1 with xsplits == 8, rows = B * Nq, 16-byte aligned");
    const int parts = a.kind == 0 ? 1 : a.kind == 1 ? 4 : (a.Wn ? 3 : 1);
    const unsigned grid = (unsigned)(cdiv(a.rows, RB) * parts);
    if (a.kind == 0) chain_x3_kernel<0, WRING_DEFAULT><<<grid, NTC, 0, s>>>(a);
    else if (a.kind == 1 && a.xpart) chain_x3_kernel<1, WRING_DEFAULT, true><<<grid, NTC, 0, s>>>(a);
    else if (a.kind == 1) chain_x3_kernel<1, WRING_DEFAULT><<<grid, NTC, 0, s>>>(a);
    else chain_x3_kernel<2, WRING_DEFAULT><<<grid, NTC, 0, s>>>(a);
    return cmt_check_launch("cmt_chain");
}
