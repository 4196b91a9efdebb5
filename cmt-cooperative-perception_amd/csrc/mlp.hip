// Linear -> ReLU -> Linear in one launch at the reference's fp32 numerics
// (cmt_mlp2_x3, cmt_hip.h): the camera position encoder rv_embedding
// (cmt_head.py:297-301) over the frustum coordinates of _rv_pe (cmt_head.py:
// 417-433, 24 000 rows per nuScenes frame) and the query coordinates of
// _rv_query_embed (cmt_head.py:439-467).
//
// The two-GEMM form writes the 1024-wide hidden activation as f16 pairs to HBM
// (98 MB per frame) and reads it back; its short-K first GEMM (K = 192, six
// k-stages per tile) is pipeline fill and epilogue, its 256-column second GEMM
// covers 188 tiles of a 256-CU chip.  Here one wave owns 32 rows end to end:
//
//   A fragments (its rows, all K) stay in registers for the whole launch;
//   for each 32-unit hidden block hb:
//     H^T[hb] = W1[hb] . A^T            (swapped 32x32x16 form: lane = row,
//                                        registers = hidden units)
//     H = relu(H + b1) split into f16 hi / lo in registers
//     OUT^T += W2[:, hb] . H^T          (H^T's registers are the B operand: the
//                                        pack orders W2's k like them, so the
//                                        hidden tile never leaves the wave)
//
// Every product is the three-pass split-f16 product of cmt_gemm (W_hi A_lo +
// W_lo A_hi + W_hi A_hi, fp32 accumulation); fc1 runs cmt_gemm's k order, so H
// equals the two-GEMM path's hidden values bit for bit.  The weights of a hidden
// block (W1: K/16 x 2 KB, W2: 32 KB) are shared by the workgroup's 4 waves
// through LDS: a two-slot ring per matrix filled by LDS-DMA one block ahead, one
// barrier per block, and the MFMAs of fc2(hb) interleaved with those of
// fc1(hb + 1) (independent accumulators).  Each wave issues its DMA pieces one
// per MFMA step in the first half of a block, behind that step's MFMAs (issued
// as a burst after the barrier they idled the matrix pipe: 95 -> 89 us for the
// fused camera rows, profiles/r6_experiments.txt r6j).  One wave per SIMD: the 8 output
// accumulator tiles (128 registers), the A fragments (96 at K = 192) and the
// hidden tile need the whole 512-register file.
#include "cmt_common.h"

#include <type_traits>

namespace {

constexpr int MW = 4;               // waves per workgroup, one per SIMD
constexpr int MROWS = 32 * MW;      // rows per workgroup
constexpr int NOUT = 256;           // output width
constexpr int NOT = NOUT / 32;      // output tiles per wave
constexpr int FRAG_B = 1024;        // one fragment image: 64 lanes x 16 bytes
constexpr int W2_BLK = NOT * 2 * 2 * FRAG_B;   // one hidden block of W2p: 32 KB
constexpr int MAX_HD = 2048;
        // hidden width bound (b1 staged in LDS)

typedef const __attribute__((address_space(1))) void* mlp_gaddr_t;
typedef __attribute__((address_space(3))) void* mlp_laddr_t;

__device__ __forceinline__ void mlp_glds16(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds((mlp_gaddr_t)src, (mlp_laddr_t)lds, 16, 0, 0);
}

__device__ __forceinline__ f32x16 mma3(const pair8_t& wh, const pair8_t& wl, const pair8_t& xh, const pair8_t& xl,
                                       f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc, 0, 0, 0);
}

// KS = K / 16; PD = the LDS fragment prefetch distance in steps (3: same time, 4: +8 %,
// profiles/r4t_mlp_prefetch.txt)
// GEO / RX (ABI 20): the frustum coordinates generated in the prologue and the residual read
// from the NCHW image features in the epilogue (cmt_hip.h cmt_mlp2_args.geo_i2l / rx)
template <int KS, int PD = 2, bool GEO = false, bool RX = false>
__global__ __launch_bounds__(64 * MW, 1) void mlp2_x3_kernel(cmt_mlp2_args a) {
    constexpr int W1_BLK = KS * 2 * FRAG_B;
    __shared__ __attribute__((aligned(16))) char lds[2 * W1_BLK + 2 * W2_BLK + MAX_HD * 4 + (GEO ? 64 * 4 : 0)];
    char* const s1 = lds;                 // W1 ring: 2 x W1_BLK
    char* const s2 = lds + 2 * W1_BLK;    // W2 ring: 2 x W2_BLK
    float* const sb1 = (float*)(lds + 2 * W1_BLK + 2 * W2_BLK);   // b1 (a global load per block
                                                                  // cost a memory round trip each)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int z = blockIdx.y;
    const int m = blockIdx.x * MROWS + wave * 32 + lr;
    const int row = min(m, a.M - 1);
    const int nhb = a.Hd / 32;
    const char* const w1g = (const char*)a.W1p;
    const char* const w2g = (const char*)a.W2p;

    // LDS-DMA of hidden block hb's fragments: piece p of a matrix by wave p % MW
    auto issue_w1 = [&](int hb) {
        if (hb >= nhb) return;
        const char* src = w1g + (int64_t)hb * W1_BLK + lane * 16;
        char* dst = s1 + (hb & 1) * W1_BLK;
#pragma unroll
        for (int p = wave; p < 2 * KS; p += MW) mlp_glds16(src + p * FRAG_B, dst + p * FRAG_B);
    };
    auto issue_w2 = [&](int hb) {
        if (hb >= nhb) return;
        const char* src = w2g + (int64_t)hb * W2_BLK + lane * 16;
        char* dst = s2 + (hb & 1) * W2_BLK;
#pragma unroll
        for (int p = wave; p < 4 * NOT; p += MW) mlp_glds16(src + p * FRAG_B, dst + p * FRAG_B);
    };
    issue_w1(0);
    issue_w2(0);
    issue_w1(1);
    for (int i = tid; i < a.Hd / 4; i += 64 * MW) *(f32x4*)(sb1 + 4 * i) = *(const f32x4*)(a.b1 + 4 * i);

    // this lane's row of A as the B operand of fc1 (k = 16 ks + 8 lh + j), hi and lo planes
    pair8_t ah[KS], al[KS];
    const int ghw = GEO || RX ? a.geo_h * a.geo_w : 1;
    const int gview = row / ghw, gpix = row - gview * ghw;      // GEO / RX: view and pixel of the row
    const int gimg = z * (a.M / ghw) + gview;
#ifndef CMT_MLP_DIAG
#define CMT_MLP_DIAG 0   // dev diagnostics (wrong results): 1 no C2 stores, 2 no NCHW loads, 4 no coordinates,
                         // 8 no weight DMA after the prologue
#endif
    if constexpr (GEO && (CMT_MLP_DIAG & 4)) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) { ah[ks] = pair8_t{}; al[ks] = pair8_t{}; }
    } else if constexpr (GEO) {
        // rv_pe_coords_kernel8's arithmetic (elementwise.hip), element k = 3 depth + coordinate.
        // Element 16 ks + 8 lh + j is coordinate (ks + 2 lh + j) mod 3: with the matrix rows and
        // the range rotated by 2 lh once per lane, the row index (ks + j) mod 3 is a compile-time
        // constant (a lane-divergent register-array index is a waterfall loop); the depth values
        // d (one fp32 division each) come from an LDS table the workgroup fills first
        const int gw = gpix % a.geo_w, gh = gpix / a.geo_w;
        const float u = (float)gw * a.geo_pad_w / (float)a.geo_w;
        const float v = (float)gh * a.geo_pad_h / (float)a.geo_h;
        const float* Mx = a.geo_i2l + (int64_t)gimg * 16;
        float mr[3][4], plo[3], pspan[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int src0 = q, src1 = (q + 2) % 3;        // lh = 0 / lh = 1
#pragma unroll
            for (int i = 0; i < 4; ++i) mr[q][i] = lh ? Mx[src1 * 4 + i] : Mx[src0 * 4 + i];
            plo[q] = lh ? a.geo_pc[src1] : a.geo_pc[src0];
            pspan[q] = lh ? a.geo_pc[3 + src1] - a.geo_pc[src1] : a.geo_pc[3 + src0] - a.geo_pc[src0];
        }
        float* dtab = sb1 + MAX_HD;                         // 3 D depth values after b1 (KS * 16 / 3 <= 64)
        if (tid < a.geo_D) dtab[tid] = 1.f + (float)tid * (a.geo_depth_max - 1.f) / (float)a.geo_D;
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int kk = 16 * ks + 8 * lh + j;
                const int r = (ks + j) % 3;                 // the rotated row: compile-time
                const float d = dtab[kk / 3];
                const float c0 = u * d, c1 = v * d;
                float s = mr[r][0] * c0;
                s = fmaf(mr[r][1], c1, s);
                s = fmaf(mr[r][2], d, s);
                s = fmaf(mr[r][3], 1.f, s);
                const float x = (s - plo[r]) / pspan[r];
                const pair_t h = (pair_t)x;
                ah[ks][j] = h;
                al[ks][j] = (pair_t)(x - (float)h);
            }
    } else {
        const pair_t* Ar = (const pair_t*)a.A + (int64_t)z * a.a_bstride + (int64_t)row * a.lda;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            ah[ks] = *(const pair8_t*)(Ar + 16 * ks + 8 * lh);
            al[ks] = *(const pair8_t*)(Ar + a.K + 16 * ks + 8 * lh);
        }
    }

    f32x16 oacc[NOT], hacc;
#pragma unroll
    for (int t = 0; t < NOT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[t][r] = 0.f;
    pair8_t hh[2], hl[2];   // the hidden tile as fc2's B operand (k-steps 0, 1), hi and lo

    // fc1 of block hb from its W1 slot into hacc
    auto fc1 = [&](int hb) {
        const char* w = s1 + (hb & 1) * W1_BLK + lane * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) hacc[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const pair8_t wh = *(const pair8_t*)(w + (2 * ks) * FRAG_B);
            const pair8_t wl = *(const pair8_t*)(w + (2 * ks + 1) * FRAG_B);
            hacc = mma3(wh, wl, ah[ks], al[ks], hacc);
        }
    };
    // relu(hacc + b1) -> pairs; register r of lane half lh is hidden unit 8 (r >> 2) + 4 lh + (r & 3)
    auto split_hidden = [&](int hb) {
        const float* b1 = sb1 + hb * 32 + 4 * lh;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 bv = *(const f32x4*)(b1 + 8 * g);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = fmaxf(hacc[4 * g + e] + bv[e], 0.f) + 0.f;
                const pair_t h = (pair_t)x;
                hh[g >> 1][4 * (g & 1) + e] = h;
                hl[g >> 1][4 * (g & 1) + e] = (pair_t)(x - (float)h);
            }
        }
    };
    // fc2 over block hb (its W2 slot), interleaved with fc1 of block hb + 1 when there is one.
    // Step t of the block's MFMA stream: with fc1, t < 2 KS alternates fc2 step t / 2 and fc1
    // step t / 2, then fc2 steps KS .. 15 follow; each step is a triple on one accumulator whose
    // two weight fragments (hi, lo) are read from LDS two steps ahead (a 3-slot register ring),
    // the order pinned by scheduling barriers -- left to itself the compiler read each pair right
    // before its MFMAs and waited for it (lgkmcnt(0)) 28 times per block.
    // this wave's j-th LDS-DMA piece of block hb's successors: W2(hb + 1) pieces first (needed from
    // the next block's first fc2 step), then W1(hb + 2)
    constexpr int NW2 = 4 * NOT / MW, NW1 = (2 * KS + MW - 1) / MW;
    auto dma_piece = [&](int hb, int j) {
        if (j < NW2) {
            if (hb + 1 >= nhb) return;
            const int p = wave + MW * j;
            mlp_glds16(w2g + (int64_t)(hb + 1) * W2_BLK + lane * 16 + p * FRAG_B,
                       s2 + ((hb + 1) & 1) * W2_BLK + p * FRAG_B);
        } else {
            const int p = wave + MW * (j - NW2);
            if (hb + 2 >= nhb || p >= 2 * KS) return;
            mlp_glds16(w1g + (int64_t)(hb + 2) * W1_BLK + lane * 16 + p * FRAG_B, s1 + (hb & 1) * W1_BLK + p * FRAG_B);
        }
    };
    auto fc2_fc1 = [&](int hb, auto next_c) {
        constexpr bool next = decltype(next_c)::value;   // compile-time: a branch-free MFMA stream
        constexpr int NSTEP = next ? 2 * NOT + KS : 2 * NOT;
        const char* w2 = s2 + (hb & 1) * W2_BLK + lane * 16;
        const char* w1 = s1 + ((hb + 1) & 1) * W1_BLK + lane * 16;
        auto is_fc2 = [](int t) { return !next || t >= 2 * KS || (t & 1) == 0; };
        auto index = [](int t) { return !next ? t : (t < 2 * KS ? t >> 1 : t - KS); };
        auto addr = [&](int t) { return (is_fc2(t) ? w2 : w1) + index(t) * 2 * FRAG_B; };
        if constexpr (next) {
#pragma unroll
            for (int r = 0; r < 16; ++r) hacc[r] = 0.f;
        }
        // fragments PD steps ahead (a register ring of PD + 1 slots)
        pair8_t fh[PD + 1], fl[PD + 1];
#pragma unroll
        for (int t = 0; t < PD; ++t) {
            fh[t] = *(const pair8_t*)addr(t);
            fl[t] = *(const pair8_t*)(addr(t) + FRAG_B);
        }
#pragma unroll
        for (int t = 0; t < NSTEP; ++t) {
            if (t + PD < NSTEP) {
                fh[(t + PD) % (PD + 1)] = *(const pair8_t*)addr(t + PD);
                fl[(t + PD) % (PD + 1)] = *(const pair8_t*)(addr(t + PD) + FRAG_B);
            }
            const int i = index(t);
            const int sl = t % (PD + 1);
            if (is_fc2(t)) oacc[i >> 1] = mma3(fh[sl], fl[sl], hh[i & 1], hl[i & 1], oacc[i >> 1]);
            else hacc = mma3(fh[sl], fl[sl], ah[i], al[i], hacc);
            // one weight piece per step behind the step's MFMAs (NW2 + NW1 <= NSTEP for every KS):
            // the wave issues its DMA while the matrix pipe is busy, half a block ahead of the wait
            if constexpr (next && !(CMT_MLP_DIAG & 8))
                if (t < NW2 + NW1) dma_piece(hb, t);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_mem();   // W1(0), W2(0), W1(1) landed for every wave's pieces
    fc1(0);
    split_hidden(0);
    for (int hb = 0; hb + 1 < nhb; ++hb) {
        // W2(hb) and W1(hb + 1) (issued one block ago) landed; every wave is past block hb - 1,
        // so the slots of W2(hb - 1) and W1(hb) take W2(hb + 1) and W1(hb + 2)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_mem();
        fc2_fc1(hb, std::true_type{});
        split_hidden(hb + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_mem();
    // RX: the row's 256 NCHW feature values are loaded here, into the registers fc1's A operand
    // held, so their memory round trip runs under the last block's fc2 instead of the epilogue's
    const float* const xrow = RX ? a.rx + (int64_t)gimg * NOUT * ghw + gpix : nullptr;
    float xv[RX ? 4 : 1][2][4][4];
    if constexpr (RX) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        xv[q][tt][g][e] = (CMT_MLP_DIAG & 2) ? 0.f
                                                             : xrow[(int64_t)((2 * q + tt) * 32 + 8 * g + 4 * lh + e) * ghw];
    }
    fc2_fc1(nhb - 1, std::false_type{});   // the last block: fc2 only

    if constexpr (RX) {
        // ---- fused camera rows: the memory-row pair (C2) from the NCHW features and
        // out = acc + (b2 + pair value) (C), both staged through LDS per column quarter so every
        // global store is 16 contiguous bytes of a 128-byte row segment (8 lanes per row)
        __syncthreads();   // every wave is past its last weight-ring read: the rings become staging
        char* const stg = lds + wave * 16384;            // 4 slices [32 rows][64 cols] f16: C hi / lo, C2 hi / lo
        const int mw0 = blockIdx.x * MROWS + wave * 32;  // the wave's first row
        bool bad = false;
        typedef pair_t p4 __attribute__((ext_vector_type(4)));
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        auto sw = [](int r, int c16) { return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4); };
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int ot = 2 * q + tt;
                    const int n = ot * 32 + 8 * g + 4 * lh;
                    const f32x4 bv = *(const f32x4*)(a.b2 + n);
                    p4 h2, l2, hc, lc;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        // the pair cmt_nchw_to_rows writes, and its value as the pair R row reads back
                        const float x = xv[q][tt][g][e];
                        bad |= f16_unrepresentable(x);
                        h2[e] = (pair_t)x;
                        l2[e] = (pair_t)(x - (float)h2[e]);
                        const float rv = (float)h2[e] + (float)l2[e];
                        const float v = oacc[ot][4 * g + e] + (bv[e] + rv);
                        hc[e] = (pair_t)v;
                        lc[e] = (pair_t)(v - (float)hc[e]);
                    }
                    const int off = sw(lr, 4 * tt + g) + 8 * lh;
                    *(p4*)(stg + off) = hc;
                    *(p4*)(stg + 4096 + off) = lc;
                    *(p4*)(stg + 8192 + off) = h2;
                    *(p4*)(stg + 12288 + off) = l2;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 8 * i + (lane >> 3), ch = lane & 7;
                const int mr = mw0 + r;
                const int off = sw(r, ch);
                const u4 v0 = *(const u4*)(stg + off), v1 = *(const u4*)(stg + 4096 + off);
                const u4 v2 = *(const u4*)(stg + 8192 + off), v3 = *(const u4*)(stg + 12288 + off);
                if (mr < a.M && !(CMT_MLP_DIAG & 1)) {
                    pair_t* cr = (pair_t*)a.C + (int64_t)z * a.c_bstride + (int64_t)mr * a.ldc + 64 * q + 8 * ch;
                    pair_t* c2 = (pair_t*)a.C2 + (int64_t)z * a.c2_bstride + (int64_t)mr * a.ldc2 + 64 * q + 8 * ch;
                    *(u4*)cr = v0;
                    *(u4*)(cr + NOUT) = v1;
                    *(u4*)c2 = v2;
                    *(u4*)(c2 + NOUT) = v3;
                }
            }
        }
        raise_range_flag(a.range_flag, bad);
        return;
    }
    // ---- epilogue: out = acc + (b2 + R) (cmt_gemm's order), row lr, columns 32 ot + 8 g + 4 lh + 0..3
    if (m >= a.M) return;
    const char* Rrow = nullptr;
    if (a.R) {
        const int resz = a.r_dtype == CMT_F32 ? 4 : 2;
        Rrow = (const char*)a.R + ((int64_t)z * a.r_bstride + (int64_t)row * a.ldr) * resz;
    }
    const int cesz = a.c_dtype == CMT_F32 ? 4 : 2;
    char* Crow = (char*)a.C + ((int64_t)z * a.c_bstride + (int64_t)row * a.ldc) * cesz;
    typedef pair_t p4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = ot * 32 + 8 * g + 4 * lh;
            const f32x4 bv = *(const f32x4*)(a.b2 + n);
            f32x4 rv = {0.f, 0.f, 0.f, 0.f};
            if (Rrow) {
                if (a.r_dtype == CMT_F32) {
                    rv = *(const f32x4*)((const float*)Rrow + n);
                } else {
                    const p4 h = *(const p4*)((const pair_t*)Rrow + n);
                    const p4 l = *(const p4*)((const pair_t*)Rrow + NOUT + n);
#pragma unroll
                    for (int e = 0; e < 4; ++e) rv[e] = (float)h[e] + (float)l[e];
                }
            }
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = oacc[ot][4 * g + e] + (bv[e] + rv[e]);
            if (a.c_dtype == CMT_F32) *(f32x4*)((float*)Crow + n) = v;
            else store_pair4((pair_t*)Crow, NOUT, n, v);
        }
}

}  // namespace

extern "C" int64_t cmt_mlp2_args_size(void) { return (int64_t)sizeof(cmt_mlp2_args); }

extern "C" int cmt_mlp2_x3(const cmt_mlp2_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_mlp2_x3: null args");
    const cmt_mlp2_args& a = *ap;
    CMT_REQUIRE(a.M > 0 && a.batch > 0, "cmt_mlp2_x3: empty problem");
    CMT_REQUIRE(a.N == NOUT, "cmt_mlp2_x3: the output width must be 256");
    CMT_REQUIRE(a.K > 0 && a.K % 16 == 0 && a.K <= 192, "cmt_mlp2_x3: K must be a multiple of 16, at most 192");
    CMT_REQUIRE(a.Hd > 0 && a.Hd % 32 == 0 && a.Hd <= MAX_HD,
                "cmt_mlp2_x3: the hidden width must be a multiple of 32, at most 2048");
    CMT_REQUIRE((a.A || a.geo_i2l) && a.W1p && a.W2p && a.b1 && a.b2 && a.C, "cmt_mlp2_x3: null pointer");
    CMT_REQUIRE(a.geo_i2l || (a.lda >= 2 * a.K && a.lda % 8 == 0 && a.a_bstride % 8 == 0),
                "cmt_mlp2_x3: A pair rows need lda >= 2K, 16-byte aligned");
    CMT_REQUIRE(a.c_dtype == CMT_F32 || a.c_dtype == CMT_F16P, "cmt_mlp2_x3: C must be fp32 or an f16 pair");
    CMT_REQUIRE(a.c_dtype == CMT_F32 ? a.ldc >= NOUT && a.ldc % 4 == 0 && a.c_bstride % 4 == 0
                                     : a.ldc >= 2 * NOUT && a.ldc % 4 == 0 && a.c_bstride % 4 == 0,
                "cmt_mlp2_x3: bad C row stride");
    CMT_REQUIRE(a.R == nullptr || ((a.r_dtype == CMT_F32 && a.ldr >= NOUT) ||
                                   (a.r_dtype == CMT_F16P && a.ldr >= 2 * NOUT)) && a.ldr % 4 == 0 &&
                                      a.r_bstride % 4 == 0,
                "cmt_mlp2_x3: R must be fp32 or f16-pair rows of 256");
    CMT_REQUIRE(((uintptr_t)a.A | (uintptr_t)a.W1p | (uintptr_t)a.W2p) % 16 == 0 && (uintptr_t)a.b1 % 16 == 0 &&
                    (uintptr_t)a.b2 % 16 == 0,
                "cmt_mlp2_x3: A / packs / biases must be 16-byte aligned");
    const dim3 grid((unsigned)cdiv(a.M, MROWS), (unsigned)a.batch);
    hipStream_t s = (hipStream_t)stream;
    if (a.geo_i2l || a.rx) {
        CMT_REQUIRE(a.geo_i2l && a.rx && a.C2 && a.K == 192 && a.geo_D * 3 == a.K && a.geo_h > 0 && a.geo_w > 0 &&
                        a.M % (a.geo_h * a.geo_w) == 0 && a.c_dtype == CMT_F16P && a.R == nullptr &&
                        a.ldc2 >= 2 * NOUT && a.ldc2 % 4 == 0 && a.c2_bstride % 4 == 0 &&
                        (uintptr_t)a.C2 % 8 == 0,
                    "cmt_mlp2_x3: the fused camera-row form takes geo_i2l, rx and C2 together, K = 3 geo_D = 192, "
                    "M a multiple of geo_h * geo_w, a pair C and no R");
        mlp2_x3_kernel<12, 2, true, true><<<grid, 64 * MW, 0, s>>>(a);
        return cmt_check_launch("cmt_mlp2_x3");
    }
    switch (a.K / 16) {
#define MLP_K(KS) case KS: mlp2_x3_kernel<KS><<<grid, 64 * MW, 0, s>>>(a); break;
        MLP_K(1) MLP_K(2) MLP_K(3) MLP_K(4) MLP_K(5) MLP_K(6) MLP_K(7) MLP_K(8) MLP_K(9) MLP_K(10) MLP_K(11)
        MLP_K(12)
#undef MLP_K
        default: return cmt_fail(CMT_ENOTSUP, "cmt_mlp2_x3: unsupported K");
    }
    return cmt_check_launch("cmt_mlp2_x3");
}
