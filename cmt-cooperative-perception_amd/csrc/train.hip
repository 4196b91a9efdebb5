// Training-path kernels of the CMT / CMTCoop head for gfx950 (SURVEY.md
// 8(f) next #2; reference training step: cmt_head.py:339-415 DN queries,
// 556-903 losses, 68-81 GroupLayerNorm1d backward; torch autograd + mmcv
// optimizer hook for the rest).  Exact-f32 throughout (the reference trains
// the head in fp32: custom_fp16 keeps pts_bbox_head fp32):
//
//   cmt_gemm_f32_ex      general-stride GEMM on v_mfma_f32_32x32x2_f32 (any
//                        operand transposed, batched, split-K by f32 atomics):
//                        every Linear forward / dX / dW of the training step
//   cmt_ln_train_fwd/bwd row LayerNorm (C = 64 / 256) with saved mean/rstd,
//                        dW / dB sums; C = 64 with per-row-group weights is
//                        the task heads' GroupLayerNorm1d (eps 1e-6)
//   cmt_bn_relu_train    BatchNorm2d (batch statistics) + ReLU on NHWC rows,
//                        running-stat update; and its backward
//   cmt_im2col3x3        the shared_conv input gather for the weight gradient
//   cmt_det_loss         FocalLoss (sigmoid) + L1Loss values and input grads
//   cmt_match_cost       FocalLossCost + BBox3DL1Cost matrix of the Hungarian
//                        assigner (hungarian_assigner_3d.py:68-156)
//   cmt_adamw_step       torch AdamW step over one flat parameter buffer with
//                        clip_grad_norm_ (mmcv OptimizerHook grad_clip)
//   cmt_sumsq            partial sums of squares (the clip's global norm)
#include "cmt_common.h"

namespace {

constexpr int TBK = 32;     // k-step
constexpr int TLD = 36;     // padded LDS row (floats)
constexpr int TNT = 256;

// k-contiguous, row(m/n)-contiguous, scalar; OP_IM: the implicit im2col of a 3x3 / pad 1 conv on
// NHWC rows (bf16x3 GEMM only): element (n, k) = X[token k shifted by tap n / Cin][channel n % Cin]
enum { OP_KC = 0, OP_MC = 1, OP_SC = 2, OP_IM = 3 };

// OP_IM's geometry: H x W images of Cin channels, rows (img * H + y) * W + x
struct X3Conv {
    int H, W, Cin;
};

// Stage a 64-row x 32-k tile of X (rows r0.., k0..) into LDS [row][TLD]:
// element (r, k) at X[r * s_r + k * s_k].
template <int MODE>
__device__ __forceinline__ void stage_tile(float* __restrict__ lds, const float* __restrict__ X, int64_t s_r,
                                           int64_t s_k, int rows, int K, int r0, int k0, int tid) {
    if (MODE == OP_KC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = tid + TNT * i;
            const int r = idx >> 3, c = (idx & 7) * 4;
            const int gr = r0 + r, gk = k0 + c;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (gr < rows) {
                const float* p = X + (int64_t)gr * s_r + gk;
                if (gk + 3 < K) v = *(const f32x4*)p;
                else
                    for (int j = 0; j < 4; ++j) v[j] = gk + j < K ? p[j] : 0.f;
            }
            *(f32x4*)(lds + r * TLD + c) = v;
        }
    } else if (MODE == OP_MC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = tid + TNT * i;
            const int k = idx >> 4, r = (idx & 15) * 4;
            const int gr = r0 + r, gk = k0 + k;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (gk < K) {
                const float* p = X + (int64_t)gk * s_k + gr;
                if (gr + 3 < rows) v = *(const f32x4*)p;
                else
                    for (int j = 0; j < 4; ++j) v[j] = gr + j < rows ? p[j] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) lds[(r + j) * TLD + k] = v[j];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int idx = tid + TNT * i;
            const int r = idx >> 5, k = idx & 31;
            const int gr = r0 + r, gk = k0 + k;
            lds[r * TLD + k] = (gr < rows && gk < K) ? X[(int64_t)gr * s_r + (int64_t)gk * s_k] : 0.f;
        }
    }
}

template <int AM, int BM>
__global__ __launch_bounds__(TNT) void gemm_ex_kernel(cmt_gemm_ex_args a, int kchunk) {
    __shared__ __attribute__((aligned(16))) float As[64 * TLD];
    __shared__ __attribute__((aligned(16))) float Bs[64 * TLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
    const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int z = blockIdx.z / a.ksplit, ks = blockIdx.z - z * a.ksplit;
    const float* A = a.A + (int64_t)z * a.a_bs;
    const float* B = a.B + (int64_t)z * a.b_bs;
    const int kb = ks * kchunk, ke = min(a.K, kb + kchunk);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int k0 = kb; k0 < ke; k0 += TBK) {
        __syncthreads();
        stage_tile<AM>(As, A, a.a_sm, a.a_sk, a.M, ke, m0, k0, tid);
        stage_tile<BM>(Bs, B, a.b_sn, a.b_sk, a.N, ke, n0, k0, tid);
        __syncthreads();
        const float* ar = As + (wm * 32 + lr) * TLD + 16 * lh;
        const float* br = Bs + (wn * 32 + lr) * TLD + 16 * lh;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const f32x4 av = *(const f32x4*)(ar + 4 * c);
            const f32x4 bv = *(const f32x4*)(br + 4 * c);
#pragma unroll
            for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv[t], acc, 0, 0, 0);
        }
    }
    float* C = a.C + (int64_t)z * a.c_bs;
    const int col = n0 + wn * 32 + lr;
    if (col >= a.N) return;
    const float bias = (a.bias && ks == 0) ? a.bias[(int64_t)z * a.bias_bs + col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= a.M) continue;
        float* c = C + (int64_t)row * a.ldc + col;
        const float v = a.alpha * acc[r] + bias;
        if (a.ksplit > 1) atomicAdd(c, v);
        else *c = a.beta != 0.f ? v + a.beta * *c : v;
    }
}

// ---------------------------------------------------------------------------
// The same general-stride GEMM on bf16 MFMA in three passes (cmt_gemm_bf16x3_ex):
// every fp32 operand is split x = hi + lo, both bf16 (RNE) -- bf16 keeps the
// fp32 exponent range, so the small gradients of a backward pass stay exact to
// ~2^-17 where an f16 pair would flush them -- and each 16-deep k step runs
// lo*hi + hi*lo + hi*hi on v_mfma_f32_32x32x16_bf16, fp32 accumulate: ~2^-16
// relative per product (the dropped lo*lo term and the pair's representation),
// at 3 x 32 cycles per 16 k against 8 x 64 for the f32 MFMA (5.3x the rate).
// Tiles 64 x 64 x 32 as gemm_ex_kernel, staged through registers (any operand
// stride) into bf16 LDS images, hi and lo planes: [row][32 k] (64-byte rows, 16-byte
// chunks XOR-swizzled by (row >> 2) & 3) for k-contiguous and scalar operands,
// [32 k][row] for row-contiguous ones (x3_timg below).
// ---------------------------------------------------------------------------
constexpr int X3RB = 64;   // bytes per staged row (32 k of bf16)

__device__ __forceinline__ int x3_off(int row, int k) {
    return row * X3RB + ((((k >> 3) ^ ((row >> 2) & 3))) << 4) + (k & 7) * 2;
}
// Row-contiguous operands (OP_MC, OP_IM: four consecutive rows per fetched vector) are staged
// TRANSPOSED, [k][row] -- two 32-row halves of 32 k-rows x 64 bytes, 16-byte chunks XOR-swizzled by
// (k >> 2) & 3 -- so each fetched vector leaves as one 8-byte LDS write per plane (the [row][k]
// image took four conflicted 2-byte writes), and the MFMA operand comes back through
// ds_read_b64_tr_b16.  Both images hand lane (lr, lh) of a 16-deep k slice the k order
// 4 lh + 0..3, 8 + 4 lh + 0..3 (the transposed read's), so the two operands agree.  Conv-shaped
// weight gradient 950 -> 611 us, K/V-shaped 77 -> 61 us (profiles/r5_experiments.txt r5af).
template <int MODE>
constexpr bool x3_timg() {
    return MODE == 1 || MODE == 3;   // OP_MC, OP_IM
}
__device__ __forceinline__ int x3_toff(int row, int k) {
    return ((row >> 5) << 11) + k * 64 + (((((row & 31) >> 3) ^ ((k >> 2) & 3))) << 4) + (row & 7) * 2;
}
// the 32x32x16 MFMA operand of rows [r0, r0 + 32) (lane row = r) and k slice 16 kk .. 16 kk + 15;
// PERM: the transposed read's k order (some operand of the product is transposed), else the
// natural 8 lh + 0..7 in one ds_read_b128
template <int MODE, bool PERM>
__device__ __forceinline__ bf16x8 x3_frag(const char* img, int r0, int r, int kk, int lane) {
    const int lh = lane >> 5;
    if constexpr (x3_timg<MODE>()) {
        const char* base = img + ((r0 >> 5) << 11);
        const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
        const int c = 2 * (g & 1) + (pp >> 1);
        const int ka = 16 * kk + 4 * lh + qq, kb = ka + 8;
        const char* pa = base + ka * 64 + ((c ^ ((ka >> 2) & 3)) << 4) + 8 * (pp & 1);
        const char* pb = base + kb * 64 + ((c ^ ((kb >> 2) & 3)) << 4) + 8 * (pp & 1);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((CMT_LDS s16v4_lds*)pa);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((CMT_LDS s16v4_lds*)pb);
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    } else if constexpr (PERM) {
        const s16x4 lo = *(const s16x4*)(img + x3_off(r, 16 * kk + 4 * lh));
        const s16x4 hi = *(const s16x4*)(img + x3_off(r, 16 * kk + 8 + 4 * lh));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    } else {
        return *(const bf16x8*)(img + x3_off(r, 16 * kk + 8 * lh));
    }
}

__device__ __forceinline__ void split_bf16(float x, bf16_t& hi, bf16_t& lo) {
    hi = (bf16_t)x;
    lo = (bf16_t)(x - (float)hi);
}

// An R-row x 32-k fp32 tile (element (r, k) at X[r * s_r + k * s_k]) staged by NT threads moves in
// two steps so the next tile's global loads are in flight while the current one is multiplied:
// fetch_x3 loads this thread's R * 32 / NT elements into registers, put_x3 splits them into the bf16
// hi / lo LDS images.  Row-contiguous modes: R / 4 threads per k row, each four consecutive rows.
template <int MODE, int R, int NT>
__device__ __forceinline__ void fetch_x3(float (&v)[R * 32 / NT], const float* __restrict__ X, int64_t s_r, int64_t s_k,
                                         int rows, int K, int r0, int k0, int tid, const X3Conv& cv = X3Conv{}) {
    constexpr int TPR = R / 4, VI = R * 8 / NT;
    if (MODE == OP_IM) {
        // OP_MC's thread layout: 4 consecutive n (channels of one tap, Cin % 4 == 0) at one token
        const int hw = cv.H * cv.W;
#pragma unroll
        for (int i = 0; i < VI; ++i) {
            const int idx = tid + NT * i;
            const int k = idx / TPR, r = (idx % TPR) * 4;
            const int gr = r0 + r, gk = k0 + k;
            f32x4 t = {0.f, 0.f, 0.f, 0.f};
            if (gk < K && gr < rows) {
                const int tap = gr / cv.Cin, c = gr - tap * cv.Cin;
                const int img = gk / hw, pix = gk - img * hw;
                const int py = pix / cv.W;
                const int y = py + tap / 3 - 1, x = pix - py * cv.W + tap % 3 - 1;
                if (y >= 0 && y < cv.H && x >= 0 && x < cv.W)
                    t = *(const f32x4*)(X + (((int64_t)img * cv.H + y) * cv.W + x) * cv.Cin + c);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = t[j];
        }
    } else if (MODE == OP_KC) {
#pragma unroll
        for (int i = 0; i < VI; ++i) {
            const int idx = tid + NT * i;
            const int r = idx >> 3, c = (idx & 7) * 4;
            const int gr = r0 + r, gk = k0 + c;
            f32x4 t = {0.f, 0.f, 0.f, 0.f};
            if (gr < rows) {
                const float* p = X + (int64_t)gr * s_r + gk;
                if (gk + 3 < K) t = *(const f32x4*)p;
                else
                    for (int j = 0; j < 4; ++j) t[j] = gk + j < K ? p[j] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = t[j];
        }
    } else if (MODE == OP_MC) {
#pragma unroll
        for (int i = 0; i < VI; ++i) {
            const int idx = tid + NT * i;
            const int k = idx / TPR, r = (idx % TPR) * 4;
            const int gr = r0 + r, gk = k0 + k;
            f32x4 t = {0.f, 0.f, 0.f, 0.f};
            if (gk < K) {
                const float* p = X + (int64_t)gk * s_k + gr;
                if (gr + 3 < rows) t = *(const f32x4*)p;
                else
                    for (int j = 0; j < 4; ++j) t[j] = gr + j < rows ? p[j] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = t[j];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4 * VI; ++i) {
            const int idx = tid + NT * i;
            const int r = idx >> 5, k = idx & 31;
            const int gr = r0 + r, gk = k0 + k;
            v[i] = (gr < rows && gk < K) ? X[(int64_t)gr * s_r + (int64_t)gk * s_k] : 0.f;
        }
    }
}

template <int MODE, int R, int NT>
__device__ __forceinline__ void put_x3(char* __restrict__ hi, char* __restrict__ lo, const float (&v)[R * 32 / NT], int tid) {
    typedef bf16_t b4 __attribute__((ext_vector_type(4)));
    constexpr int TPR = R / 4, VI = R * 8 / NT;
    if (MODE == OP_KC) {
#pragma unroll
        for (int i = 0; i < VI; ++i) {
            const int idx = tid + NT * i;
            const int r = idx >> 3, c = (idx & 7) * 4;
            b4 h, l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bf16_t hj, lj;
                split_bf16(v[4 * i + j], hj, lj);
                h[j] = hj;
                l[j] = lj;
            }
            *(b4*)(hi + x3_off(r, c)) = h;
            *(b4*)(lo + x3_off(r, c)) = l;
        }
    } else if (x3_timg<MODE>()) {
#pragma unroll
        for (int i = 0; i < VI; ++i) {
            const int idx = tid + NT * i;
            const int k = idx / TPR, r = (idx % TPR) * 4;
            b4 h, l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bf16_t hj, lj;
                split_bf16(v[4 * i + j], hj, lj);
                h[j] = hj;
                l[j] = lj;
            }
            *(b4*)(hi + x3_toff(r, k)) = h;
            *(b4*)(lo + x3_toff(r, k)) = l;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4 * VI; ++i) {
            const int idx = tid + NT * i;
            const int r = idx >> 5, k = idx & 31;
            bf16_t h, l;
            split_bf16(v[i], h, l);
            *(bf16_t*)(hi + x3_off(r, k)) = h;
            *(bf16_t*)(lo + x3_off(r, k)) = l;
        }
    }
}

// Row (m) of each of fetch_x3's elements within the R-row tile.
template <int MODE, int R, int NT>
__device__ __forceinline__ int x3_row(int e, int tid) {
    if (MODE == OP_KC) return ((tid + NT * (e >> 2)) >> 3);
    if (MODE == OP_MC || MODE == OP_IM) return ((tid + NT * (e >> 2)) % (R / 4)) * 4 + (e & 3);
    return (tid + NT * e) >> 5;
}

// Workgroups are dealt to the 8 XCDs round-robin by linear id; renumber them so each XCD runs a
// contiguous range of tiles (the column tiles of one row block, the tiles of one K chunk) and
// reads their shared operand rows through its own L2 once.
__device__ __forceinline__ void xcd_tile(int& bx, int& by, int& bz) {
    const int nx = gridDim.x, ny = gridDim.y, total = nx * ny * gridDim.z;
    int b = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    if ((total & 7) == 0) b = (b & 7) * (total >> 3) + (b >> 3);
    bx = b % nx;
    by = (b / nx) % ny;
    bz = b / (nx * ny);
}

// T = 1: 64 x 64 tiles, each wave one 32 x 32 accumulator; T = 2: 128 x 128 tiles, each wave 2 x 2
// of them -- 4x the MFMAs per staged k-step for 2x the loads and splits (the long-K weight gradients
// and the 44 400-row K/V products, gemm_ex_launch)
template <int AM, int BM, int T>
__global__ __launch_bounds__(TNT) void gemm_ex3_kernel(cmt_gemm_ex_args a, int kchunk, X3Conv cv) {
    constexpr int R = 64 * T;   // tile rows and columns
    __shared__ __attribute__((aligned(16))) char As[2][2][R * X3RB];   // [buffer][hi, lo]
    __shared__ __attribute__((aligned(16))) char Bs[2][2][R * X3RB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
    int bx, by, bz;
    xcd_tile(bx, by, bz);
    const int n0 = bx * R, m0 = by * R;
    const int z = bz / a.ksplit, ks = bz - z * a.ksplit;
    const float* A = a.A + (int64_t)z * a.a_bs;
    const float* B = a.B + (int64_t)z * a.b_bs;
    const int kb = ks * kchunk, ke = min(a.K, kb + kchunk);
    f32x16 acc[T][T];
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j < T; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int ar0 = wm * 32 * T, br0 = wn * 32 * T;   // the wave's first A / B tile row
    float va[8 * T], vb[8 * T];
    // a_rowsum: the first column tile also sums its A elements (fp32, before the split) per row
    const bool rowsum = a.a_rowsum != nullptr && bx == 0;
    float rs[8 * T];
#pragma unroll
    for (int e = 0; e < 8 * T; ++e) rs[e] = 0.f;
    fetch_x3<AM, R, TNT>(va, A, a.a_sm, a.a_sk, a.M, ke, m0, kb, tid);
    fetch_x3<BM, R, TNT>(vb, B, a.b_sn, a.b_sk, a.N, ke, n0, kb, tid, cv);
    int buf = 0;
    for (int k0 = kb; k0 < ke; k0 += TBK, buf ^= 1) {
        if (rowsum) {
#pragma unroll
            for (int e = 0; e < 8 * T; ++e) rs[e] += va[e];
        }
        // one barrier per step: buffer buf was last read two steps ago, before the previous barrier
        put_x3<AM, R, TNT>(As[buf][0], As[buf][1], va, tid);
        put_x3<BM, R, TNT>(Bs[buf][0], Bs[buf][1], vb, tid);
        __syncthreads();
        if (k0 + TBK < ke) {
            fetch_x3<AM, R, TNT>(va, A, a.a_sm, a.a_sk, a.M, ke, m0, k0 + TBK, tid);
            fetch_x3<BM, R, TNT>(vb, B, a.b_sn, a.b_sk, a.N, ke, n0, k0 + TBK, tid, cv);
        }
        constexpr bool perm = x3_timg<AM>() || x3_timg<BM>();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 ah[T], al[T], bh[T], bl[T];
#pragma unroll
            for (int i = 0; i < T; ++i) {
                ah[i] = x3_frag<AM, perm>(As[buf][0], ar0 + 32 * i, ar0 + 32 * i + lr, kk, lane);
                al[i] = x3_frag<AM, perm>(As[buf][1], ar0 + 32 * i, ar0 + 32 * i + lr, kk, lane);
                bh[i] = x3_frag<BM, perm>(Bs[buf][0], br0 + 32 * i, br0 + 32 * i + lr, kk, lane);
                bl[i] = x3_frag<BM, perm>(Bs[buf][1], br0 + 32 * i, br0 + 32 * i + lr, kk, lane);
            }
#pragma unroll
            for (int i = 0; i < T; ++i)
#pragma unroll
                for (int j = 0; j < T; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
    }
    if (rowsum) {   // uniform per workgroup: per-row partials through LDS, one atomic per row
        float* red = (float*)As[0][0];
        __syncthreads();
        if (tid < R) red[tid] = 0.f;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8 * T; ++e) atomicAdd(red + x3_row<AM, R, TNT>(e, tid), rs[e]);
        __syncthreads();
        if (tid < R && m0 + tid < a.M) atomicAdd(a.a_rowsum + (int64_t)z * a.M + m0 + tid, red[tid]);
    }
    float* C = a.C + (int64_t)z * a.c_bs;
#pragma unroll
    for (int j = 0; j < T; ++j) {
        const int col = n0 + br0 + 32 * j + lr;
        if (col >= a.N) continue;
        const float bias = (a.bias && ks == 0) ? a.bias[(int64_t)z * a.bias_bs + col] : 0.f;
#pragma unroll
        for (int i = 0; i < T; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + ar0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (row >= a.M) continue;
                float* c = C + (int64_t)row * a.ldc + col;
                const float v = a.alpha * acc[i][j][r] + bias;
                if (a.ksplit > 1) atomicAdd(c, v);
                else *c = a.beta != 0.f ? v + a.beta * *c : v;
            }
    }
}

// Small products (fewer than 256 workgroups of 64 x 64 tiles, >= 4 k-steps each): a workgroup's
// chain of dependent k-steps is its time (each step's MFMAs far shorter than its loads' latency).
// Here the 4 waves split the tile's k-steps round-robin, each staging its own steps through a
// private LDS slice (no workgroup barrier in the loop) into a full 64 x 64 partial tile, then the
// partials are summed through LDS: a quarter of the chain per workgroup.
template <int AM, int BM>
__global__ __launch_bounds__(TNT) void gemm_ex3_kw_kernel(cmt_gemm_ex_args a, int kchunk, X3Conv cv) {
    constexpr int R = 64, NT = 64, EPT = R * 32 / NT;   // 32 staged elements per lane and operand
    constexpr int PLANE = R * X3RB;                      // one bf16 plane image: 4 KB
    // [wave][A hi, A lo, B hi, B lo] staging; after the k loop: [wave][tile (i, j)][lane][16] partials
    __shared__ __attribute__((aligned(16))) char lds[4 * 4 * PLANE];
    __shared__ float red[R];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    int bx, by, bz;
    xcd_tile(bx, by, bz);
    const int n0 = bx * R, m0 = by * R;
    const int z = bz / a.ksplit, ks = bz - z * a.ksplit;
    const float* A = a.A + (int64_t)z * a.a_bs;
    const float* B = a.B + (int64_t)z * a.b_bs;
    const int kb = ks * kchunk, ke = min(a.K, kb + kchunk);
    const int nsteps = (ke - kb + TBK - 1) / TBK;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const bool rowsum = a.a_rowsum != nullptr && bx == 0;
    float rs[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) rs[e] = 0.f;
    char* const my = lds + wave * 4 * PLANE;
    float va[EPT], vb[EPT];
    if (wave < nsteps) {
        fetch_x3<AM, R, NT>(va, A, a.a_sm, a.a_sk, a.M, ke, m0, kb + wave * TBK, lane);
        fetch_x3<BM, R, NT>(vb, B, a.b_sn, a.b_sk, a.N, ke, n0, kb + wave * TBK, lane, cv);
    }
    constexpr bool perm = x3_timg<AM>() || x3_timg<BM>();
    for (int s = wave; s < nsteps; s += 4) {
        if (rowsum) {
#pragma unroll
            for (int e = 0; e < EPT; ++e) rs[e] += va[e];
        }
        put_x3<AM, R, NT>(my, my + PLANE, va, lane);
        put_x3<BM, R, NT>(my + 2 * PLANE, my + 3 * PLANE, vb, lane);
        // the wave reads what its own lanes wrote: LDS operations of a wave complete in order, the
        // fence keeps the compiler from moving the reads above the writes
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (s + 4 < nsteps) {
            fetch_x3<AM, R, NT>(va, A, a.a_sm, a.a_sk, a.M, ke, m0, kb + (s + 4) * TBK, lane);
            fetch_x3<BM, R, NT>(vb, B, a.b_sn, a.b_sk, a.N, ke, n0, kb + (s + 4) * TBK, lane, cv);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ah[i] = x3_frag<AM, perm>(my, 32 * i, 32 * i + lr, kk, lane);
                al[i] = x3_frag<AM, perm>(my + PLANE, 32 * i, 32 * i + lr, kk, lane);
                bh[i] = x3_frag<BM, perm>(my + 2 * PLANE, 32 * i, 32 * i + lr, kk, lane);
                bl[i] = x3_frag<BM, perm>(my + 3 * PLANE, 32 * i, 32 * i + lr, kk, lane);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
        // this step's fragment reads complete before the next step's writes to the same slice
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (rowsum) {
        if (tid < R) red[tid] = 0.f;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < EPT; ++e) atomicAdd(red + x3_row<AM, R, NT>(e, lane), rs[e]);
    }
    __syncthreads();   // every wave is past its staging: the slices take the partial tiles
    float* part = (float*)lds;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(f32x4*)(part + (((wave * 4 + 2 * i + j) * 64 + lane) * 16 + 4 * q)) =
                    f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
    __syncthreads();
    if (rowsum && tid < R && m0 + tid < a.M) atomicAdd(a.a_rowsum + (int64_t)z * a.M + m0 + tid, red[tid]);
    // wave w sums tile (w >> 1, w & 1) of the four partials, in wave order
    const int ti = wave >> 1, tj = wave & 1;
    f32x16 sum;
#pragma unroll
    for (int r = 0; r < 16; ++r) sum[r] = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 v = *(const f32x4*)(part + (((w * 4 + 2 * ti + tj) * 64 + lane) * 16 + 4 * q));
            sum[4 * q] += v[0]; sum[4 * q + 1] += v[1]; sum[4 * q + 2] += v[2]; sum[4 * q + 3] += v[3];
        }
    float* C = a.C + (int64_t)z * a.c_bs;
    const int col = n0 + 32 * tj + lr;
    if (col >= a.N) return;
    const float bias = (a.bias && ks == 0) ? a.bias[(int64_t)z * a.bias_bs + col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = m0 + 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= a.M) continue;
        float* c = C + (int64_t)row * a.ldc + col;
        const float v = a.alpha * sum[r] + bias;
        if (a.ksplit > 1) atomicAdd(c, v);
        else *c = a.beta != 0.f ? v + a.beta * *c : v;
    }
}

int op_mode(int64_t s_row, int64_t s_k, const float* p) {
    const bool al = ((uintptr_t)p & 15) == 0;
    if (s_k == 1 && s_row % 4 == 0 && al) return OP_KC;
    if (s_row == 1 && s_k % 4 == 0 && al) return OP_MC;
    return OP_SC;
}

// ---------------------------------------------------------------------------
// Row LayerNorm, C = 64 or 256: one wave per row, C/64 elements per lane.
// ---------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void ln_fwd_kernel(cmt_ln_train_args a) {
    constexpr int E = C / 64;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int g = a.rows_per_wset > 0 ? row / a.rows_per_wset : 0;
    const float* x = a.X + (int64_t)row * a.ldx;
    float v[E], s = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) { v[e] = x[lane + 64 * e]; s += v[e]; }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / C;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) { const float d = v[e] - mean; q += d * d; }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o);
    const float rstd = 1.f / sqrtf(q / C + a.eps);
    float* y = a.Y + (int64_t)row * a.ldy;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int c = lane + 64 * e;
        y[c] = (v[e] - mean) * rstd * a.W[g * C + c] + a.B[g * C + c];
    }
    if (lane == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
}

// dx = rstd * (gw - mean(gw) - xhat * mean(gw * xhat)), gw = dy * w;
// dW[g] += sum dy * xhat, dB[g] += sum dy over the rows of weight set g.
template <int C>
__global__ __launch_bounds__(256) void ln_bwd_kernel(cmt_ln_train_args a) {
    constexpr int E = C / 64;
    const int lane = threadIdx.x & 63;
    const int w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    float dw[E], db[E];
    int cur_g = -1;
    auto flush = [&]() {
        if (cur_g < 0) return;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (a.dW) atomicAdd(a.dW + cur_g * C + lane + 64 * e, dw[e]);
            if (a.dB) atomicAdd(a.dB + cur_g * C + lane + 64 * e, db[e]);
        }
    };
    if (a.rows_per_wset <= 0) {
        // one weight set (nn.LayerNorm): the block's 4 waves sum their dW / dB partials through LDS
        // and the block issues one atomic per column (one per row and column made the ~1 100-row
        // decoder LayerNorms ~30 us of atomic contention on 512 addresses)
        __shared__ float red[2][4][C];
#pragma unroll
        for (int e = 0; e < E; ++e) dw[e] = db[e] = 0.f;
        for (int row = w0; row < a.rows; row += nw) {
            const float* x = a.X + (int64_t)row * a.ldx;
            const float* dy = a.dY + (int64_t)row * a.ldy;
            const float mean = a.mean[row], rstd = a.rstd[row];
            float xh[E], gw[E], s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int c = lane + 64 * e;
                xh[e] = (x[c] - mean) * rstd;
                const float d = dy[c];
                gw[e] = d * a.W[c];
                s1 += gw[e];
                s2 += gw[e] * xh[e];
                dw[e] += d * xh[e];
                db[e] += d;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) { s1 += __shfl_xor(s1, o); s2 += __shfl_xor(s2, o); }
            s1 /= C;
            s2 /= C;
            float* dx = a.dX + (int64_t)row * a.lddx;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int c = lane + 64 * e;
                const float v = rstd * (gw[e] - s1 - xh[e] * s2);
                dx[c] = a.accumulate ? dx[c] + v : v;
            }
        }
        const int wv = threadIdx.x >> 6;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            red[0][wv][lane + 64 * e] = dw[e];
            red[1][wv][lane + 64 * e] = db[e];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 2 * C; i += 256) {
            const int which = i / C, c = i - which * C;
            const float v = red[which][0][c] + red[which][1][c] + red[which][2][c] + red[which][3][c];
            float* dst = which ? a.dB : a.dW;
            if (dst) atomicAdd(dst + c, v);
        }
        return;
    }
    for (int row = w0; row < a.rows; row += nw) {
        const int g = a.rows_per_wset > 0 ? row / a.rows_per_wset : 0;
        if (g != cur_g) {
            flush();
            cur_g = g;
#pragma unroll
            for (int e = 0; e < E; ++e) dw[e] = db[e] = 0.f;
        }
        const float* x = a.X + (int64_t)row * a.ldx;
        const float* dy = a.dY + (int64_t)row * a.ldy;
        const float mean = a.mean[row], rstd = a.rstd[row];
        float xh[E], gw[E], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int c = lane + 64 * e;
            xh[e] = (x[c] - mean) * rstd;
            const float d = dy[c];
            gw[e] = d * a.W[g * C + c];
            s1 += gw[e];
            s2 += gw[e] * xh[e];
            dw[e] += d * xh[e];
            db[e] += d;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) { s1 += __shfl_xor(s1, o); s2 += __shfl_xor(s2, o); }
        s1 /= C;
        s2 /= C;
        float* dx = a.dX + (int64_t)row * a.lddx;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int c = lane + 64 * e;
            const float v = rstd * (gw[e] - s1 - xh[e] * s2);
            dx[c] = a.accumulate ? dx[c] + v : v;
        }
    }
    flush();
}

// ---------------------------------------------------------------------------
// BatchNorm2d (training: batch statistics over all rows) + ReLU on [rows][C]
// NHWC rows.  Column sums are deterministic at any row count: each row block
// writes its partial sums to the workspace (no atomics), and bn_reduce_kernel
// adds the partials of every column in a fixed order (two passes: mean, then
// centred squares).  Row blocks of >= 64 rows, at most BN_MAXB of them.
// ---------------------------------------------------------------------------
constexpr int BN_MAXB = 512;
inline int bn_rows_per_block(int rows) { return max(64, (cdiv(rows, BN_MAXB) + 7) / 8 * 8); }

__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ X, int rows, int C,
                                                      const float* __restrict__ shift, float* __restrict__ part,
                                                      int squares, int rows_per_block) {
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= C) return;
    const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
    const float sh = shift ? shift[c] : 0.f;
    float s = 0.f;
#pragma unroll 8
    for (int r = r0; r < r1; ++r) {
        const float v = X[(int64_t)r * C + c] - sh;
        s += squares ? v * v : v;
    }
    part[(int64_t)blockIdx.x * C + c] = s;
}

// out[c] = scale * sum over blocks of part[blk][c], c < ncols (ldp floats per block): 8 groups of
// 32 columns per workgroup, group g adds blocks g, g + 8, ... in order, then the 8 group sums are
// added in order -- the same order on every run
__global__ __launch_bounds__(256) void bn_reduce_kernel(const float* __restrict__ part, int nblk, int ldp, int ncols,
                                                        float* __restrict__ out, float scale) {
    __shared__ float red[8][32];
    const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int c = blockIdx.x * 32 + cl;
    float s = 0.f;
    if (c < ncols) {
#pragma unroll 4
        for (int b = g; b < nblk; b += 8) s += part[(int64_t)b * ldp + c];
    }
    red[g][cl] = s;
    __syncthreads();
    if (g == 0 && c < ncols) {
        float t = red[0][cl];
#pragma unroll
        for (int j = 1; j < 8; ++j) t += red[j][cl];
        out[c] = t * scale;
    }
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(cmt_bn_args a, const float* __restrict__ sums) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= a.C) return;
    const float var = sums[c] / a.rows;   // biased (normalisation)
    a.mean_save[c] = sums[a.C + c];        // the shift = batch mean (first pass)
    a.rstd_save[c] = 1.f / sqrtf(var + a.eps);
    if (a.running_mean) {
        const float unb = a.rows > 1 ? var * a.rows / (a.rows - 1) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * sums[a.C + c];
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
    }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(cmt_bn_args a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)a.rows * a.C) return;
    const int c = (int)(i % a.C);
    const float v = (a.X[i] - a.mean_save[c]) * a.rstd_save[c] * a.W[c] + a.B[c];
    a.Y[i] = fmaxf(v, 0.f);
}

// backward: g = dY * (Y > 0); per row block part[blk][0:C] = sum g, part[blk][C:2C] = sum g * xhat
__global__ __launch_bounds__(256) void bn_bwd_sums_kernel(cmt_bn_args a, float* __restrict__ part, int rpb) {
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= a.C) return;
    const int r0 = blockIdx.x * rpb, r1 = min(a.rows, r0 + rpb);
    const float mu = a.mean_save[c], rs = a.rstd_save[c];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int r = r0; r < r1; ++r) {
        const int64_t i = (int64_t)r * a.C + c;
        const float g = a.Y[i] > 0.f ? a.dY[i] : 0.f;
        s1 += g;
        s2 += g * (a.X[i] - mu) * rs;
    }
    float* row = part + (int64_t)blockIdx.x * 2 * a.C;
    row[c] = s1;
    row[a.C + c] = s2;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(cmt_bn_args a, const float* __restrict__ sums) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)a.rows * a.C) return;
    const int c = (int)(i % a.C);
    const float g = a.Y[i] > 0.f ? a.dY[i] : 0.f;
    const float xh = (a.X[i] - a.mean_save[c]) * a.rstd_save[c];
    const float n = (float)a.rows;
    a.dX[i] = a.W[c] * a.rstd_save[c] / n * (n * g - sums[c] - xh * sums[a.C + c]);
}

__global__ __launch_bounds__(256) void bn_param_grads_kernel(cmt_bn_args a, const float* __restrict__ sums) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= a.C) return;
    if (a.dB) a.dB[c] = sums[c];
    if (a.dW) a.dW[c] = sums[a.C + c];
}

// ---------------------------------------------------------------------------
// im2col of a 3x3 / pad 1 convolution on NHWC rows: out[(img*H + y)*W + x][tap*C + c]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void im2col3x3_kernel(const float* __restrict__ X, int nimg, int H, int W, int C,
                                                        float* __restrict__ out) {
    const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    const int64_t total = (int64_t)nimg * H * W * 9 * C;
    if (i4 >= total) return;
    const int K = 9 * C;
    const int64_t row = i4 / K;
    const int k = (int)(i4 - row * K);
    const int tap = k / C, c = k - tap * C;
    const int img = (int)(row / (H * W));
    const int p = (int)(row - (int64_t)img * H * W);
    const int y = p / W + tap / 3 - 1, x = p % W + tap % 3 - 1;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (y >= 0 && y < H && x >= 0 && x < W) v = *(const f32x4*)(X + (((int64_t)img * H + y) * W + x) * C + c);
    *(f32x4*)(out + i4) = v;
}

// ---------------------------------------------------------------------------
// Detection losses (one workgroup, deterministic reduction order).
//  FocalLoss(use_sigmoid, gamma, alpha) over logits [R][ncls] with labels
//  (ncls = background) and per-row weights, sum / cls_avg * cls_weight;
//  L1Loss over boxes [Rb][10] with per-element weights, sum / box_avg * box_weight.
//  Writes loss values and d(loss)/d(input) (mmdet 2.28.2 FocalLoss / L1Loss).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float softplus(float x) { return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x)); }

__global__ __launch_bounds__(1024) void det_loss_kernel(cmt_det_loss_args a) {
    __shared__ float red[32];
    float lc = 0.f, lb = 0.f;
    const float g = a.gamma, al = a.alpha;
    const float cls_k = a.cls_weight / a.cls_avg, box_k = a.box_weight / a.box_avg;
    for (int i = threadIdx.x; i < a.R * a.ncls; i += blockDim.x) {
        const int r = i / a.ncls, c = i - r * a.ncls;
        const float x = a.logits[(int64_t)r * a.ld_logits + c];
        const float w = a.label_w ? a.label_w[r] : 1.f;
        const bool pos = a.labels[r] == c;
        const float p = 1.f / (1.f + expf(-x));
        float loss, grad;
        if (pos) {   // -alpha (1-p)^g log p
            const float omp = 1.f - p, pw = powf(omp, g), lp = -softplus(-x);
            loss = -al * pw * lp;
            grad = al * pw * (g * p * lp - omp);
        } else {     // -(1-alpha) p^g log(1-p)
            const float pw = powf(p, g), l1p = -softplus(x);
            loss = -(1.f - al) * pw * l1p;
            grad = (1.f - al) * pw * (p - g * (1.f - p) * l1p);
        }
        lc += loss * w;
        if (a.dlogits) a.dlogits[(int64_t)r * a.ld_logits + c] = grad * w * cls_k * a.gscale;
    }
    for (int i = threadIdx.x; i < a.Rb * 10; i += blockDim.x) {
        const int r = i / 10, c = i - r * 10;
        const float d = a.boxes[(int64_t)r * a.ld_boxes + c] - a.targets[r * 10 + c];
        const float w = a.box_w[r * 10 + c];
        lb += fabsf(d) * w;
        if (a.dboxes) a.dboxes[(int64_t)r * a.ld_boxes + c] = (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) * w * box_k * a.gscale;
    }
    // block reductions (fixed order)
    for (int pass = 0; pass < 2; ++pass) {
        float v = pass == 0 ? lc : lb;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
            a.out[pass] = s * (pass == 0 ? cls_k : box_k);
        }
    }
}

// cost[q][j] = w_cls * (pos(q, label_j) - neg(q, label_j)) + w_reg * sum_c |cw_c (box[q][c] - gt[j][c])|, c < 8
__global__ __launch_bounds__(256) void match_cost_kernel(cmt_match_cost_args a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.Nq * a.ngt) return;
    const int q = i / a.ngt, j = i - q * a.ngt;
    const float x = a.logits[(int64_t)q * a.ld_logits + a.gt_labels[j]];
    const float p = 1.f / (1.f + expf(-x));
    const float eps = 1e-12f;
    const float neg = -logf(1.f - p + eps) * (1.f - a.alpha) * powf(p, a.gamma);
    const float pos = -logf(p + eps) * a.alpha * powf(1.f - p, a.gamma);
    float l1 = 0.f;
    for (int c = 0; c < 8; ++c)
        l1 += fabsf(a.code_w[c] * a.boxes[(int64_t)q * a.ld_boxes + c] - a.code_w[c] * a.gt[j * 10 + c]);
    a.cost[i] = a.cls_weight * (pos - neg) + a.reg_weight * l1;
}

// ---------------------------------------------------------------------------
// AdamW over one flat buffer (torch.optim.AdamW, amsgrad off) with the
// clip_grad_norm_ coefficient read from the device sum of squares.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += x[i] * x[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

__global__ __launch_bounds__(256) void adamw_kernel(cmt_adamw_args a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    float coef = 1.f;
    if (a.max_norm > 0.f && a.sumsq) {
        const float norm = sqrtf(*a.sumsq);
        coef = fminf(1.f, a.max_norm / (norm + 1e-6f));
    }
    const float g = a.grad[i] * coef;
    float p = a.param[i];
    p *= 1.f - a.lr * a.weight_decay;
    const float m = a.beta1 * a.exp_avg[i] + (1.f - a.beta1) * g;
    const float v = a.beta2 * a.exp_avg_sq[i] + (1.f - a.beta2) * g * g;
    a.exp_avg[i] = m;
    a.exp_avg_sq[i] = v;
    const float bc1 = 1.f - powf(a.beta1, (float)a.step), bc2 = 1.f - powf(a.beta2, (float)a.step);
    const float denom = sqrtf(v) / sqrtf(bc2) + a.eps;
    a.param[i] = p - (a.lr / bc1) * m / denom;
}

}  // namespace

namespace {
// 128 x 128 tiles for long reductions (the weight gradients) and very large products, when they
// alone, or with the reduction split further, still give the chip >= 256 workgroups: a split-K launch
// (C accumulated, beta 1) may re-choose its split (chunks >= 256 k).  A 44 400 x 256 x 256 product
// keeps 64 x 64 tiles (694 big tiles are 1.4 rounds of two per CU: 49 vs 42 us, r5an).
bool x3_big_tiles(cmt_gemm_ex_args& a) {
    if (a.M < 128 || a.N < 128) return false;
    const int64_t tiles = (int64_t)cdiv(a.M, 128) * cdiv(a.N, 128) * a.batch;
    if (a.K < 1024 && tiles < 1536) return false;
    int ks = a.ksplit;
    if (ks > 1)
        while (tiles * ks < 512 && a.K / (2 * ks) >= 256) ks *= 2;
    if (tiles * ks < 256) return false;
    a.ksplit = ks;
    return true;
}

// the k-wave split (gemm_ex3_kw_kernel) for unsplit launches of < 256 64 x 64 tiles with >= 4 k-steps
// each: the decoder's forward / dX products 15.3-16.3 -> 12.1-13.3 us; a split-K weight gradient
// (16 tiles x 4 splits) measured 18.1 -> 24.9 us and keeps the one-wave-per-tile kernel (r5aq)
bool x3_kwave(const dim3& grid, int kchunk, int ksplit) {
    return ksplit == 1 && (int64_t)grid.x * grid.y * grid.z < 256 && kchunk >= 4 * TBK;
}

int gemm_ex_launch(const cmt_gemm_ex_args* ap, void* stream, bool x3) {
    CMT_REQUIRE(ap != nullptr, "cmt_gemm_f32_ex: null args");
    cmt_gemm_ex_args a = *ap;
    CMT_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.batch > 0, "cmt_gemm_f32_ex: empty problem");
    CMT_REQUIRE(a.A && a.B && a.C, "cmt_gemm_f32_ex: null pointer");
    if (a.ksplit < 1) a.ksplit = 1;
    CMT_REQUIRE(a.ksplit == 1 || a.beta == 1.f, "cmt_gemm_f32_ex: split-K accumulates (beta must be 1)");
    const int am = op_mode(a.a_sm, a.a_sk, a.A), bm = op_mode(a.b_sn, a.b_sk, a.B);
    const bool big = x3 && x3_big_tiles(a);
    int kchunk = cdiv(cdiv(a.K, a.ksplit), TBK) * TBK;
    a.ksplit = cdiv(a.K, kchunk);
    const int R = big ? 128 : 64;
    dim3 grid(cdiv(a.N, R), cdiv(a.M, R), a.batch * a.ksplit);
    // small products with >= 4 k-steps per tile: the waves of a workgroup split its k-steps
    const bool kw = x3 && !big && x3_kwave(grid, kchunk, a.ksplit);
    hipStream_t s = (hipStream_t)stream;
#define GX(AM, BM)                                                                      \
    do {                                                                                \
        if (big) gemm_ex3_kernel<AM, BM, 2><<<grid, TNT, 0, s>>>(a, kchunk, X3Conv{});  \
        else if (kw) gemm_ex3_kw_kernel<AM, BM><<<grid, TNT, 0, s>>>(a, kchunk, X3Conv{}); \
        else if (x3) gemm_ex3_kernel<AM, BM, 1><<<grid, TNT, 0, s>>>(a, kchunk, X3Conv{}); \
        else gemm_ex_kernel<AM, BM><<<grid, TNT, 0, s>>>(a, kchunk);                    \
    } while (0)
    switch (am * 3 + bm) {
        case 0: GX(0, 0); break; case 1: GX(0, 1); break; case 2: GX(0, 2); break;
        case 3: GX(1, 0); break; case 4: GX(1, 1); break; case 5: GX(1, 2); break;
        case 6: GX(2, 0); break; case 7: GX(2, 1); break; default: GX(2, 2); break;
    }
#undef GX
    return cmt_check_launch(x3 ? "cmt_gemm_bf16x3_ex" : "cmt_gemm_f32_ex");
}
}  // namespace

extern "C" int cmt_gemm_f32_ex(const cmt_gemm_ex_args* ap, void* stream) { return gemm_ex_launch(ap, stream, false); }
extern "C" int cmt_gemm_bf16x3_ex(const cmt_gemm_ex_args* ap, void* stream) { return gemm_ex_launch(ap, stream, true); }

extern "C" int cmt_linear_bwd_bf16x3_ex(const float* dY, const float* X, const float* W, float* dX, float* dW,
                                        float* dB, int M, int K, int N, int64_t ldx, int ksplit, int flags,
                                        void* stream) {
    CMT_REQUIRE(dY && X && W && M > 0 && K > 0 && N > 0 && ldx >= K, "cmt_linear_bwd_bf16x3: bad arguments");
    CMT_REQUIRE(dB == nullptr || dW != nullptr, "cmt_linear_bwd_bf16x3: dB comes with dW");
    CMT_REQUIRE((flags & ~CMT_LINEAR_BWD_ACCUMULATE) == 0, "cmt_linear_bwd_bf16x3: unknown flags");
    const bool acc = (flags & CMT_LINEAR_BWD_ACCUMULATE) != 0;
    hipStream_t s = (hipStream_t)stream;
    if (dX) {
        cmt_gemm_ex_args a{};
        a.M = M; a.N = K; a.K = N; a.batch = 1; a.alpha = 1.f; a.beta = 0.f; a.ksplit = 1;
        a.A = dY; a.a_sm = N; a.a_sk = 1;
        a.B = W; a.b_sn = 1; a.b_sk = K;
        a.C = dX; a.ldc = K;
        const int rc = gemm_ex_launch(&a, stream, true);
        if (rc != 0) return rc;
    }
    if (dW) {
        cmt_gemm_ex_args a{};
        a.M = N; a.N = K; a.K = M; a.batch = 1; a.alpha = 1.f;
        a.ksplit = ksplit < 1 ? 1 : ksplit;
        // accumulate (ABI 24): dW / dB already hold a sum to add to (a parameter's .grad): C read and
        // rewritten (unsplit) or f32 atomics (split), the row sums atomic -- no zero fill
        a.beta = acc || a.ksplit > 1 ? 1.f : 0.f;
        a.A = dY; a.a_sm = 1; a.a_sk = N;
        a.B = X; a.b_sn = 1; a.b_sk = ldx;
        a.C = dW; a.ldc = K;
        a.a_rowsum = dB;
        if (!acc && a.ksplit > 1)
            CMT_REQUIRE(hipMemsetAsync(dW, 0, (size_t)N * K * sizeof(float), s) == hipSuccess,
                        "cmt_linear_bwd_bf16x3: memset");
        if (!acc && dB) CMT_REQUIRE(hipMemsetAsync(dB, 0, (size_t)N * sizeof(float), s) == hipSuccess,
                                    "cmt_linear_bwd_bf16x3: memset");
        return gemm_ex_launch(&a, stream, true);
    }
    return 0;
}

extern "C" int cmt_linear_bwd_bf16x3(const float* dY, const float* X, const float* W, float* dX, float* dW, float* dB,
                                     int M, int K, int N, int64_t ldx, int ksplit, void* stream) {
    return cmt_linear_bwd_bf16x3_ex(dY, X, W, dX, dW, dB, M, K, N, ldx, ksplit, 0, stream);
}

// shared_conv's weight gradient as the bf16x3 GEMM dW[cout][n] = sum_r dY[r][cout] im2col(X)[r][n]
// with the im2col operand gathered inside the kernel (OP_IM): no [rows, 9 Cin] matrix
extern "C" int cmt_conv3x3_wgrad_bf16x3(const float* X, const float* dY, float* dW, int nimg, int H, int W, int Cin,
                                        int Cout, int ksplit, void* stream) {
    CMT_REQUIRE(X && dY && dW && nimg > 0 && H > 0 && W > 0 && Cout > 0, "cmt_conv3x3_wgrad_bf16x3: bad arguments");
    CMT_REQUIRE(Cin > 0 && Cin % 4 == 0 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)dY & 15) == 0 && Cout % 4 == 0,
                "cmt_conv3x3_wgrad_bf16x3: Cin and Cout multiples of 4, 16-byte aligned X / dY");
    const int64_t rows = (int64_t)nimg * H * W;
    CMT_REQUIRE(rows < (int64_t)1 << 31, "cmt_conv3x3_wgrad_bf16x3: too many rows");
    cmt_gemm_ex_args a{};
    a.M = Cout; a.N = 9 * Cin; a.K = (int)rows; a.batch = 1;
    a.alpha = 1.f; a.beta = ksplit > 1 ? 1.f : 0.f;
    a.A = dY; a.a_sm = 1; a.a_sk = Cout;    // A(m, k) = dY[k][m]: OP_MC
    a.B = X;                                // B(n, k): the implicit im2col
    a.C = dW; a.ldc = 9 * Cin;
    a.ksplit = ksplit < 1 ? 1 : ksplit;
    const bool big = x3_big_tiles(a);
    int kchunk = cdiv(cdiv(a.K, a.ksplit), TBK) * TBK;
    a.ksplit = cdiv(a.K, kchunk);
    const int R = big ? 128 : 64;
    const dim3 grid(cdiv(a.N, R), cdiv(a.M, R), a.ksplit);
    const X3Conv cv{H, W, Cin};
    if (big) gemm_ex3_kernel<OP_MC, OP_IM, 2><<<grid, TNT, 0, (hipStream_t)stream>>>(a, kchunk, cv);
    else if (x3_kwave(grid, kchunk, a.ksplit)) gemm_ex3_kw_kernel<OP_MC, OP_IM><<<grid, TNT, 0, (hipStream_t)stream>>>(a, kchunk, cv);
    else gemm_ex3_kernel<OP_MC, OP_IM, 1><<<grid, TNT, 0, (hipStream_t)stream>>>(a, kchunk, cv);
    return cmt_check_launch("cmt_conv3x3_wgrad_bf16x3");
}

extern "C" int cmt_ln_train_fwd(const cmt_ln_train_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->rows > 0 && (ap->C == 64 || ap->C == 256), "cmt_ln_train_fwd: C must be 64 or 256");
    CMT_REQUIRE(ap->X && ap->Y && ap->W && ap->B && ap->mean && ap->rstd, "cmt_ln_train_fwd: null pointer");
    const unsigned g = (unsigned)cdiv(ap->rows, 4);
    if (ap->C == 64) ln_fwd_kernel<64><<<g, 256, 0, (hipStream_t)stream>>>(*ap);
    else ln_fwd_kernel<256><<<g, 256, 0, (hipStream_t)stream>>>(*ap);
    return cmt_check_launch("cmt_ln_train_fwd");
}

extern "C" int cmt_ln_train_bwd(const cmt_ln_train_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->rows > 0 && (ap->C == 64 || ap->C == 256), "cmt_ln_train_bwd: C must be 64 or 256");
    CMT_REQUIRE(ap->X && ap->dY && ap->dX && ap->W && ap->mean && ap->rstd, "cmt_ln_train_bwd: null pointer");
    // one weight set: ~2 rows per wave, blocks reduce before their atomics; GroupLayerNorm1d: a wave
    // per row as before
    const unsigned g = ap->rows_per_wset <= 0 ? (unsigned)min(cdiv(ap->rows, 8), 128) : (unsigned)min(cdiv(ap->rows, 4), 512);
    if (ap->C == 64) ln_bwd_kernel<64><<<g, 256, 0, (hipStream_t)stream>>>(*ap);
    else ln_bwd_kernel<256><<<g, 256, 0, (hipStream_t)stream>>>(*ap);
    return cmt_check_launch("cmt_ln_train_bwd");
}

// sums (2C floats) + the row blocks' partial sums (BN_MAXB x 2C floats)
extern "C" int64_t cmt_bn_workspace_bytes(int C) { return (int64_t)(2 + 2 * BN_MAXB) * C * sizeof(float); }

extern "C" int cmt_bn_relu_train_fwd(const cmt_bn_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->rows > 0 && ap->C > 0 && ap->X && ap->Y && ap->W && ap->B && ap->mean_save &&
                ap->rstd_save && ap->workspace, "cmt_bn_relu_train_fwd: bad arguments");
    const cmt_bn_args& a = *ap;
    hipStream_t s = (hipStream_t)stream;
    float* sums = (float*)a.workspace;   // [0:C) centred squares, [C:2C) mean
    float* part = sums + 2 * a.C;        // [nblk][C] partial sums of one pass
    const int rpb = bn_rows_per_block(a.rows);   // 507 blocks of 64 rows at 32 400 rows
    const int nblk = cdiv(a.rows, rpb);
    dim3 grid(nblk, cdiv(a.C, 256));
    col_sum_kernel<<<grid, 256, 0, s>>>(a.X, a.rows, a.C, nullptr, part, 0, rpb);
    bn_reduce_kernel<<<cdiv(a.C, 32), 256, 0, s>>>(part, nblk, a.C, a.C, sums + a.C, 1.f / a.rows);
    col_sum_kernel<<<grid, 256, 0, s>>>(a.X, a.rows, a.C, sums + a.C, part, 1, rpb);
    bn_reduce_kernel<<<cdiv(a.C, 32), 256, 0, s>>>(part, nblk, a.C, a.C, sums, 1.f);
    bn_finalize_kernel<<<cdiv(a.C, 256), 256, 0, s>>>(a, sums);
    bn_apply_kernel<<<(unsigned)cdiv64((int64_t)a.rows * a.C, 256), 256, 0, s>>>(a);
    return cmt_check_launch("cmt_bn_relu_train_fwd");
}

extern "C" int cmt_bn_relu_train_bwd(const cmt_bn_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->rows > 0 && ap->X && ap->Y && ap->dY && ap->dX && ap->W && ap->mean_save &&
                ap->rstd_save && ap->workspace, "cmt_bn_relu_train_bwd: bad arguments");
    const cmt_bn_args& a = *ap;
    hipStream_t s = (hipStream_t)stream;
    float* sums = (float*)a.workspace;
    float* part = sums + 2 * a.C;        // [nblk][2C]
    const int rpb = bn_rows_per_block(a.rows);
    const int nblk = cdiv(a.rows, rpb);
    bn_bwd_sums_kernel<<<dim3(nblk, cdiv(a.C, 256)), 256, 0, s>>>(a, part, rpb);
    bn_reduce_kernel<<<cdiv(2 * a.C, 32), 256, 0, s>>>(part, nblk, 2 * a.C, 2 * a.C, sums, 1.f);
    bn_bwd_apply_kernel<<<(unsigned)cdiv64((int64_t)a.rows * a.C, 256), 256, 0, s>>>(a, sums);
    bn_param_grads_kernel<<<cdiv(a.C, 256), 256, 0, s>>>(a, sums);
    return cmt_check_launch("cmt_bn_relu_train_bwd");
}

extern "C" int cmt_im2col3x3(const float* X, int nimg, int H, int W, int C, float* out, void* stream) {
    CMT_REQUIRE(X && out && nimg > 0 && H > 0 && W > 0 && C % 4 == 0, "cmt_im2col3x3: C must be a multiple of 4");
    const int64_t total4 = (int64_t)nimg * H * W * 9 * C / 4;
    im2col3x3_kernel<<<(unsigned)cdiv64(total4, 256), 256, 0, (hipStream_t)stream>>>(X, nimg, H, W, C, out);
    return cmt_check_launch("cmt_im2col3x3");
}

extern "C" int cmt_det_loss(const cmt_det_loss_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->out && ap->ncls > 0 && (ap->R == 0 || (ap->logits && ap->labels)) &&
                (ap->Rb == 0 || (ap->boxes && ap->targets && ap->box_w)), "cmt_det_loss: bad arguments");
    CMT_REQUIRE(ap->cls_avg > 0.f && ap->box_avg > 0.f, "cmt_det_loss: average factors must be > 0");
    det_loss_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(*ap);
    return cmt_check_launch("cmt_det_loss");
}

extern "C" int cmt_match_cost(const cmt_match_cost_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->Nq > 0 && ap->ngt > 0 && ap->logits && ap->boxes && ap->gt && ap->gt_labels && ap->cost,
                "cmt_match_cost: bad arguments");
    match_cost_kernel<<<cdiv(ap->Nq * ap->ngt, 256), 256, 0, (hipStream_t)stream>>>(*ap);
    return cmt_check_launch("cmt_match_cost");
}

extern "C" int cmt_sumsq(const float* x, int64_t n, float* out, void* stream) {
    CMT_REQUIRE(x && out && n >= 0, "cmt_sumsq: bad arguments");
    const int64_t nb = cdiv64(n, 256);
    const unsigned g = (unsigned)(nb < 1024 ? nb : 1024);
    if (g > 0) sumsq_kernel<<<g, 256, 0, (hipStream_t)stream>>>(x, n, out);
    return cmt_check_launch("cmt_sumsq");
}

extern "C" int cmt_adamw_step(const cmt_adamw_args* ap, void* stream) {
    CMT_REQUIRE(ap && ap->param && ap->grad && ap->exp_avg && ap->exp_avg_sq && ap->n > 0 && ap->step >= 1,
                "cmt_adamw_step: bad arguments");
    adamw_kernel<<<(unsigned)cdiv64(ap->n, 256), 256, 0, (hipStream_t)stream>>>(*ap);
    return cmt_check_launch("cmt_adamw_step");
}
