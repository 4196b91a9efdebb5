// Wavefront-reduction / elementwise kernels of the decoder head (gfx950):
// LayerNorm (+post-norm, nan_to_num, coop max), positional encodings,
// camera-frustum geometry, layout transposes, task-head tail.
// All are HBM- or latency-bound; one wave64 per row where a row reduction is
// needed, 16-byte vector accesses where the layout allows.
#include "cmt_common.h"

#include <cstdlib>

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Typed scalar store / 8-wide vector store for the dtype-generic outputs.
__device__ __forceinline__ void store_dt(void* p, int64_t idx, int dt, float v) {
    if (dt == CMT_F32) ((float*)p)[idx] = v;
    else if (dt == CMT_F16) ((f16_t*)p)[idx] = (f16_t)v;
    else ((bf16_t*)p)[idx] = (bf16_t)v;
}

// ---------------------------------------------------------------------------
// LayerNorm: one wave per row, VPT = C / 64 values per lane (lane-strided so
// the loads are 256-byte coalesced per instruction).  Optional outputs from
// the same registers: a second LN of the result (post_norm), and the next
// GEMMs' operands in the compute dtype (lowp(y), lowp(y + P)).
// ---------------------------------------------------------------------------
// NP > 0: the number of split-K parts known at compile time -- every part's loads, the
// affine weights and P are issued before the first use (one memory round trip per row
// instead of one per part: the decoder's 900-row LayerNorms are latency-bound); NP = 0
// reads a.nparts at run time.  Same summation order either way.
template <int VPT, typename LT, bool PAIR = false, int NP = 0>
__global__ __launch_bounds__(256) void layernorm_kernel(cmt_ln_args a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= a.rows) return;
    constexpr int C = VPT * 64;
    float v[VPT];
    const float* x = a.X + (int64_t)row * a.ldx;
    float wv[VPT], bv[VPT];
    if constexpr (NP > 0) {
        float xv[NP][VPT];
#pragma unroll
        for (int q = 0; q < NP; ++q)
#pragma unroll
            for (int i = 0; i < VPT; ++i) xv[q][i] = x[q * a.part_stride + lane + 64 * i];
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            wv[i] = a.W[lane + 64 * i];
            bv[i] = a.B[lane + 64 * i];
        }
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            v[i] = xv[0][i];
#pragma unroll
            for (int q = 1; q < NP; ++q) v[i] += xv[q][i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < VPT; ++i) v[i] = x[lane + 64 * i];
        for (int q = 1; q < a.nparts; ++q) {   // split-K partial products (cmt_gemm k_splits)
            const float* xq = x + q * a.part_stride;
#pragma unroll
            for (int i = 0; i < VPT; ++i) v[i] += xq[lane + 64 * i];
        }
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            wv[i] = a.W[lane + 64 * i];
            bv[i] = a.B[lane + 64 * i];
        }
    }
    float w2v[VPT], b2v[VPT];
    if (a.Y2) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            w2v[i] = a.W2[lane + 64 * i];
            b2v[i] = a.B2[lane + 64 * i];
        }
    }
    float pv[VPT];
    if (a.Yp) {
        const float* pr = a.P + (int64_t)row * a.ldp;
#pragma unroll
        for (int i = 0; i < VPT; ++i) pv[i] = pr[lane + 64 * i];
    }
    float yold[VPT];
    if (a.Y && (a.flags & CMT_LN_MAX_INTO)) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) yold[i] = a.Y[(int64_t)row * a.ldy + lane + 64 * i];
    }
    float y2old[VPT];
    if (a.Y2 && (a.flags2 & CMT_LN_MAX_INTO)) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) y2old[i] = a.Y2[(int64_t)row * a.ldy2 + lane + 64 * i];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += v[i];
    const float mean = wave_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) { float d = v[i] - mean; ss += d * d; }
    const float rstd = rsqrtf(wave_sum(ss) / (float)C + a.eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = lane + 64 * i;
        float o = (v[i] - mean) * rstd * wv[i] + bv[i];
        v[i] = o;   // the second LN consumes the first LN's output
        if (a.flags & CMT_LN_NAN_TO_NUM) o = nan_to_num(o);
        if (a.flags & CMT_LN_MAX_INTO) o = fmaxf(o, yold[i]);
        if (a.Y) a.Y[(int64_t)row * a.ldy + c] = o;
        if constexpr (PAIR) {   // CMT_F16P rows [hi(C) | lo(C)]
            if (a.Yl) store_pair((pair_t*)a.Yl + (int64_t)row * a.ldyl, C, c, o);
            if (a.Yp) store_pair((pair_t*)a.Yp + (int64_t)row * a.ldyp, C, c, o + pv[i]);
        } else {
            if (a.Yl) ((LT*)a.Yl)[(int64_t)row * a.ldyl + c] = (LT)o;
            if (a.Yp) ((LT*)a.Yp)[(int64_t)row * a.ldyp + c] = (LT)(o + pv[i]);
        }
    }
    if (a.Y2 == nullptr) return;
    s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += v[i];
    const float mean2 = wave_sum(s) / (float)C;
    ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) { float d = v[i] - mean2; ss += d * d; }
    const float rstd2 = rsqrtf(wave_sum(ss) / (float)C + a.eps);
    float* y2 = a.Y2 + (int64_t)row * a.ldy2;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = lane + 64 * i;
        float o = (v[i] - mean2) * rstd2 * w2v[i] + b2v[i];
        if (a.flags2 & CMT_LN_NAN_TO_NUM) o = nan_to_num(o);
        if (a.flags2 & CMT_LN_MAX_INTO) o = fmaxf(o, y2old[i]);
        y2[c] = o;
    }
}

// CMT_F16P form: one thread per 4 values of a row of width C (rows [hi(C) | lo(C)])
__global__ __launch_bounds__(256) void add_cast_pair_kernel(const float* __restrict__ X, const float* __restrict__ P,
                                                            int64_t n4, int C, pair_t* Yl, pair_t* Yp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const int64_t row = i / (C / 4);
    const int c = (int)(i - row * (C / 4)) * 4;
    const f32x4 x = X ? ((const f32x4*)X)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    if (Yl) store_pair4(Yl + row * 2 * C, C, c, x);
    if (Yp) store_pair4(Yp + row * 2 * C, C, c, x + ((const f32x4*)P)[i]);
}

template <typename LT>
__global__ __launch_bounds__(256) void add_cast_kernel(const float* __restrict__ X, const float* __restrict__ P,
                                                       int64_t n4, LT* Yl, LT* Yp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const f32x4 x = X ? ((const f32x4*)X)[i] : f32x4{0.f, 0.f, 0.f, 0.f};   // X == NULL: zeros
    typedef LT l4 __attribute__((ext_vector_type(4)));
    if (Yl) ((l4*)Yl)[i] = l4{(LT)x[0], (LT)x[1], (LT)x[2], (LT)x[3]};
    if (Yp) {
        const f32x4 y = x + ((const f32x4*)P)[i];
        ((l4*)Yp)[i] = l4{(LT)y[0], (LT)y[1], (LT)y[2], (LT)y[3]};
    }
}

// ---------------------------------------------------------------------------
// pos2embed (cmt_head.py:40-50), optionally fused with coords_bev (324-337) or
// with sigmoid(inverse_sigmoid(.)) of the query reference points (470).
// One thread per output element.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float inv_sigmoid_dev(float x) {
    x = fminf(fmaxf(x, 0.f), 1.f);
    const float x1 = fmaxf(x, 1e-5f);
    const float x2 = fmaxf(1.f - x, 1e-5f);
    return logf(x1 / x2);
}
__device__ __forceinline__ float sigmoid_dev(float x) { return 1.f / (1.f + expf(-x)); }

template <typename OT, bool PAIR = false>
__global__ __launch_bounds__(256) void pos2embed_kernel(const float* __restrict__ pos, int64_t pos_stride, int n,
                                                        int F, int mode, int x_size, int y_size, OT* out,
                                                        int64_t ldo) {
    // one thread = 8 consecutive outputs (4 sin/cos pairs sharing an argument)
    // 32-bit index math (the host checks n * groups < 2^31): a 64-bit division
    // per thread was most of this kernel's VALU time
    const unsigned groups = (unsigned)(2 * F) >> 3;
    const unsigned idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (unsigned)n * groups) return;
    const int i = (int)(idx / groups);
    const int f0 = (int)(idx - (unsigned)i * groups) * 8;
    float px, py;
    if (pos == nullptr) {
        // coords_bev: token t = r * y_size + c  ->  x = (c+0.5)/x_size, y = (r+0.5)/y_size
        const int r = i / y_size;
        const int c = i - r * y_size;
        px = ((float)c + 0.5f) / (float)x_size;
        py = ((float)r + 0.5f) / (float)y_size;
    } else {
        px = pos[(int64_t)i * pos_stride];
        py = pos[(int64_t)i * pos_stride + 1];
        if (mode == 1) {
            px = sigmoid_dev(inv_sigmoid_dev(px));
            py = sigmoid_dev(inv_sigmoid_dev(py));
        }
    }
    const float scale = 6.283185307179586f;
    const float p = (f0 < F ? py : px) * scale;   // first F outputs embed y, the next F embed x
    const int j0 = f0 < F ? f0 : f0 - F;
    float o[8];
    // 2k / F is exact as 2k * (1/F) when F is a power of two (every CMT config)
    const bool f_pow2 = (F & (F - 1)) == 0;
    const float inv_f = 1.f / (float)F;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float two_k = 2.f * (float)((j0 >> 1) + t);
        const float dim_t = (f_pow2 ? two_k * inv_f : two_k / (float)F) + 1.f;
        const float v = p / dim_t;                 // |v| <= 2*pi: v_sin/v_cos are accurate here
        o[2 * t] = __sinf(v);
        o[2 * t + 1] = __cosf(v);
    }
    OT* dst = out + (int64_t)i * ldo + f0;
    if constexpr (PAIR) {
        store_pair8((pair_t*)out + (int64_t)i * ldo, 2 * F, f0, o);
    } else if constexpr (sizeof(OT) == 4) {
        *(f32x4*)dst = f32x4{o[0], o[1], o[2], o[3]};
        *(f32x4*)(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
        typedef OT o8 __attribute__((ext_vector_type(8)));
        *(o8*)dst = o8{(OT)o[0], (OT)o[1], (OT)o[2], (OT)o[3], (OT)o[4], (OT)o[5], (OT)o[6], (OT)o[7]};
    }
}

// ---------------------------------------------------------------------------
// _rv_pe geometry (cmt_head.py:417-432): one thread per (bv, h, w, depth).
// ---------------------------------------------------------------------------
struct PcRange { float v[6]; };

template <typename OT, bool PAIR = false>
__global__ void rv_pe_coords_kernel8(int BV, int H, int W, int D, float pad_h, float pad_w, float dstep,
                                     const float* __restrict__ i2l, PcRange pc, OT* out) {
    // one thread = 8 consecutive depth samples of one image token: 24 outputs, written as whole
    // 16-byte (16-bit outputs) or 32-byte (fp32) pieces; 32-bit index math
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int dg = D >> 3;
    const int total = BV * H * W * dg;
    if (idx >= total) return;
    const int k0 = (idx % dg) * 8;
    const int tok = idx / dg;
    const int w = tok % W;
    const int h = (tok / W) % H;
    const int bv = tok / (W * H);
    const float u = (float)w * pad_w / (float)W;
    const float v = (float)h * pad_h / (float)H;
    const float* M = i2l + bv * 16;
    float m[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) m[i] = M[i];
    float res[24];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float d = 1.f + (float)(k0 + j) * dstep / (float)D;
        const float c[4] = {u * d, v * d, d, 1.f};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            float a = m[r * 4 + 0] * c[0];
            a = fmaf(m[r * 4 + 1], c[1], a);
            a = fmaf(m[r * 4 + 2], c[2], a);
            a = fmaf(m[r * 4 + 3], c[3], a);
            res[3 * j + r] = (a - pc.v[r]) / (pc.v[3 + r] - pc.v[r]);
        }
    }
    OT* o = out + (int64_t)tok * (3 * D) + 3 * k0;   // 24 consecutive outputs
    if constexpr (PAIR) {
        pair_t* prow = (pair_t*)out + (int64_t)tok * (6 * D);   // [hi(3D) | lo(3D)]
#pragma unroll
        for (int q = 0; q < 3; ++q) store_pair8(prow, 3 * D, 3 * k0 + 8 * q, res + 8 * q);
    } else if constexpr (sizeof(OT) == 2) {
        typedef OT o8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            o8 pk;
#pragma unroll
            for (int e = 0; e < 8; ++e) pk[e] = (OT)res[8 * q + e];
            *(o8*)(o + 8 * q) = pk;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 6; ++q)
            *(f32x4*)(o + 4 * q) = f32x4{res[4 * q], res[4 * q + 1], res[4 * q + 2], res[4 * q + 3]};
    }
}

template <typename OT>
__global__ void rv_pe_coords_kernel(int BV, int H, int W, int D, float pad_h, float pad_w, float dstep,
                                    const float* __restrict__ i2l, PcRange pc, OT* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)BV * H * W * D;
    if (idx >= total) return;
    const int k = (int)(idx % D);
    const int64_t tok = idx / D;
    const int w = (int)(tok % W);
    const int h = (int)((tok / W) % H);
    const int bv = (int)(tok / ((int64_t)W * H));
    const float u = (float)w * pad_w / (float)W;
    const float v = (float)h * pad_h / (float)H;
    const float d = 1.f + (float)k * dstep / (float)D;
    const float c[4] = {u * d, v * d, d, 1.f};
    const float* M = i2l + (int64_t)bv * 16;
    OT* o = out + tok * (3 * D) + 3 * k;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float a = M[r * 4 + 0] * c[0];
        a = fmaf(M[r * 4 + 1], c[1], a);
        a = fmaf(M[r * 4 + 2], c[2], a);
        a = fmaf(M[r * 4 + 3], c[3], a);
        o[r] = (OT)((a - pc.v[r]) / (pc.v[3 + r] - pc.v[r]));
    }
}

// _rv_query_embed geometry (cmt_head.py:446-463): one thread per (b, v, q, depth).
template <typename TO, bool PAIR = false>
__global__ void rv_query_coords_kernel(const float* __restrict__ ref, int B, int V, int Nq, int D,
                                       float pad_h, float pad_w, float dstep,
                                       const float* __restrict__ l2i, const float* __restrict__ i2l,
                                       PcRange pc, TO* out, float* mask) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * V * Nq * D;
    if (idx >= total) return;
    const int k = (int)(idx % D);
    const int64_t bvq = idx / D;
    const int q = (int)(bvq % Nq);
    const int64_t bv = bvq / Nq;
    const int b = (int)(bv / V);
    float r[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float x = sigmoid_dev(inv_sigmoid_dev(ref[((int64_t)b * Nq + q) * 3 + c]));
        r[c] = x * (pc.v[3 + c] - pc.v[c]) + pc.v[c];
    }
    const float* L = l2i + bv * 16;
    float pr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float a = L[c * 4 + 0] * r[0];
        a = fmaf(L[c * 4 + 1], r[1], a);
        a = fmaf(L[c * 4 + 2], r[2], a);
        pr[c] = a + L[c * 4 + 3];
    }
    const bool zpos = pr[2] > 0.f;
    const float den = pr[2] + (zpos ? 1e-6f : -1e-6f);
    const float px = pr[0] / den, py = pr[1] / den, pz = pr[2] / den;
    if (k == 0) {
        const bool m = (px < pad_w) && (px >= 0.f) && (py < pad_h) && (py >= 0.f) && zpos;
        mask[bvq] = m ? 1.f : 0.f;
    }
    const float d = 1.f + (float)k * dstep / (float)D;
    const float c4[4] = {px * d, py * d, pz * d, 1.f};
    const float* M = i2l + bv * 16;
    TO* o = out + bvq * (3 * D) + 3 * k;
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
        float a = M[rr * 4 + 0] * c4[0];
        a = fmaf(M[rr * 4 + 1], c4[1], a);
        a = fmaf(M[rr * 4 + 2], c4[2], a);
        a = fmaf(M[rr * 4 + 3], c4[3], a);
        const float v = (a - pc.v[rr]) / (pc.v[3 + rr] - pc.v[rr]);
        if constexpr (PAIR) store_pair((pair_t*)out + bvq * (6 * D), 3 * D, 3 * k + rr, v);   // [hi(3D) | lo(3D)]
        else o[rr] = (TO)v;   // RNE, as cmt_cast
    }
}

__global__ void masked_view_sum_kernel(const float* __restrict__ X, const float* __restrict__ mask, int B, int V,
                                       int Nq, int C, float* Y) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * Nq * C;
    if (idx >= total) return;
    const int c = (int)(idx % C);
    const int64_t bq = idx / C;
    const int q = (int)(bq % Nq);
    const int b = (int)(bq / Nq);
    float s = 0.f;
    for (int v = 0; v < V; ++v) {
        const int64_t bvq = ((int64_t)b * V + v) * Nq + q;
        s += X[bvq * C + c] * mask[bvq];
    }
    Y[idx] += s;
}

// Y[b,q,:] = base[q,:] + sum_v X[b,v,q,:] * mask[b,v,q]  (base NULL: Y += ...), and, when
// given, the decoder's first operands Yp = lowp(Y) (= lowp(0 + query_pos)) and Yl = lowp(0).
template <typename TL, bool PAIR = false>
__global__ void masked_view_sum_ex_kernel(const float* __restrict__ X, const float* __restrict__ mask, int B, int V,
                                          int Nq, int C, const float* __restrict__ base, float* Y, TL* Yl, TL* Yp) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * Nq * C;
    if (idx >= total) return;
    const int c = (int)(idx % C);
    const int64_t bq = idx / C;
    const int q = (int)(bq % Nq);
    const int b = (int)(bq / Nq);
    float s = 0.f;
    for (int v = 0; v < V; ++v) {
        const int64_t bvq = ((int64_t)b * V + v) * Nq + q;
        s += X[bvq * C + c] * mask[bvq];
    }
    const float y = (base ? base[(int64_t)q * C + c] : Y[idx]) + s;
    Y[idx] = y;
    if constexpr (PAIR) {   // rows [hi(C) | lo(C)]
        if (Yp) store_pair((pair_t*)Yp + bq * 2 * C, C, c, y);
        if (Yl) store_pair((pair_t*)Yl + bq * 2 * C, C, c, 0.f);
    } else {
        if (Yp) Yp[idx] = (TL)y;
        if (Yl) Yl[idx] = (TL)0.f;
    }
}

// ---------------------------------------------------------------------------
// NCHW -> token rows (64x64 tile transpose through LDS).
// ---------------------------------------------------------------------------
template <typename TO, bool PAIR = false>
__global__ __launch_bounds__(256) void nchw_to_rows_kernel(const float* __restrict__ X, int nv, int C, int HW,
                                                           TO* Y, int64_t ldy, int64_t rows_per_batch,
                                                           int64_t row_offset, int* range_flag) {
    __shared__ float tile[64][65];
    const int img = blockIdx.z;
    const int c0 = blockIdx.y * 64;
    const int p0 = blockIdx.x * 64;
    const float* xs = X + (int64_t)img * C * HW;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    bool bad = false;
    for (int i = ty; i < 64; i += 4) {
        const int c = c0 + i, p = p0 + tx;
        tile[i][tx] = (c < C && p < HW) ? xs[(int64_t)c * HW + p] : 0.f;
        bad |= f16_unrepresentable(tile[i][tx]);
    }
    // f16 / pair outputs cannot carry the value; an fp32 output with a flag is the training conv's
    // input, which the split-f16 conv reads as pairs next (bf16 carries any fp32 exponent)
    if constexpr (!std::is_same<TO, bf16_t>::value) raise_range_flag(range_flag, bad);
    __syncthreads();
    const int bo = img / nv, v = img - bo * nv;
    for (int i = ty; i < 64; i += 4) {
        const int p = p0 + i, c = c0 + tx;
        if (p < HW && c < C) {
            const int64_t row = (int64_t)bo * rows_per_batch + row_offset + (int64_t)v * HW + p;
            if constexpr (PAIR) store_pair((pair_t*)Y + row * ldy, C, c, tile[tx][i]);
            else Y[row * ldy + c] = (TO)tile[tx][i];
        }
    }
}

// Vector form (HW % 4 == 0, C % 64 == 0, 16-byte aligned output rows): 16-byte
// loads along pixels and 16-byte stores along channels.  The scalar kernel's
// 4-byte loads and 2-byte stores (128 B per wave instruction) held the BEV
// layout pass to ~3.3 TB/s.  LDS tile [64 c][65]: bank (c + p) % 64, so both
// the pixel-major scalar writes (16 pixel quads x 4 channels per wave) and the
// transposed reads (8 channel groups x 8 pixels per wave) are conflict-free.
template <typename TO, bool PAIR = false>
__global__ __launch_bounds__(256) void nchw_to_rows_vec_kernel(const float* __restrict__ X, int nv, int C, int HW,
                                                               TO* Y, int64_t ldy, int64_t rows_per_batch,
                                                               int64_t row_offset, int* range_flag) {
    constexpr int VW = 16 / sizeof(TO);          // channels per 16-byte store
    constexpr int TPP = 64 / VW;                 // threads per pixel
    __shared__ float tile[64][65];
    const int img = blockIdx.z;
    const int c0 = blockIdx.y * 64;
    const int p0 = blockIdx.x * 64;
    const float* xs = X + (int64_t)img * C * HW;
    const int t = threadIdx.x;
    {
        const int q = (t & 15) * 4, cr = t >> 4;   // 16 threads x 4 pixels per channel row, 16 rows per pass
        f32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = c0 + cr + 16 * k, p = p0 + q;
            v[k] = p < HW ? *(const f32x4*)(xs + (int64_t)c * HW + p) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                tile[cr + 16 * k][q + e] = v[k][e];
                bad |= f16_unrepresentable(v[k][e]);
            }
        // as nchw_to_rows_kernel: every format but bf16 (an fp32 output with a flag feeds a split conv)
        if constexpr (!std::is_same<TO, bf16_t>::value) raise_range_flag(range_flag, bad);
    }
    __syncthreads();
    const int bo = img / nv, v = img - bo * nv;
    const int cg = (t % TPP) * VW;
#pragma unroll
    for (int pass = 0; pass < 64 / (256 / TPP); ++pass) {
        const int pi = pass * (256 / TPP) + t / TPP;
        const int p = p0 + pi;
        if (p >= HW) continue;
        float o[VW];
#pragma unroll
        for (int j = 0; j < VW; ++j) o[j] = tile[cg + j][pi];
        const int64_t row = (int64_t)bo * rows_per_batch + row_offset + (int64_t)v * HW + p;
        TO* dst = Y + row * ldy + c0 + cg;
        if constexpr (PAIR) {
            store_pair8((pair_t*)Y + row * ldy, C, c0 + cg, o);   // rows [hi(C) | lo(C)]
        } else if constexpr (VW == 4) {
            *(f32x4*)dst = f32x4{o[0], o[1], o[2], o[3]};
        } else {
            typedef TO o8 __attribute__((ext_vector_type(8)));
            *(o8*)dst = o8{(TO)o[0], (TO)o[1], (TO)o[2], (TO)o[3], (TO)o[4], (TO)o[5], (TO)o[6], (TO)o[7]};
        }
    }
}

// fp32 rows (leading dimension ldx) -> CMT_F16P rows [hi(C) | lo(C)], 4 values per thread
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ X, int64_t ldx, int64_t n4, int C,
                                                         pair_t* Y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const int64_t row = i / (C / 4);
    const int c = (int)(i - row * (C / 4)) * 4;
    store_pair4(Y + row * 2 * C, C, c, *(const f32x4*)(X + row * ldx + c));
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ X, TO* Y, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) Y[i] = (TO)(float)X[i];
}

// ---------------------------------------------------------------------------
// Task-head tail (cmt_head.py:136-203, 501-513), one launch.
// A workgroup owns (layer l, TQ-query block, batch b).  It stages the block's
// conv-1 rows H1 [l][b*Nq + q][nheads*hc] (+ k/2 halo rows each side) in LDS,
// applies GroupLayerNorm1d (per head, hc = 64 channels, biased var, eps 1e-6,
// cmt_head.py:56-66) + ReLU there -- one wave per (row, head) -- and then the
// grouped Conv1d #2 (+bias, kernel k along queries, zero pad: halo rows
// outside [0, Nq) stay 0 AFTER the norm, as the conv pads its input) with the
// center/height box epilogue; one thread per (query, output) pair.  H1 is only
// read.  LDS rows are padded by 4 floats so the query-strided f32x4 reads of
// a wave spread over all banks (an unpadded 384-float row put the 16..32
// queries of a wave on one bank).
// ---------------------------------------------------------------------------
struct TailParams {
    const float* G; int L, B, Nq, nheads, hc;
    const float* gw; const float* gb;
    const float* W2; const float* B2;
    int head_of[64];
    int out_total, k;
    const float* ref; int center_col, height_col;
    float pc[6];
    float* OUT;
};

constexpr int TQ = 16;

__device__ __forceinline__ int tail_gstride(int width) { return width + 4; }
__device__ __forceinline__ int tail_wstride(int hc) { return hc + 4; }

__global__ __launch_bounds__(256) void task_head_tail_kernel(TailParams p) {
    extern __shared__ __attribute__((aligned(16))) float tsm[];
    const int l = blockIdx.x;
    const int q0 = blockIdx.y * TQ;
    const int b = blockIdx.z;
    const int width = p.nheads * p.hc;
    const int gs = tail_gstride(width), ws = tail_wstride(p.hc);
    const int half = p.k >> 1;
    const int nrows = TQ + 2 * half;
    float* G = tsm;                                   // [nrows][gs]
    float* W = tsm + nrows * gs;                      // [out_total * k][ws]
    const float* Gsrc = p.G + ((int64_t)l * p.B + b) * p.Nq * width;
    const float* Wsrc = p.W2 + (int64_t)l * p.out_total * p.k * p.hc;
    // staging: batches of 8 independent 16-B loads per thread before their LDS stores
    const int ng = nrows * width / 4, nw = p.out_total * p.k * p.hc / 4;
    for (int i0 = 0; i0 < ng + nw; i0 += 8 * 256) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + threadIdx.x;
            v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (i < ng) {
                const int r = (i * 4) / width, c = (i * 4) - r * width;
                const int q = q0 - half + r;
                if (q >= 0 && q < p.Nq) v[u] = *(const f32x4*)(Gsrc + (int64_t)q * width + c);
            } else if (i < ng + nw) {
                v[u] = *(const f32x4*)(Wsrc + 4 * (i - ng));
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + threadIdx.x;
            if (i < ng) {
                const int r = (i * 4) / width, c = (i * 4) - r * width;
                *(f32x4*)(G + r * gs + c) = v[u];
            } else if (i < ng + nw) {
                const int r = ((i - ng) * 4) / p.hc, c = ((i - ng) * 4) - r * p.hc;
                *(f32x4*)(W + r * ws + c) = v[u];
            }
        }
    }
    __syncthreads();
    {
        // GroupLayerNorm1d + ReLU: 16 lanes per (row, head) group, 4 channels per lane
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int sub = lane >> 4, j = lane & 15;
        const int ngroups = nrows * p.nheads;
        const float* w = p.gw + (int64_t)l * width;
        const float* bb = p.gb + (int64_t)l * width;
        for (int g0 = wave * 4; g0 < ngroups; g0 += 16) {
            const int g = g0 + sub;
            const int r = g / p.nheads, hd = g - r * p.nheads;
            const int q = q0 - half + r;
            const bool ok = g < ngroups && q >= 0 && q < p.Nq;   // rows outside [0, Nq) stay 0 (conv #2 pad)
            const int c = hd * 64 + 4 * j;
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            if (ok) x = *(const f32x4*)(G + r * gs + c);
            float s = (x[0] + x[1]) + (x[2] + x[3]);
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off);
            const float mu = s / 64.f;
            const f32x4 d = {x[0] - mu, x[1] - mu, x[2] - mu, x[3] - mu};
            float v2 = (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) v2 += __shfl_xor(v2, off);
            const float inv = 1.f / sqrtf(v2 / 64.f + 1e-6f);
            if (ok) {
                f32x4 y;
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = fmaxf(w[c + e] * (d[e] * inv) + bb[c + e], 0.f);
                *(f32x4*)(G + r * gs + c) = y;
            }
        }
    }
    __syncthreads();
    const int qi = threadIdx.x % TQ;
    const int q = q0 + qi;
    if (q >= p.Nq) return;
    for (int o = threadIdx.x / TQ; o < p.out_total; o += blockDim.x / TQ) {
        const int hd = p.head_of[o];
        float acc = p.B2[(int64_t)l * p.out_total + o];
        for (int t = 0; t < p.k; ++t) {
            const float* g = G + (qi + t) * gs + hd * p.hc;
            const float* w = W + (o * p.k + t) * ws;
            float s0 = 0.f, s1 = 0.f;
            for (int c = 0; c < p.hc; c += 8) {
                const f32x4 g0 = *(const f32x4*)(g + c), g1 = *(const f32x4*)(g + c + 4);
                const f32x4 w0 = *(const f32x4*)(w + c), w1 = *(const f32x4*)(w + c + 4);
                s0 = fmaf(w0[0], g0[0], s0); s0 = fmaf(w0[1], g0[1], s0);
                s0 = fmaf(w0[2], g0[2], s0); s0 = fmaf(w0[3], g0[3], s0);
                s1 = fmaf(w1[0], g1[0], s1); s1 = fmaf(w1[1], g1[1], s1);
                s1 = fmaf(w1[2], g1[2], s1); s1 = fmaf(w1[3], g1[3], s1);
            }
            acc += s0 + s1;
        }
        const int rel_c = o - p.center_col;
        const int rel_h = o - p.height_col;
        if (p.center_col >= 0 && rel_c >= 0 && rel_c < 2) {
            const float rf = inv_sigmoid_dev(p.ref[((int64_t)b * p.Nq + q) * 3 + rel_c]);
            acc = sigmoid_dev(acc + rf) * (p.pc[3 + rel_c] - p.pc[rel_c]) + p.pc[rel_c];
        } else if (p.height_col >= 0 && rel_h == 0) {
            const float rf = inv_sigmoid_dev(p.ref[((int64_t)b * p.Nq + q) * 3 + 2]);
            acc = sigmoid_dev(acc + rf) * (p.pc[5] - p.pc[2]) + p.pc[2];
        }
        p.OUT[(((int64_t)l * p.B + b) * p.Nq + q) * p.out_total + o] = acc;
    }
}

inline unsigned nblocks(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" int cmt_layernorm_ex(const cmt_ln_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_layernorm: null args");
    const cmt_ln_args& a = *ap;
    CMT_REQUIRE(a.X && a.W && a.B && a.rows >= 0 && (a.Y || a.Yl || a.Yp || a.Y2), "cmt_layernorm: null pointer");
    CMT_REQUIRE(a.C % 64 == 0 && a.C >= 64 && a.C <= 1024, "cmt_layernorm: C must be a multiple of 64 in [64, 1024]");
    CMT_REQUIRE(a.Y2 == nullptr || (a.W2 && a.B2), "cmt_layernorm: second LN needs W2/B2");
    CMT_REQUIRE(a.Yp == nullptr || a.P != nullptr, "cmt_layernorm: Yp needs P");
    CMT_REQUIRE((a.Yl == nullptr && a.Yp == nullptr) || a.lowp_dtype == CMT_F16 || a.lowp_dtype == CMT_BF16 ||
                    a.lowp_dtype == CMT_F16P, "cmt_layernorm: lowp_dtype must be f16, bf16 or f16 pair");
    if (a.rows == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    dim3 grid(cdiv(a.rows, 4));
    const int np = a.nparts > 1 ? a.nparts : 1;
    if (a.C == 256 && (np == 1 || np == 2 || np == 4)) {   // the decoder's LayerNorms
#define LN_NP(NP)                                                                                          \
        if (np == NP) {                                                                                    \
            if (a.lowp_dtype == CMT_F16) layernorm_kernel<4, f16_t, false, NP><<<grid, 256, 0, s>>>(a);     \
            else if (a.lowp_dtype == CMT_F16P) layernorm_kernel<4, pair_t, true, NP><<<grid, 256, 0, s>>>(a); \
            else layernorm_kernel<4, bf16_t, false, NP><<<grid, 256, 0, s>>>(a);                            \
        }
        LN_NP(1) LN_NP(2) LN_NP(4)
#undef LN_NP
        return cmt_check_launch("cmt_layernorm");
    }
#define LN_CASE(V)                                                                              \
    case V:                                                                                     \
        if (a.lowp_dtype == CMT_F16) layernorm_kernel<V, f16_t><<<grid, 256, 0, s>>>(a);        \
        else if (a.lowp_dtype == CMT_F16P) layernorm_kernel<V, pair_t, true><<<grid, 256, 0, s>>>(a); \
        else layernorm_kernel<V, bf16_t><<<grid, 256, 0, s>>>(a);                               \
        break;
    switch (a.C / 64) {
        LN_CASE(1) LN_CASE(2) LN_CASE(3) LN_CASE(4) LN_CASE(5) LN_CASE(6) LN_CASE(7) LN_CASE(8)
        LN_CASE(9) LN_CASE(10) LN_CASE(11) LN_CASE(12) LN_CASE(13) LN_CASE(14) LN_CASE(15) LN_CASE(16)
    }
#undef LN_CASE
    return cmt_check_launch("cmt_layernorm");
}

extern "C" int cmt_layernorm(const float* X, int64_t ldx, int rows, int C, const float* W, const float* Bv,
                             float eps, float* Y, int64_t ldy, int flags, const float* W2, const float* B2,
                             float* Y2, int64_t ldy2, int flags2, void* stream) {
    CMT_REQUIRE(Y != nullptr, "cmt_layernorm: null pointer");
    cmt_ln_args a = {};
    a.X = X; a.ldx = ldx; a.rows = rows; a.C = C; a.W = W; a.B = Bv; a.eps = eps;
    a.Y = Y; a.ldy = ldy; a.flags = flags;
    a.W2 = W2; a.B2 = B2; a.Y2 = Y2; a.ldy2 = ldy2; a.flags2 = flags2;
    a.lowp_dtype = CMT_BF16;
    return cmt_layernorm_ex(&a, stream);
}

extern "C" int cmt_add_cast(const float* X, const float* P, int rows, int C, int lowp_dtype, void* Yl, void* Yp,
                            void* stream) {
    CMT_REQUIRE(rows >= 0 && C % 4 == 0 && (Yp == nullptr || P), "cmt_add_cast: bad arguments");
    CMT_REQUIRE(lowp_dtype == CMT_F16 || lowp_dtype == CMT_BF16 || lowp_dtype == CMT_F16P,
                "cmt_add_cast: lowp_dtype must be f16, bf16 or f16 pair");
    const int64_t n4 = (int64_t)rows * C / 4;
    if (n4 == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (lowp_dtype == CMT_F16P)
        add_cast_pair_kernel<<<nblocks(n4, 256), 256, 0, s>>>(X, P, n4, C, (pair_t*)Yl, (pair_t*)Yp);
    else if (lowp_dtype == CMT_F16)
        add_cast_kernel<f16_t><<<nblocks(n4, 256), 256, 0, s>>>(X, P, n4, (f16_t*)Yl, (f16_t*)Yp);
    else
        add_cast_kernel<bf16_t><<<nblocks(n4, 256), 256, 0, s>>>(X, P, n4, (bf16_t*)Yl, (bf16_t*)Yp);
    return cmt_check_launch("cmt_add_cast");
}

extern "C" int cmt_pos2embed(const float* pos, int64_t pos_stride, int n, int F, int mode, int grid_h,
                             int grid_w, void* out, int odtype, int64_t ldo, void* stream) {
    CMT_REQUIRE(out && n >= 0 && F > 0 && F % 4 == 0 && ldo % 8 == 0, "cmt_pos2embed: bad arguments");
    CMT_REQUIRE(pos != nullptr || (grid_h > 0 && grid_w > 0 && n == grid_h * grid_w),
                "cmt_pos2embed: grid mode needs n == grid_h*grid_w");
    CMT_REQUIRE(odtype == CMT_F32 || odtype == CMT_F16 || odtype == CMT_BF16 || odtype == CMT_F16P,
                "cmt_pos2embed: bad odtype");
    if (n == 0) return 0;
    const int64_t total = (int64_t)n * (2 * F / 8);
    CMT_REQUIRE(total < ((int64_t)1 << 31), "cmt_pos2embed: n * F too large for one launch");
    hipStream_t s = (hipStream_t)stream;
    if (odtype == CMT_F32)
        pos2embed_kernel<float><<<nblocks(total, 256), 256, 0, s>>>(pos, pos_stride, n, F, mode, grid_h, grid_w,
                                                                    (float*)out, ldo);
    else if (odtype == CMT_F16)
        pos2embed_kernel<f16_t><<<nblocks(total, 256), 256, 0, s>>>(pos, pos_stride, n, F, mode, grid_h, grid_w,
                                                                    (f16_t*)out, ldo);
    else if (odtype == CMT_F16P)
        pos2embed_kernel<pair_t, true><<<nblocks(total, 256), 256, 0, s>>>(pos, pos_stride, n, F, mode, grid_h,
                                                                           grid_w, (pair_t*)out, ldo);
    else
        pos2embed_kernel<bf16_t><<<nblocks(total, 256), 256, 0, s>>>(pos, pos_stride, n, F, mode, grid_h, grid_w,
                                                                     (bf16_t*)out, ldo);
    return cmt_check_launch("cmt_pos2embed");
}

extern "C" int cmt_rv_pe_coords(int BV, int h, int w, int D, float pad_h, float pad_w, float depth_max,
                                const float* i2l, const float* pc_range6, void* out, int odtype, void* stream) {
    CMT_REQUIRE(i2l && pc_range6 && out && BV > 0 && h > 0 && w > 0 && D > 0, "cmt_rv_pe_coords: bad arguments");
    CMT_REQUIRE(odtype == CMT_F32 || odtype == CMT_F16 || odtype == CMT_BF16 || odtype == CMT_F16P,
                "cmt_rv_pe_coords: bad odtype");
    CMT_REQUIRE(odtype != CMT_F16P || (D % 8 == 0 && (uintptr_t)out % 16 == 0),
                "cmt_rv_pe_coords: the f16-pair output needs D % 8 == 0 and a 16-byte aligned out");
    PcRange pc;
    for (int i = 0; i < 6; ++i) pc.v[i] = pc_range6[i];
    hipStream_t s = (hipStream_t)stream;
    // eight depths per thread when D and the output allow it, else one thread per depth
    if (D % 8 == 0 && (int64_t)BV * h * w * (D / 8) < ((int64_t)1 << 31) && (uintptr_t)out % 16 == 0) {
        const int64_t t8 = (int64_t)BV * h * w * (D / 8);
        if (odtype == CMT_F32)
            rv_pe_coords_kernel8<float><<<nblocks(t8, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w, depth_max - 1.f,
                                                                         i2l, pc, (float*)out);
        else if (odtype == CMT_F16)
            rv_pe_coords_kernel8<f16_t><<<nblocks(t8, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w, depth_max - 1.f,
                                                                         i2l, pc, (f16_t*)out);
        else if (odtype == CMT_F16P)
            rv_pe_coords_kernel8<pair_t, true><<<nblocks(t8, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w,
                                                                                depth_max - 1.f, i2l, pc,
                                                                                (pair_t*)out);
        else
            rv_pe_coords_kernel8<bf16_t><<<nblocks(t8, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w,
                                                                          depth_max - 1.f, i2l, pc, (bf16_t*)out);
        return cmt_check_launch("cmt_rv_pe_coords");
    }
    const int64_t total = (int64_t)BV * h * w * D;
    if (odtype == CMT_F32)
        rv_pe_coords_kernel<float><<<nblocks(total, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w, depth_max - 1.f,
                                                                       i2l, pc, (float*)out);
    else if (odtype == CMT_F16)
        rv_pe_coords_kernel<f16_t><<<nblocks(total, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w, depth_max - 1.f,
                                                                       i2l, pc, (f16_t*)out);
    else
        rv_pe_coords_kernel<bf16_t><<<nblocks(total, 256), 256, 0, s>>>(BV, h, w, D, pad_h, pad_w, depth_max - 1.f,
                                                                        i2l, pc, (bf16_t*)out);
    return cmt_check_launch("cmt_rv_pe_coords");
}

extern "C" int cmt_rv_query_coords(const float* ref, int B, int V, int Nq, int D, float pad_h, float pad_w,
                                   const float* l2i, const float* i2l, const float* pc_range6, float* out,
                                   float* mask, void* stream) {
    CMT_REQUIRE(ref && l2i && i2l && pc_range6 && out && mask && B > 0 && V > 0 && Nq > 0 && D > 0,
                "cmt_rv_query_coords: bad arguments");
    PcRange pc;
    for (int i = 0; i < 6; ++i) pc.v[i] = pc_range6[i];
    const int64_t total = (int64_t)B * V * Nq * D;
    rv_query_coords_kernel<float><<<nblocks(total, 256), 256, 0, (hipStream_t)stream>>>(
        ref, B, V, Nq, D, pad_h, pad_w, pc.v[3] - 1.f, l2i, i2l, pc, out, mask);
    return cmt_check_launch("cmt_rv_query_coords");
}

extern "C" int cmt_rv_query_coords_ex(const float* ref, int B, int V, int Nq, int D, float pad_h, float pad_w,
                                      const float* l2i, const float* i2l, const float* pc_range6, void* out,
                                      int odtype, float* mask, void* stream) {
    CMT_REQUIRE(ref && l2i && i2l && pc_range6 && out && mask && B > 0 && V > 0 && Nq > 0 && D > 0,
                "cmt_rv_query_coords_ex: bad arguments");
    CMT_REQUIRE(odtype == CMT_F32 || odtype == CMT_F16 || odtype == CMT_BF16 || odtype == CMT_F16P,
                "cmt_rv_query_coords_ex: bad odtype");
    PcRange pc;
    for (int i = 0; i < 6; ++i) pc.v[i] = pc_range6[i];
    const int64_t total = (int64_t)B * V * Nq * D;
    hipStream_t s = (hipStream_t)stream;
    if (odtype == CMT_F32)
        rv_query_coords_kernel<float><<<nblocks(total, 256), 256, 0, s>>>(ref, B, V, Nq, D, pad_h, pad_w,
                                                                          pc.v[3] - 1.f, l2i, i2l, pc, (float*)out, mask);
    else if (odtype == CMT_F16)
        rv_query_coords_kernel<f16_t><<<nblocks(total, 256), 256, 0, s>>>(ref, B, V, Nq, D, pad_h, pad_w,
                                                                          pc.v[3] - 1.f, l2i, i2l, pc, (f16_t*)out, mask);
    else if (odtype == CMT_F16P)
        rv_query_coords_kernel<pair_t, true><<<nblocks(total, 256), 256, 0, s>>>(ref, B, V, Nq, D, pad_h, pad_w,
                                                                                 pc.v[3] - 1.f, l2i, i2l, pc,
                                                                                 (pair_t*)out, mask);
    else
        rv_query_coords_kernel<bf16_t><<<nblocks(total, 256), 256, 0, s>>>(ref, B, V, Nq, D, pad_h, pad_w,
                                                                           pc.v[3] - 1.f, l2i, i2l, pc, (bf16_t*)out,
                                                                           mask);
    return cmt_check_launch("cmt_rv_query_coords_ex");
}

extern "C" int cmt_masked_view_sum(const float* X, const float* mask, int B, int V, int Nq, int C, float* Y,
                                   void* stream) {
    CMT_REQUIRE(X && mask && Y && B > 0 && V > 0 && Nq > 0 && C > 0, "cmt_masked_view_sum: bad arguments");
    const int64_t total = (int64_t)B * Nq * C;
    masked_view_sum_kernel<<<nblocks(total, 256), 256, 0, (hipStream_t)stream>>>(X, mask, B, V, Nq, C, Y);
    return cmt_check_launch("cmt_masked_view_sum");
}

extern "C" int cmt_masked_view_sum_ex(const float* X, const float* mask, int B, int V, int Nq, int C,
                                      const float* base, float* Y, void* Yl, void* Yp, int lowp_dtype, void* stream) {
    CMT_REQUIRE(X && mask && Y && B > 0 && V > 0 && Nq > 0 && C > 0, "cmt_masked_view_sum_ex: bad arguments");
    CMT_REQUIRE((!Yl && !Yp) || lowp_dtype == CMT_F16 || lowp_dtype == CMT_BF16 || lowp_dtype == CMT_F16P,
                "cmt_masked_view_sum_ex: lowp_dtype must be f16, bf16 or f16 pair");
    const int64_t total = (int64_t)B * Nq * C;
    hipStream_t s = (hipStream_t)stream;
    if (lowp_dtype == CMT_F16P)
        masked_view_sum_ex_kernel<pair_t, true><<<nblocks(total, 256), 256, 0, s>>>(X, mask, B, V, Nq, C, base, Y,
                                                                                    (pair_t*)Yl, (pair_t*)Yp);
    else if (lowp_dtype == CMT_F16)
        masked_view_sum_ex_kernel<f16_t><<<nblocks(total, 256), 256, 0, s>>>(X, mask, B, V, Nq, C, base, Y,
                                                                             (f16_t*)Yl, (f16_t*)Yp);
    else
        masked_view_sum_ex_kernel<bf16_t><<<nblocks(total, 256), 256, 0, s>>>(X, mask, B, V, Nq, C, base, Y,
                                                                              (bf16_t*)Yl, (bf16_t*)Yp);
    return cmt_check_launch("cmt_masked_view_sum_ex");
}

extern "C" int cmt_nchw_to_rows_ex(const float* X, int nb, int nv, int C, int HW, void* Y, int ydtype, int64_t ldy,
                                   int64_t rows_per_batch, int64_t row_offset, int* range_flag, void* stream);

extern "C" int cmt_nchw_to_rows(const float* X, int nb, int nv, int C, int HW, void* Y, int ydtype, int64_t ldy,
                                int64_t rows_per_batch, int64_t row_offset, void* stream) {
    return cmt_nchw_to_rows_ex(X, nb, nv, C, HW, Y, ydtype, ldy, rows_per_batch, row_offset, nullptr, stream);
}

extern "C" int cmt_nchw_to_rows_ex(const float* X, int nb, int nv, int C, int HW, void* Y, int ydtype, int64_t ldy,
                                   int64_t rows_per_batch, int64_t row_offset, int* range_flag, void* stream) {
    CMT_REQUIRE(X && Y && nb > 0 && nv > 0 && C > 0 && HW > 0, "cmt_nchw_to_rows: bad arguments");
    dim3 grid(cdiv(HW, 64), cdiv(C, 64), nb * nv);
    hipStream_t s = (hipStream_t)stream;
    const int esz = ydtype == CMT_F32 ? 4 : 2;
    if (ydtype == CMT_F16P) {
        CMT_REQUIRE(ldy == 2 * C, "cmt_nchw_to_rows: f16-pair rows need ldy == 2C (hi row, then lo row)");
        if (HW % 4 == 0 && C % 64 == 0 && (uintptr_t)Y % 16 == 0 && (uintptr_t)X % 16 == 0)
            nchw_to_rows_vec_kernel<pair_t, true><<<grid, 256, 0, s>>>(X, nv, C, HW, (pair_t*)Y, ldy, rows_per_batch,
                                                                       row_offset, range_flag);
        else
            nchw_to_rows_kernel<pair_t, true><<<grid, 256, 0, s>>>(X, nv, C, HW, (pair_t*)Y, ldy, rows_per_batch,
                                                                   row_offset, range_flag);
        return cmt_check_launch("cmt_nchw_to_rows");
    }
    if (HW % 4 == 0 && C % 64 == 0 && (ldy * esz) % 16 == 0 && (uintptr_t)Y % 16 == 0 && (uintptr_t)X % 16 == 0 &&
        (ydtype == CMT_F32 || ydtype == CMT_F16 || ydtype == CMT_BF16)) {
        if (ydtype == CMT_F32)
            nchw_to_rows_vec_kernel<float><<<grid, 256, 0, s>>>(X, nv, C, HW, (float*)Y, ldy, rows_per_batch,
                                                                row_offset, range_flag);
        else if (ydtype == CMT_F16)
            nchw_to_rows_vec_kernel<f16_t><<<grid, 256, 0, s>>>(X, nv, C, HW, (f16_t*)Y, ldy, rows_per_batch,
                                                                row_offset, range_flag);
        else
            nchw_to_rows_vec_kernel<bf16_t><<<grid, 256, 0, s>>>(X, nv, C, HW, (bf16_t*)Y, ldy, rows_per_batch,
                                                                 row_offset, range_flag);
        return cmt_check_launch("cmt_nchw_to_rows");
    }
    if (ydtype == CMT_F32)
        nchw_to_rows_kernel<float><<<grid, 256, 0, s>>>(X, nv, C, HW, (float*)Y, ldy, rows_per_batch, row_offset, range_flag);
    else if (ydtype == CMT_F16)
        nchw_to_rows_kernel<f16_t><<<grid, 256, 0, s>>>(X, nv, C, HW, (f16_t*)Y, ldy, rows_per_batch, row_offset, range_flag);
    else if (ydtype == CMT_BF16)
        nchw_to_rows_kernel<bf16_t><<<grid, 256, 0, s>>>(X, nv, C, HW, (bf16_t*)Y, ldy, rows_per_batch, row_offset, range_flag);
    else
        return cmt_fail(CMT_EINVAL, "cmt_nchw_to_rows: bad ydtype");
    return cmt_check_launch("cmt_nchw_to_rows");
}

extern "C" int cmt_split_rows(const float* X, int64_t ldx, int64_t rows, int C, void* Y, void* stream) {
    CMT_REQUIRE(X && Y && rows >= 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0 && (uintptr_t)X % 16 == 0 &&
                    (uintptr_t)Y % 8 == 0, "cmt_split_rows: bad arguments");
    const int64_t n4 = rows * (C / 4);
    if (n4 == 0) return 0;
    split_rows_kernel<<<nblocks(n4, 256), 256, 0, (hipStream_t)stream>>>(X, ldx, n4, C, (pair_t*)Y);
    return cmt_check_launch("cmt_split_rows");
}

extern "C" int cmt_cast(const void* X, int xdtype, void* Y, int ydtype, int64_t n, void* stream) {
    CMT_REQUIRE(X && Y && n >= 0, "cmt_cast: bad arguments");
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = nblocks(n, 256);
#define CAST(TI, TO) cast_kernel<TI, TO><<<g, 256, 0, s>>>((const TI*)X, (TO*)Y, n)
    if (xdtype == CMT_F32 && ydtype == CMT_BF16) CAST(float, bf16_t);
    else if (xdtype == CMT_F32 && ydtype == CMT_F16) CAST(float, f16_t);
    else if (xdtype == CMT_F32 && ydtype == CMT_F32) CAST(float, float);
    else if (xdtype == CMT_BF16 && ydtype == CMT_F32) CAST(bf16_t, float);
    else if (xdtype == CMT_F16 && ydtype == CMT_F32) CAST(f16_t, float);
    else return cmt_fail(CMT_EINVAL, "cmt_cast: unsupported dtype pair");
#undef CAST
    return cmt_check_launch("cmt_cast");
}

extern "C" int cmt_task_head_tail(const float* H1, int L, int B, int Nq, int nheads, int hc, const float* gln_w,
                                  const float* gln_b, const float* W2, const float* B2, const int* head_out,
                                  int out_total, int k, const float* ref, int center_col, int height_col,
                                  const float* pc_range6, float* OUT, void* stream) {
    CMT_REQUIRE(H1 && gln_w && gln_b && W2 && B2 && head_out && ref && pc_range6 && OUT,
                "cmt_task_head_tail: null pointer");
    CMT_REQUIRE(hc == 64, "cmt_task_head_tail: head_conv must be 64");
    CMT_REQUIRE(nheads > 0 && nheads <= 16 && out_total > 0 && out_total <= 64 && (k == 1 || k == 3),
                "cmt_task_head_tail: unsupported head geometry");
    hipStream_t s = (hipStream_t)stream;
    TailParams p;
    p.G = H1; p.L = L; p.B = B; p.Nq = Nq; p.nheads = nheads; p.hc = hc;
    p.gw = gln_w; p.gb = gln_b;
    p.W2 = W2; p.B2 = B2; p.out_total = out_total; p.k = k;
    p.ref = ref; p.center_col = center_col; p.height_col = height_col;
    for (int i = 0; i < 6; ++i) p.pc[i] = pc_range6[i];
    p.OUT = OUT;
    int o = 0;
    for (int hd = 0; hd < nheads; ++hd) {
        for (int j = 0; j < head_out[hd]; ++j) {
            if (o >= 64) return cmt_fail(CMT_EINVAL, "cmt_task_head_tail: too many outputs");
            p.head_of[o++] = hd;
        }
    }
    CMT_REQUIRE(o == out_total, "cmt_task_head_tail: head_out does not sum to out_total");
    const int width = nheads * hc;
    const size_t smem = sizeof(float) * ((size_t)(TQ + 2 * (k >> 1)) * (width + 4) + (size_t)out_total * k * (hc + 4));
    CMT_REQUIRE(smem <= 160 * 1024, "cmt_task_head_tail: head too wide for LDS staging");
    dim3 g2(L, cdiv(Nq, TQ), B);
    task_head_tail_kernel<<<g2, 256, smem, s>>>(p);
    return cmt_check_launch("cmt_task_head_tail");
}
