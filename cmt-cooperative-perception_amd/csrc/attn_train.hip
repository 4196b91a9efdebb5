// Attention forward-with-statistics and backward for the training path
// (exact f32, v_mfma_f32_32x32x2_f32, head_dim 32).  Reference: the
// self-attention nn.MultiheadAttention (mmcv MultiheadAttention, with the
// training-time DN mask of cmt_head.py:386-398 and attn_drop) and the
// FlashMHA cross-attention core (attention.py:46-92, flash-attn 0.2.2 fp16
// core: fp16_inputs rounds q, k, v, P and O to fp16 as that core does).
//
// Forward: one wave per 32 queries, 4 waves per workgroup share 64-key K/V
// tiles in LDS (padded rows), swapped S^T = K Q^T so a lane owns one query,
// online softmax in exp2 units, key range split over workgroups (combine
// kernel) so ~1000-query problems fill the chip.  Writes O and the row
// statistic LSE2 = m + log2(l) (exp2 units of c = scale * log2 e).
//
// Backward (flash-style, P recomputed from LSE2, delta = rowsum(dO * O)):
//   dq kernel   one wave per 32 queries over a key slice:  S^T, dP^T = V dO^T,
//               dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T  (f32 atomics into dQ
//               when the key range is split)
//   dkv kernel  one wave per 32 keys over all queries: S = Q K^T, dV^T += dO^T P,
//               dP = dO V^T, dS = P (dP - delta), dK^T += Q^T dS
// Every product is a chain of 32x32x2 MFMAs whose accumulator layout is the
// next product's B operand (lane = the free index, register pairs = the
// contraction index), so no tile is transposed through LDS.
//
// DN mask (dn_pad > 0): key k is hidden from query q if k < dn_pad and
// (q >= dn_pad or k / dn_group != q / dn_group).  Dropout (p > 0) keeps
// P(q, k) with probability 1 - p by a counter hash of (seed, b, h, q, k),
// recomputed identically in the backward.
#include "cmt_common.h"

#include <cstdlib>

namespace {

constexpr int D = 32;
constexpr int KT = 64;
constexpr int LDK = 36;      // padded f32 LDS row
constexpr float LOG2E = 1.4426950408889634f;

struct AP {                  // device-side copy of cmt_attn_train_args + derived values
    cmt_attn_train_args a;
    float c;                 // scale * log2(e)
    int tiles_per_split;
    float keep_scale;        // 1 / (1 - p)
    uint32_t drop_thr;       // keep iff hash >= thr
};

__device__ __forceinline__ float r16(float x) { return (float)(_Float16)x; }

// dev diagnostic bits (dev/build_exp.sh -DCMT_AT_VAR=n; the product builds 0): 2 / 4 = no dropout
// hash / no DN mask (wrong results, for timing what each costs: dev/attn_train_probe.py)
#ifndef CMT_AT_VAR
#define CMT_AT_VAR 0
#endif
// exp2 as one v_exp_f32 (exp2f adds denormal range scaling around it): the exact-f32 kernels'
// softmax arguments are <= 0 and a flushed denormal P is below every tolerance of the step
// (profiles/r6_experiments.txt r6f: 70.8 -> 66.7 us forward at the coop self-attention shape)
__device__ __forceinline__ float xexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bool masked(const cmt_attn_train_args& a, int q, int k) {
    if (a.dn_pad <= 0 || k >= a.dn_pad) return false;
    return q >= a.dn_pad || (k / a.dn_group) != (q / a.dn_group);
}

// masked() without a per-element integer division: the DN groups tile [0, dn_pad) (dn_pad is a
// multiple of dn_group), so for a FIXED query q the keys it sees below dn_pad are its own group
// [lo, hi) (none when q >= dn_pad), and for a FIXED key k < dn_pad the queries that see it are
// k's group.  One division per lane; per element two or three compares.
struct DnRange {
    int lo, hi;
};
// the lane's query q: key k is hidden iff dn_hidden_key(a, r, k)
__device__ __forceinline__ DnRange dn_query_range(const cmt_attn_train_args& a, int q) {
    if (a.dn_pad <= 0 || q >= a.dn_pad) return DnRange{0, 0};
    const int lo = (q / a.dn_group) * a.dn_group;
    return DnRange{lo, min(lo + a.dn_group, a.dn_pad)};
}
__device__ __forceinline__ bool dn_hidden_key(const cmt_attn_train_args& a, const DnRange& r, int k) {
    if constexpr ((CMT_AT_VAR & 4) != 0) return false;
    return k < a.dn_pad && (k < r.lo || k >= r.hi);
}
// the lane's key k: query q is hidden from it iff dn_hidden_query(r, q)
__device__ __forceinline__ DnRange dn_key_range(const cmt_attn_train_args& a, int k) {
    if (a.dn_pad <= 0 || k >= a.dn_pad) return DnRange{INT_MIN, INT_MAX};
    const int lo = (k / a.dn_group) * a.dn_group;
    return DnRange{lo, min(lo + a.dn_group, a.dn_pad)};
}
__device__ __forceinline__ bool dn_hidden_query(const DnRange& r, int q) {
    if constexpr ((CMT_AT_VAR & 4) != 0) return false;
    return q < r.lo || q >= r.hi;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// the dropout seed of the launch: seed (+ *seed_dev, ABI 22), resolved once per kernel into p.a.seed
__device__ __forceinline__ void resolve_seed(AP& p) {
    if (p.a.seed_dev) p.a.seed += *p.a.seed_dev;
}
__device__ __forceinline__ bool keep(const AP& p, int bh, int q, int k) {
    if constexpr ((CMT_AT_VAR & 2) != 0) return true;
    uint32_t h = mix32(p.a.seed ^ mix32((uint32_t)bh * 0x9e3779b9U + (uint32_t)q));
    h = mix32(h ^ (uint32_t)k * 0x85ebca6bU);
    return h >= p.drop_thr;
}

__device__ __forceinline__ int key_of(int r, int lh) { return (r & 3) + 8 * (r >> 2) + 4 * lh; }

// stage a 64-row x 32 tile of X (row stride rs) into LDS rows of LDK floats
__device__ __forceinline__ void stage64(float* lds, const float* X, int64_t rs, int r0, int nrows, bool f16, int tid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int idx = tid + 256 * i;
        const int r = idx >> 3, c = (idx & 7) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r0 + r < nrows) v = *(const f32x4*)(X + (int64_t)(r0 + r) * rs + c);
        if (f16)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = r16(v[j]);
        *(f32x4*)(lds + r * LDK + c) = v;
    }
}

// acc (+)= X_rows . Y^T over d: lane supplies row (l & 31) of X (LDS, 32 rows
// starting at xr) and Y fragments yf[4] (its own row, d = 16*lh + 4i + j)
__device__ __forceinline__ void mma_rows(f32x16& acc, const float* xrow, const f32x4 (&yf)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x4 xv = *(const f32x4*)(xrow + 4 * i);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[j], yf[i][j], acc, 0, 0, 0);
    }
}

// acc^T[d][col] += sum_k Z[k][d] * W[k][col] where W is an accumulator tile
// (lane = col, register r <-> k = key_of(r, lh) + base) and Z rows are in LDS
__device__ __forceinline__ void mma_acc(f32x16& acc, const float* zbase, const f32x16& w, int lane) {
    const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zbase[key_of(r, lh) * LDK + lr], w[r], acc, 0, 0, 0);
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void train_fwd_kernel(AP p) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) float Ks[KT * LDK];
    __shared__ __attribute__((aligned(16))) float Vs[KT * LDK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H, split = blockIdx.z;
    const bool f16 = a.fp16_inputs != 0;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const int q = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_query_range(a, q);
    const int qc = min(q, a.Nq - 1);
    f32x4 qf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        qf[i] = *(const f32x4*)(Qb + (int64_t)qc * a.q_rs + 16 * lh + 4 * i);
        if (f16)
#pragma unroll
            for (int j = 0; j < 4; ++j) qf[i][j] = r16(qf[i][j]);
    }
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
    float m_run = -__builtin_inff(), l_run = 0.f;
    for (int t = t0; t < t1; ++t) {
        __syncthreads();
        stage64(Ks, Kb, a.k_rs, t * KT, a.Nk, f16, tid);
        stage64(Vs, Vb, a.v_rs, t * KT, a.Nk, f16, tid);
        __syncthreads();
        f32x16 s[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
            mma_rows(s[kb], Ks + (kb * 32 + lr) * LDK + 16 * lh, qf);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = t * KT + kb * 32 + key_of(r, lh);
                s[kb][r] = (k >= a.Nk || dn_hidden_key(a, dnr, k)) ? -__builtin_inff() : s[kb][r] * p.c;
            }
        }
        float mt = -__builtin_inff();
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kb][r]);
        mt = fmaxf(mt, __shfl_xor(mt, 32));
        const float m_new = fmaxf(m_run, mt);
        const float m_use = m_new == -__builtin_inff() ? 0.f : m_new;   // fully masked so far
        const float alpha = xexp2(m_run - m_use);
        float ls = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = xexp2(s[kb][r] - m_use);
                ls += e;
                float pe = f16 ? r16(e) : e;
                if (a.dropout_p > 0.f) {
                    const int k = t * KT + kb * 32 + key_of(r, lh);
                    pe = keep(p, bh, q, k) ? pe * p.keep_scale : 0.f;
                }
                s[kb][r] = pe;
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= alpha;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) mma_acc(o, Vs + kb * 32 * LDK, s[kb], lane);
    }
    const float l_tot = l_run + __shfl_xor(l_run, 32);
    if (q >= a.Nq) return;
    if (a.kv_splits <= 1) {
        const float inv = 1.f / l_tot;
        float* Ob = a.O + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs + (int64_t)q * a.o_rs;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = o[r] * inv;
            Ob[key_of(r, lh)] = f16 ? r16(v) : v;
        }
        if (lh == 0) a.LSE[(int64_t)bh * a.Nq + q] = m_run + log2f(l_tot);
    } else {
        float* ws = (float*)a.workspace;
        const int64_t rows = (int64_t)a.B * a.H * a.Nq;
        const int64_t row = (int64_t)split * rows + (int64_t)bh * a.Nq + q;
        float* Op = ws + row * D;
#pragma unroll
        for (int r = 0; r < 16; ++r) Op[key_of(r, lh)] = o[r];
        if (lh == 0) {
            ws[(int64_t)a.kv_splits * rows * D + row] = m_run;
            ws[(int64_t)a.kv_splits * rows * (D + 1) + row] = l_tot;
        }
    }
}

__global__ __launch_bounds__(256) void train_combine_kernel(AP p) {
    const cmt_attn_train_args& a = p.a;
    const int64_t rows = (int64_t)a.B * a.H * a.Nq;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rows * D) return;
    const int64_t row = i / D;
    const int d = (int)(i - row * D);
    const float* ws = (const float*)a.workspace;
    const int S = a.kv_splits;
    float M = -__builtin_inff();
    for (int s = 0; s < S; ++s) {
        const float l = ws[(int64_t)S * rows * (D + 1) + s * rows + row];
        if (l > 0.f) M = fmaxf(M, ws[(int64_t)S * rows * D + s * rows + row]);
    }
    float num = 0.f, den = 0.f;
    for (int s = 0; s < S; ++s) {
        const float l = ws[(int64_t)S * rows * (D + 1) + s * rows + row];
        if (!(l > 0.f)) continue;
        const float w = xexp2(ws[(int64_t)S * rows * D + s * rows + row] - M);
        num += w * ws[(s * rows + row) * D + d];
        den += w * l;
    }
    const int bh = (int)(row / a.Nq), q = (int)(row - (int64_t)bh * a.Nq);
    const int b = bh / a.H, h = bh - b * a.H;
    const float v = num / den;
    a.O[(int64_t)b * a.o_bs + (int64_t)h * a.o_hs + (int64_t)q * a.o_rs + d] = a.fp16_inputs ? r16(v) : v;
    if (d == 0) a.LSE[row] = M + log2f(den);
}

// delta[b,h,q] = sum_d dO * O
__global__ __launch_bounds__(256) void train_delta_kernel(AP p) {
    const cmt_attn_train_args& a = p.a;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= (int64_t)a.B * a.H * a.Nq) return;
    const int bh = (int)(row / a.Nq), q = (int)(row - (int64_t)bh * a.Nq);
    const int b = bh / a.H, h = bh - b * a.H;
    const int64_t off = (int64_t)b * a.o_bs + (int64_t)h * a.o_hs + (int64_t)q * a.o_rs;
    float v = lane < D ? a.dO[off + lane] * a.O[off + lane] : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) a.delta[row] = v;
}

// dQ: waves own 32 queries; key tiles [t0, t1) of this split; f32 atomics into dQ
__global__ __launch_bounds__(256) void train_dq_kernel(AP p) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) float Ks[KT * LDK];
    __shared__ __attribute__((aligned(16))) float Vs[KT * LDK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H, split = blockIdx.z;
    const bool f16 = a.fp16_inputs != 0;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const float* dOb = a.dO + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
    const int q = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_query_range(a, q);
    const int qc = min(q, a.Nq - 1);
    f32x4 qf[4], df[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        qf[i] = *(const f32x4*)(Qb + (int64_t)qc * a.q_rs + 16 * lh + 4 * i);
        df[i] = *(const f32x4*)(dOb + (int64_t)qc * a.o_rs + 16 * lh + 4 * i);
        if (f16)
#pragma unroll
            for (int j = 0; j < 4; ++j) qf[i][j] = r16(qf[i][j]);
    }
    const float lse = a.LSE[(int64_t)bh * a.Nq + qc];
    const float dl = a.delta[(int64_t)bh * a.Nq + qc];
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);
    f32x16 dq;
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[r] = 0.f;
    for (int t = t0; t < t1; ++t) {
        __syncthreads();
        stage64(Ks, Kb, a.k_rs, t * KT, a.Nk, f16, tid);
        stage64(Vs, Vb, a.v_rs, t * KT, a.Nk, f16, tid);
        __syncthreads();
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 s, dp;
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
            mma_rows(s, Ks + (kb * 32 + lr) * LDK + 16 * lh, qf);     // S^T  (lane = query)
            mma_rows(dp, Vs + (kb * 32 + lr) * LDK + 16 * lh, df);    // dP^T = V dO^T
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = t * KT + kb * 32 + key_of(r, lh);
                float pr = (k >= a.Nk || dn_hidden_key(a, dnr, k)) ? 0.f : xexp2(s[r] * p.c - lse);
                float g = dp[r];
                if (a.dropout_p > 0.f) g = keep(p, bh, q, k) ? g * p.keep_scale : 0.f;
                s[r] = pr * (g - dl);                                    // dS^T
            }
            mma_acc(dq, Ks + kb * 32 * LDK, s, lane);                    // dQ^T += K^T dS^T
        }
    }
    if (q >= a.Nq) return;
    float* dQb = a.dQ + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs + (int64_t)q * a.q_rs;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float v = dq[r] * a.scale;
        if (a.kv_splits > 1) atomicAdd(dQb + key_of(r, lh), v);
        else dQb[key_of(r, lh)] = v;
    }
}

// dK, dV: waves own 32 keys; loop over 64-query tiles (Q, dO, LSE2, delta in LDS), query tiles
// [z qt_per, (z + 1) qt_per) of split z = blockIdx.z (f32 atomics into zeroed dK / dV when split:
// the self-attention's ~1 100 keys alone are 9 x 8 workgroups)
__global__ __launch_bounds__(256) void train_dkv_kernel(AP p, int qt_per) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) float Qs[KT * LDK];
    __shared__ __attribute__((aligned(16))) float Ds[KT * LDK];
    __shared__ float Ls[KT], Dl[KT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const bool f16 = a.fp16_inputs != 0;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const float* dOb = a.dO + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
    const int k = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_key_range(a, k);
    const int kc = min(k, a.Nk - 1);
    f32x4 kf[4], vf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        kf[i] = *(const f32x4*)(Kb + (int64_t)kc * a.k_rs + 16 * lh + 4 * i);
        vf[i] = *(const f32x4*)(Vb + (int64_t)kc * a.v_rs + 16 * lh + 4 * i);
        if (f16)
#pragma unroll
            for (int j = 0; j < 4; ++j) { kf[i][j] = r16(kf[i][j]); vf[i][j] = r16(vf[i][j]); }
    }
    f32x16 dk, dv;
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[r] = dv[r] = 0.f;
    const int nqt = (a.Nq + KT - 1) / KT;
    const int tq0 = blockIdx.z * qt_per, tq1 = min(nqt, tq0 + qt_per);
    for (int t = tq0; t < tq1; ++t) {
        __syncthreads();
        stage64(Qs, Qb, a.q_rs, t * KT, a.Nq, f16, tid);
        stage64(Ds, dOb, a.o_rs, t * KT, a.Nq, false, tid);
        if (tid < KT) {
            const int qq = min(t * KT + tid, a.Nq - 1);
            Ls[tid] = a.LSE[(int64_t)bh * a.Nq + qq];
            Dl[tid] = a.delta[(int64_t)bh * a.Nq + qq];
        }
        __syncthreads();
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            f32x16 s, dp;
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
            mma_rows(s, Qs + (qb * 32 + lr) * LDK + 16 * lh, kf);     // S = Q K^T (lane = key)
            mma_rows(dp, Ds + (qb * 32 + lr) * LDK + 16 * lh, vf);    // dP = dO V^T
            f32x16 pd;                                                 // dropped P (dV operand)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int qi = qb * 32 + key_of(r, lh), qq = t * KT + qi;
                const bool valid = qq < a.Nq && k < a.Nk && !dn_hidden_query(dnr, qq);
                const float pr = valid ? xexp2(s[r] * p.c - Ls[qi]) : 0.f;
                float g = dp[r], pe = f16 ? r16(pr) : pr;
                if (a.dropout_p > 0.f) {
                    const bool kp = keep(p, bh, qq, k);
                    g = kp ? g * p.keep_scale : 0.f;
                    pe = kp ? pe * p.keep_scale : 0.f;
                }
                pd[r] = pe;
                s[r] = pr * (g - Dl[qi]);                              // dS
            }
            mma_acc(dv, Ds + qb * 32 * LDK, pd, lane);                 // dV^T += dO^T P
            mma_acc(dk, Qs + qb * 32 * LDK, s, lane);                  // dK^T += Q^T dS
        }
    }
    if (k >= a.Nk) return;
    float* dKb = a.dK + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs + (int64_t)k * a.k_rs;
    float* dVb = a.dV + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs + (int64_t)k * a.v_rs;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (gridDim.z > 1) {
            atomicAdd(dKb + key_of(r, lh), dk[r] * a.scale);
            atomicAdd(dVb + key_of(r, lh), dv[r]);
        } else {
            dKb[key_of(r, lh)] = dk[r] * a.scale;
            dVb[key_of(r, lh)] = dv[r];
        }
    }
}

// ---------------------------------------------------------------------------
// f16 MFMA forms of the three kernels for the flash-attn fp16 core
// (fp16_inputs): q, k, v, dO, P and dS enter every product as f16 -- the
// operands flash-attn 0.2.2's fp16 forward / backward multiply -- on
// v_mfma_f32_32x32x16_f16 (16x the rate of the f32 MFMA), fp32 accumulate;
// softmax statistics, dS = P (dP - delta) and every accumulator stay fp32.
// Tiles of 64 keys (queries in the dK/dV kernel) are staged in LDS as f16,
// row-major [row][32 d] (16-byte chunks XOR-swizzled by (row >> 2) & 3: the
// 16-lane groups of ds_read_b128 hit distinct bank slots) and, where a tile is
// the A operand of a product over its rows, transposed [32 d][64 rows].  A
// product whose B operand is an accumulator tile (P^T, dS^T, P, dS) takes the
// accumulator's own row order as its k order: register 8 ss + j of lane half
// lh is row (j & 3) + 16 ss + 8 (j >> 2) + 4 lh, and the transposed A reads
// the same rows as two 4-element runs.
// MASK: the DN mask can hide keys; DROP: dropout (counter hash, as above); the
// dropout scale 1 / (1 - p) multiplies O, dV and dP' once instead of each P.
// ---------------------------------------------------------------------------
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
constexpr int RMB = 64;    // bytes per row-major LDS row (32 d)
constexpr int TRB = 128;   // bytes per transposed LDS row (64 rows)

__device__ __forceinline__ int rm_off(int row, int chunk) { return row * RMB + ((chunk ^ ((row >> 2) & 3)) << 4); }

// stage rows r0 .. r0+63 of X (fp32, row stride rs; rows >= nrows are zero) as f16
// into the row-major image rm and / or the transposed image tr
__device__ __forceinline__ void stage16(char* rm, char* tr, const float* X, int64_t rs, int r0, int nrows, int tid) {
    const int r = tid >> 2, c = tid & 3;
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
    if (r0 + r < nrows) {
        a = *(const f32x4*)(X + (int64_t)(r0 + r) * rs + 8 * c);
        b = *(const f32x4*)(X + (int64_t)(r0 + r) * rs + 8 * c + 4);
    }
    h8_t hv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        hv[j] = (_Float16)a[j];
        hv[4 + j] = (_Float16)b[j];
    }
    if (rm) *(h8_t*)(rm + rm_off(r, c)) = hv;
    if (tr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) *(_Float16*)(tr + (8 * c + j) * TRB + 2 * r) = hv[j];
    }
}

// A fragment of rows rb*32 + (lane & 31) of a row-major image, d half kk
__device__ __forceinline__ h8_t frag_rm(const char* rm, int rb, int kk, int lane) {
    return *(const h8_t*)(rm + rm_off(rb * 32 + (lane & 31), 2 * kk + (lane >> 5)));
}
// A fragment of a transposed image: row d = lane & 31, the 8 rows of k half ss of block rb
// in the accumulator order (two 4-element runs)
__device__ __forceinline__ h8_t frag_tr(const char* tr, int rb, int ss, int lane) {
    const char* base = tr + (lane & 31) * TRB + 2 * (rb * 32 + 16 * ss + 4 * (lane >> 5));
    const h4_t lo = *(const h4_t*)base, hi = *(const h4_t*)(base + 16);
    return h8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// B fragment from accumulator registers 8 ss .. 8 ss + 7 (rounded to f16)
__device__ __forceinline__ h8_t frag_acc(const f32x16& x, int ss) {
    h8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (_Float16)x[8 * ss + j];
    return v;
}
// a lane's own row of 32 fp32 values as the two B fragments (d = 16 kk + 8 lh + j)
__device__ __forceinline__ void own_row16(const float* row, int lh, h8_t (&f)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const f32x4 a = *(const f32x4*)(row + 16 * kk + 8 * lh), b = *(const f32x4*)(row + 16 * kk + 8 * lh + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f[kk][j] = (_Float16)a[j];
            f[kk][4 + j] = (_Float16)b[j];
        }
    }
}
__device__ __forceinline__ f32x16 mma16(h8_t a, h8_t b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <bool MASK, bool DROP>
__global__ __launch_bounds__(256) void train16_fwd_kernel(AP p) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) char Ks[KT * RMB];   // [key][d]
    __shared__ __attribute__((aligned(16))) char Vt[D * TRB];    // [d][key]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H, split = blockIdx.z;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const int q = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_query_range(a, q);
    const int qc = min(q, a.Nq - 1);
    h8_t qf[2];
    own_row16(Qb + (int64_t)qc * a.q_rs, lh, qf);
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
    float m_run = -__builtin_inff(), l_run = 0.f;
    for (int t = t0; t < t1; ++t) {
        __syncthreads();
        stage16(Ks, nullptr, Kb, a.k_rs, t * KT, a.Nk, tid);
        stage16(nullptr, Vt, Vb, a.v_rs, t * KT, a.Nk, tid);
        __syncthreads();
        const bool edge = (t + 1) * KT > a.Nk;
        f32x16 s[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) s[kb] = mma16(frag_rm(Ks, kb, kk, lane), qf[kk], s[kb]);   // S^T
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = t * KT + kb * 32 + key_of(r, lh);
                const bool hide = (edge && k >= a.Nk) || (MASK && dn_hidden_key(a, dnr, k));
                s[kb][r] = hide ? -__builtin_inff() : s[kb][r] * p.c;
            }
        }
        float mt = -__builtin_inff();
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kb][r]);
        mt = fmaxf(mt, __shfl_xor(mt, 32));
        const float m_new = fmaxf(m_run, mt);
        const float m_use = m_new == -__builtin_inff() ? 0.f : m_new;   // fully masked so far
        const float alpha = exp2f(m_run - m_use);
        float ls = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = exp2f(s[kb][r] - m_use);
                ls += e;
                float pe = e;
                if (DROP) {
                    const int k = t * KT + kb * 32 + key_of(r, lh);
                    pe = keep(p, bh, q, k) ? pe : 0.f;
                }
                s[kb][r] = pe;
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= alpha;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) o = mma16(frag_tr(Vt, kb, ss, lane), frag_acc(s[kb], ss), o);   // O^T += V^T P^T
    }
    const float l_tot = l_run + __shfl_xor(l_run, 32);
    if (DROP) {
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= p.keep_scale;
    }
    if (q >= a.Nq) return;
    if (a.kv_splits <= 1) {
        const float inv = 1.f / l_tot;
        float* Ob = a.O + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs + (int64_t)q * a.o_rs;
#pragma unroll
        for (int r = 0; r < 16; ++r) Ob[key_of(r, lh)] = r16(o[r] * inv);
        if (lh == 0) a.LSE[(int64_t)bh * a.Nq + q] = m_run + log2f(l_tot);
    } else {
        float* ws = (float*)a.workspace;
        const int64_t rows = (int64_t)a.B * a.H * a.Nq;
        const int64_t row = (int64_t)split * rows + (int64_t)bh * a.Nq + q;
        float* Op = ws + row * D;
#pragma unroll
        for (int r = 0; r < 16; ++r) Op[key_of(r, lh)] = o[r];
        if (lh == 0) {
            ws[(int64_t)a.kv_splits * rows * D + row] = m_run;
            ws[(int64_t)a.kv_splits * rows * (D + 1) + row] = l_tot;
        }
    }
}

template <bool MASK, bool DROP>
__global__ __launch_bounds__(256) void train16_dq_kernel(AP p) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) char Ks[KT * RMB];   // [key][d]
    __shared__ __attribute__((aligned(16))) char Kt[D * TRB];    // [d][key]
    __shared__ __attribute__((aligned(16))) char Vs[KT * RMB];   // [key][d]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H, split = blockIdx.z;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const float* dOb = a.dO + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
    const int q = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_query_range(a, q);
    const int qc = min(q, a.Nq - 1);
    h8_t qf[2], df[2];
    own_row16(Qb + (int64_t)qc * a.q_rs, lh, qf);
    own_row16(dOb + (int64_t)qc * a.o_rs, lh, df);
    const float lse = a.LSE[(int64_t)bh * a.Nq + qc];
    const float dl = a.delta[(int64_t)bh * a.Nq + qc];
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);
    f32x16 dq;
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[r] = 0.f;
    for (int t = t0; t < t1; ++t) {
        __syncthreads();
        stage16(Ks, Kt, Kb, a.k_rs, t * KT, a.Nk, tid);
        stage16(Vs, nullptr, Vb, a.v_rs, t * KT, a.Nk, tid);
        __syncthreads();
        const bool edge = (t + 1) * KT > a.Nk;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 s, dp;
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                s = mma16(frag_rm(Ks, kb, kk, lane), qf[kk], s);      // S^T
                dp = mma16(frag_rm(Vs, kb, kk, lane), df[kk], dp);    // dP^T = V dO^T
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = t * KT + kb * 32 + key_of(r, lh);
                const bool hide = (edge && k >= a.Nk) || (MASK && dn_hidden_key(a, dnr, k));
                const float pr = hide ? 0.f : exp2f(s[r] * p.c - lse);
                float g = dp[r];
                if (DROP) g = keep(p, bh, q, k) ? g * p.keep_scale : 0.f;
                s[r] = pr * (g - dl);                                   // dS^T
            }
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) dq = mma16(frag_tr(Kt, kb, ss, lane), frag_acc(s, ss), dq);   // dQ^T += K^T dS^T
        }
    }
    if (q >= a.Nq) return;
    float* dQb = a.dQ + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs + (int64_t)q * a.q_rs;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float v = dq[r] * a.scale;
        if (a.kv_splits > 1) atomicAdd(dQb + key_of(r, lh), v);
        else dQb[key_of(r, lh)] = v;
    }
}

template <bool MASK, bool DROP>
__global__ __launch_bounds__(256) void train16_dkv_kernel(AP p) {
    resolve_seed(p);
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) char Qs[KT * RMB];   // [q][d]
    __shared__ __attribute__((aligned(16))) char Qt[D * TRB];    // [d][q]
    __shared__ __attribute__((aligned(16))) char Ds[KT * RMB];   // dO [q][d]
    __shared__ __attribute__((aligned(16))) char Dt[D * TRB];    // dO [d][q]
    __shared__ float Ls[KT], Dl[KT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const float* Qb = a.Q + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const float* Kb = a.K + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs;
    const float* Vb = a.V + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs;
    const float* dOb = a.dO + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
    const int k = blockIdx.x * 128 + wave * 32 + lr;
    const DnRange dnr = dn_key_range(a, k);
    const int kc = min(k, a.Nk - 1);
    h8_t kf[2], vf[2];
    own_row16(Kb + (int64_t)kc * a.k_rs, lh, kf);
    own_row16(Vb + (int64_t)kc * a.v_rs, lh, vf);
    f32x16 dk, dv;
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[r] = dv[r] = 0.f;
    const int nqt = (a.Nq + KT - 1) / KT;
    for (int t = 0; t < nqt; ++t) {
        __syncthreads();
        stage16(Qs, Qt, Qb, a.q_rs, t * KT, a.Nq, tid);
        stage16(Ds, Dt, dOb, a.o_rs, t * KT, a.Nq, tid);
        if (tid < KT) {
            const int qq = min(t * KT + tid, a.Nq - 1);
            Ls[tid] = a.LSE[(int64_t)bh * a.Nq + qq];
            Dl[tid] = a.delta[(int64_t)bh * a.Nq + qq];
        }
        __syncthreads();
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            f32x16 s, dp;
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                s = mma16(frag_rm(Qs, qb, kk, lane), kf[kk], s);      // S = Q K^T (lane = key)
                dp = mma16(frag_rm(Ds, qb, kk, lane), vf[kk], dp);    // dP = dO V^T
            }
            f32x16 pd;                                                 // P, dropped (dV operand; scale later)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int qi = qb * 32 + key_of(r, lh), qq = t * KT + qi;
                const bool valid = qq < a.Nq && k < a.Nk && !(MASK && dn_hidden_query(dnr, qq));
                const float pr = valid ? exp2f(s[r] * p.c - Ls[qi]) : 0.f;
                float g = dp[r], pe = pr;
                if (DROP) {
                    const bool kp = keep(p, bh, qq, k);
                    g = kp ? g * p.keep_scale : 0.f;
                    pe = kp ? pe : 0.f;
                }
                pd[r] = pe;
                s[r] = pr * (g - Dl[qi]);                              // dS
            }
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                dv = mma16(frag_tr(Dt, qb, ss, lane), frag_acc(pd, ss), dv);   // dV^T += dO^T P
                dk = mma16(frag_tr(Qt, qb, ss, lane), frag_acc(s, ss), dk);    // dK^T += Q^T dS
            }
        }
    }
    if (k >= a.Nk) return;
    float* dKb = a.dK + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs + (int64_t)k * a.k_rs;
    float* dVb = a.dV + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs + (int64_t)k * a.v_rs;
    const float vs = DROP ? p.keep_scale : 1.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        dKb[key_of(r, lh)] = dk[r] * a.scale;
        dVb[key_of(r, lh)] = dv[r] * vs;
    }
}

// ---------------------------------------------------------------------------
// Long-key fp16 path (the cross-attention of the training step: FlashMHA's fp16
// core, no DN mask, no dropout; Nk of 36 400 / 44 400 keys against ~1 100
// queries).  The operands are first rounded to f16 ONCE into head-split copies
// [B][H][N][32] (to16_kernel, with the K projection's per-64-key max |k|^2 for
// the bounded forward), then:
//   forward   the inference core (attention.hip attn_pb2_kernel + split combine,
//             cmt_attn_fwd_lse) with the row statistic;
//   dK / dV   train16_dkv2_kernel: 8 waves x 32 keys, the head's whole Q and dO
//             (f16, <= 1 152 queries) resident in LDS -- no per-tile staging or
//             barrier; S and dP with the key on the lane, so P and dS are the B
//             operands of dV^T += dO^T P and dK^T += Q^T dS, whose A operands are
//             ds_read_b64_tr_b16 transposed reads of the same row-major images;
//   dQ        train16_dq2_kernel: 8 waves x 32 queries, K / V tiles by LDS-DMA
//             into a 4-slot ring (one barrier per tile), S^T and dP^T with the
//             query on the lane, dQ^T += K^T dS^T on transposed reads of the K
//             image, key splits summed by f32 atomics.
// Each f16 image row is 64 bytes with its 16-byte chunks XOR-swizzled by
// (row >> 2) & 3 (row reads and transposed reads both conflict-free).
// ---------------------------------------------------------------------------
constexpr int NQ_RES = 1152;   // queries resident in LDS (dkv2): 2 x 72 KB images + statistics
constexpr int DQ_RING = 4;

__device__ __forceinline__ int sw_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// A operand of a product over 16 rows [r0, r0 + 16) of a row-major swizzled image (the rows in
// the accumulator order of frag_acc): lane (lh, d = lane & 31) gets rows r0 + 4 lh + 0..3 and
// r0 + 8 + 4 lh + 0..3 of column d (two ds_read_b64_tr_b16, cdna_hip_programming.md T10)
__device__ __forceinline__ h8_t tr_frag(const char* img, int r0, int lane) {
    const int g = lane >> 4, lh = lane >> 5, qq = (lane & 15) >> 2, pp = lane & 3;
    const int c = 2 * (g & 1) + (pp >> 1);
    const int ra = r0 + 4 * lh + qq, rb = ra + 8;
    const char* pa = img + ra * 64 + ((c ^ ((ra >> 2) & 3)) << 4) + 8 * (pp & 1);
    const char* pb = img + rb * 64 + ((c ^ ((rb >> 2) & 3)) << 4) + 8 * (pp & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((CMT_LDS s16v4_lds*)pa);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((CMT_LDS s16v4_lds*)pb);
    s16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(h8_t, v);
}

// f16 head-split copy Y[(b H + h) N + n][32] of X[b bs + h hs + n rs + d]; with kmax2, also
// kmax2[e * H + h] = max over rows r = b N + n in [64 e, 64 e + 64) of |Y row|^2 (the rounded
// values: the bound of the forward's bounded offsets).  Block (e, h): 64 rows x 4 threads.
__global__ __launch_bounds__(256) void to16_kernel(const float* X, int64_t bs, int64_t hs, int64_t rs, int B, int H,
                                                   int N, f16_t* Y, float* kmax2) {
    const int e = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
    const int64_t r = (int64_t)e * 64 + (tid >> 2);
    const int d0 = (tid & 3) * 8;
    float ss = 0.f;
    if (r < (int64_t)B * N) {
        const int b = (int)(r / N), n = (int)(r - (int64_t)b * N);
        const float* x = X + (int64_t)b * bs + (int64_t)h * hs + (int64_t)n * rs + d0;
        const f32x4 u = *(const f32x4*)x, w = *(const f32x4*)(x + 4);
        h8_t v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = (f16_t)u[j];
            v[4 + j] = (f16_t)w[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += (float)v[j] * (float)v[j];
        *(h8_t*)(Y + (((int64_t)b * H + h) * N + n) * D + d0) = v;
    }
    if (kmax2 == nullptr) return;
    ss += __shfl_xor(ss, 1);
    ss += __shfl_xor(ss, 2);
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) ss = fmaxf(ss, __shfl_xor(ss, o));
    __shared__ float wm[4];
    if ((tid & 63) == 0) wm[tid >> 6] = ss;
    __syncthreads();
    if (tid == 0) kmax2[(int64_t)e * H + h] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

__global__ __launch_bounds__(512, 1) void train16_dkv2_kernel(AP p, const f16_t* Q16, const f16_t* D16,
                                                            const f16_t* K16, const f16_t* V16, int nqp) {
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) char Qs[NQ_RES * 64];
    __shared__ __attribute__((aligned(16))) char Ds[NQ_RES * 64];
    __shared__ __attribute__((aligned(16))) float Ls[NQ_RES];
    __shared__ __attribute__((aligned(16))) float Dl[NQ_RES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
    const f16_t* Qh = Q16 + (int64_t)bh * a.Nq * D;
    const f16_t* Dh = D16 + (int64_t)bh * a.Nq * D;
    // the head's Q and dO (padded rows zero) and statistics (padded rows: P = 0)
    for (int i = tid; i < nqp * 4; i += 512) {
        const int r = i >> 2, c = i & 3;
        h8_t qv = {}, dv = {};
        if (r < a.Nq) {
            qv = *(const h8_t*)(Qh + (int64_t)r * D + 8 * c);
            dv = *(const h8_t*)(Dh + (int64_t)r * D + 8 * c);
        }
        *(h8_t*)(Qs + sw_off(r, c)) = qv;
        *(h8_t*)(Ds + sw_off(r, c)) = dv;
    }
    for (int i = tid; i < nqp; i += 512) {
        Ls[i] = i < a.Nq ? a.LSE[(int64_t)bh * a.Nq + i] : __builtin_inff();
        Dl[i] = i < a.Nq ? a.delta[(int64_t)bh * a.Nq + i] : 0.f;
    }
    // this lane's key row of K and V as the B operands (k = d = 16 kk + 8 lh + j)
    const int k = blockIdx.x * 256 + wave * 32 + lr;
    const int kc = min(k, a.Nk - 1);
    const f16_t* Kr = K16 + ((int64_t)bh * a.Nk + kc) * D;
    const f16_t* Vr = V16 + ((int64_t)bh * a.Nk + kc) * D;
    h8_t kf[2], vf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        kf[kk] = *(const h8_t*)(Kr + 16 * kk + 8 * lh);
        vf[kk] = *(const h8_t*)(Vr + 16 * kk + 8 * lh);
    }
    __syncthreads();
    f32x16 dk, dv;
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[r] = dv[r] = 0.f;
    const float c = p.c;
    for (int q0 = 0; q0 < nqp; q0 += 32) {
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int o = sw_off(q0 + lr, 2 * kk + lh);
            s = mma16(*(const h8_t*)(Qs + o), kf[kk], s);      // S = Q K^T (lane = key)
            dp = mma16(*(const h8_t*)(Ds + o), vf[kk], dp);    // dP = dO V^T
        }
        // register r of lane half lh is query q0 + 8 (r >> 2) + 4 lh + (r & 3)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 L = *(const f32x4*)(Ls + q0 + 8 * g + 4 * lh);
            const f32x4 Dv = *(const f32x4*)(Dl + q0 + 8 * g + 4 * lh);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * g + e;
                const float pr = __builtin_amdgcn_exp2f(s[r] * c - L[e]);
                s[r] = pr;                                        // P
                dp[r] = pr * (dp[r] - Dv[e]);                     // dS
            }
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            dv = mma16(tr_frag(Ds, q0 + 16 * ss, lane), frag_acc(s, ss), dv);    // dV^T += dO^T P
            dk = mma16(tr_frag(Qs, q0 + 16 * ss, lane), frag_acc(dp, ss), dk);   // dK^T += Q^T dS
        }
    }
    if (k >= a.Nk) return;
    float* dKb = a.dK + (int64_t)b * a.k_bs + (int64_t)h * a.k_hs + (int64_t)k * a.k_rs;
    float* dVb = a.dV + (int64_t)b * a.v_bs + (int64_t)h * a.v_hs + (int64_t)k * a.v_rs;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        *(f32x4*)(dKb + 8 * g + 4 * lh) = f32x4{dk[4 * g] * a.scale, dk[4 * g + 1] * a.scale, dk[4 * g + 2] * a.scale,
                                                dk[4 * g + 3] * a.scale};
        *(f32x4*)(dVb + 8 * g + 4 * lh) = f32x4{dv[4 * g], dv[4 * g + 1], dv[4 * g + 2], dv[4 * g + 3]};
    }
}

__device__ __forceinline__ void dq2_wait(int n) {   // n = this wave's DMA pieces allowed in flight
    if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// QB query blocks of 32 per wave (8 / QB waves, 256 queries per workgroup): each K / V fragment
// read from LDS serves QB blocks (QB = 2 halves the LDS reads per query but needs 240 VGPRs:
// two waves per SIMD instead of four, measured slower -- the launcher uses QB = 1)
template <int QB>
__global__ __launch_bounds__(64 * (8 / QB)) void train16_dq2_kernel(AP p, const f16_t* Q16, const f16_t* D16,
                                                                  const f16_t* K16, const f16_t* V16) {
    constexpr int NWV = 8 / QB;
    const cmt_attn_train_args& a = p.a;
    __shared__ __attribute__((aligned(16))) char ring[DQ_RING * 2 * KT * 64];   // [slot][K | V][64 rows][64 B]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H, split = blockIdx.z;
    h8_t qf[QB][2], df[QB][2];
    float L[QB], dl[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        const int q = blockIdx.x * 256 + (wave * QB + i) * 32 + lr;
        const int qc = min(q, a.Nq - 1);
        const f16_t* Qr = Q16 + ((int64_t)bh * a.Nq + qc) * D;
        const f16_t* Dr = D16 + ((int64_t)bh * a.Nq + qc) * D;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            qf[i][kk] = *(const h8_t*)(Qr + 16 * kk + 8 * lh);
            df[i][kk] = *(const h8_t*)(Dr + 16 * kk + 8 * lh);
        }
        L[i] = a.LSE[(int64_t)bh * a.Nq + qc];
        dl[i] = a.delta[(int64_t)bh * a.Nq + qc];
    }
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);
    // the 8 1-KB pieces of a tile (K rows 16 c .. 16 c + 15 for c < 4, then V): piece w + NWV i
    // by wave w; a lane's LDS destination is lane-linear, the swizzle sits on the source chunk
    const f16_t* src0[QB];
    char* dst0[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        const int pc = wave + NWV * i, mat = pc >> 2, piece = pc & 3;
        const int prow = 16 * piece + (lane >> 2);
        src0[i] = (mat ? V16 : K16) + (int64_t)bh * a.Nk * D + 8 * ((lane & 3) ^ ((prow >> 2) & 3));
        dst0[i] = ring + mat * KT * 64 + piece * 1024;
    }
    const int prow_l = lane >> 2;
    int issued = t0;
    auto issue_upto = [&](int n) {
        const int e = min(n, t1);
        while (issued < e) {
#pragma unroll
            for (int i = 0; i < QB; ++i) {
                const int pc = wave + NWV * i, piece = pc & 3;
                const int key = min(issued * KT + 16 * piece + prow_l, a.Nk - 1);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src0[i] + (int64_t)key * D),
                    (__attribute__((address_space(3))) void*)(dst0[i] + (issued % DQ_RING) * 2 * KT * 64), 16, 0, 0);
            }
            ++issued;
        }
    };
    issue_upto(t0 + DQ_RING - 1);
    f32x16 dq[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;
    const float c = p.c;
    for (int t = t0; t < t1; ++t) {
        dq2_wait(QB * (issued - t - 1));
        barrier_mem();                                  // tile t landed for every wave; tile t-1 consumed
        issue_upto(t + DQ_RING);
        const char* Ks = ring + (t % DQ_RING) * 2 * KT * 64;
        const char* Vs = Ks + KT * 64;
        const bool edge = (t + 1) * KT > a.Nk;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            h8_t kfr[2], vfr[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int o = sw_off(kb * 32 + lr, 2 * kk + lh);
                kfr[kk] = *(const h8_t*)(Ks + o);
                vfr[kk] = *(const h8_t*)(Vs + o);
            }
            f32x16 s[QB];
#pragma unroll
            for (int i = 0; i < QB; ++i) {
                f32x16 sp, dp;
#pragma unroll
                for (int r = 0; r < 16; ++r) sp[r] = dp[r] = 0.f;
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    sp = mma16(kfr[kk], qf[i][kk], sp);      // S^T = K Q^T (lane = query)
                    dp = mma16(vfr[kk], df[i][kk], dp);      // dP^T = V dO^T
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float pr = __builtin_amdgcn_exp2f(sp[r] * c - L[i]);
                    if (edge && t * KT + kb * 32 + key_of(r, lh) >= a.Nk) pr = 0.f;
                    sp[r] = pr * (dp[r] - dl[i]);              // dS^T
                }
                s[i] = sp;
            }
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const h8_t kt = tr_frag(Ks, kb * 32 + 16 * ss, lane);
#pragma unroll
                for (int i = 0; i < QB; ++i) dq[i] = mma16(kt, frag_acc(s[i], ss), dq[i]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        const int q = blockIdx.x * 256 + (wave * QB + i) * 32 + lr;
        if (q >= a.Nq) continue;
        float* dQb = a.dQ + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs + (int64_t)q * a.q_rs;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = dq[i][r] * a.scale;
            if (gridDim.z > 1) atomicAdd(dQb + key_of(r, lh), v);
            else dQb[key_of(r, lh)] = v;
        }
    }
}

AP make_ap(const cmt_attn_train_args& a, int splits) {
    AP p;
    p.a = a;
    p.a.kv_splits = splits;
    p.c = a.scale * LOG2E;
    const int ntiles = (a.Nk + KT - 1) / KT;
    p.tiles_per_split = cdiv(ntiles, splits);
    p.keep_scale = a.dropout_p > 0.f ? 1.f / (1.f - a.dropout_p) : 1.f;
    const double thr = (double)a.dropout_p * 4294967296.0;
    p.drop_thr = thr >= 4294967295.0 ? 0xffffffffU : (uint32_t)thr;
    return p;
}

int train_splits(const cmt_attn_train_args& a) {
    if (a.kv_splits > 0) return a.kv_splits;
    const int ntiles = (a.Nk + KT - 1) / KT;
    const int base = cdiv(a.Nq, 128) * a.B * a.H;
    int s = 1;
    while (base * s < 512 && ntiles / (2 * s) >= 4) s *= 2;
    return s;
}

int check_args(const cmt_attn_train_args& a, const char* who) {
    CMT_REQUIRE(a.B > 0 && a.H > 0 && a.Nq > 0 && a.Nk > 0, std::string(who) + ": empty problem");
    CMT_REQUIRE(a.Q && a.K && a.V && a.O && a.LSE, std::string(who) + ": null pointer");
    CMT_REQUIRE(a.q_rs % 4 == 0 && a.k_rs % 4 == 0 && a.v_rs % 4 == 0 && a.o_rs % 4 == 0 && a.q_hs % 4 == 0 &&
                a.k_hs % 4 == 0 && a.v_hs % 4 == 0 && a.q_bs % 4 == 0 && a.k_bs % 4 == 0 && a.v_bs % 4 == 0,
                std::string(who) + ": strides must keep 16-byte rows");
    CMT_REQUIRE(a.dn_pad <= 0 || a.dn_group > 0, std::string(who) + ": dn_group must be > 0 with dn_pad");
    CMT_REQUIRE(a.dropout_p >= 0.f && a.dropout_p < 1.f, std::string(who) + ": dropout_p must be in [0, 1)");
    return 0;
}

// ---- the long-key fp16 path: applicability and workspace layout
bool fast_path(const cmt_attn_train_args& a) {
    return a.fp16_inputs && a.dn_pad <= 0 && !(a.dropout_p > 0.f) && a.Nk >= 4096 && a.Nq > 128 &&
           a.Nq <= NQ_RES && a.o_hs == D && a.kv_splits <= 0;
}

int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// forward key splits: one round of one-per-CU workgroups (the ping-pong kernel holds a CU); at
// ~1 100 queries the inference core's automatic choice (8 splits, 320 workgroups) ran two rounds
int fwd_splits(const cmt_attn_train_args& a) { return max(1, min(16, 256 / (cdiv(a.Nq, 256) * a.B * a.H))); }

struct FastWs {   // byte offsets into the workspace
    int64_t q16, k16, v16, d16, kmax, attn, total;
};

FastWs fast_ws(const cmt_attn_train_args& a) {
    FastWs w;
    const int64_t qn = (int64_t)a.B * a.H * a.Nq * D * 2, kn = (int64_t)a.B * a.H * a.Nk * D * 2;
    w.q16 = 0;
    w.k16 = align256(w.q16 + qn);
    w.v16 = align256(w.k16 + kn);
    w.d16 = align256(w.v16 + kn);
    w.kmax = align256(w.d16 + qn);
    w.attn = align256(w.kmax + cdiv64((int64_t)a.B * a.Nk, 64) * a.H * 4);
    cmt_attn_args g = {};
    g.B = a.B; g.H = a.H; g.Nq = a.Nq; g.Nk = a.Nk; g.dtype = CMT_F16;
    g.kv_splits = fwd_splits(a);
    w.total = align256(w.attn + cmt_attn_workspace_bytes(&g));
    return w;
}

void to16(const float* X, int64_t bs, int64_t hs, int64_t rs, int B, int H, int N, f16_t* Y, float* kmax,
          hipStream_t s) {
    to16_kernel<<<dim3((unsigned)cdiv64((int64_t)B * N, 64), (unsigned)H), 256, 0, s>>>(X, bs, hs, rs, B, H, N, Y,
                                                                                        kmax);
}

// Zeroes the [N x 32] rows of every (b, h) of a strided head-split fp32 view (the accumulated
// dQ / dK / dV of a split backward): one launch instead of a 2-D memset per (b, h)
__global__ __launch_bounds__(256) void zero_heads_kernel(float* X, int64_t bs, int64_t hs, int64_t rs, int H, int N,
                                                         int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i >> 5;          // (b, h, n) row, D = 32 floats each
        const int n = (int)(r % N);
        const int64_t bh = r / N;
        X[(bh / H) * bs + (bh % H) * hs + n * rs + (i & 31)] = 0.f;
    }
}

void zero_heads(float* X, int64_t bs, int64_t hs, int64_t rs, int B, int H, int N, hipStream_t s) {
    const int64_t total = (int64_t)B * H * N * D;
    zero_heads_kernel<<<(unsigned)std::min<int64_t>(cdiv64(total, 256), 2048), 256, 0, s>>>(X, bs, hs, rs, H, N, total);
}

}  // namespace

extern "C" int64_t cmt_attn_train_workspace_bytes(const cmt_attn_train_args* a) {
    if (!a) return 0;
    if (fast_path(*a)) return fast_ws(*a).total;
    const int s = train_splits(*a);
    if (s <= 1) return 0;
    return (int64_t)s * a->B * a->H * a->Nq * (D + 2) * (int64_t)sizeof(float);
}

extern "C" int cmt_attn_train_fwd(const cmt_attn_train_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_attn_train_fwd: null args");
    if (int rc = check_args(*ap, "cmt_attn_train_fwd")) return rc;
    const int splits = train_splits(*ap);
    // the long-key f16 path always writes its f16 copies into the workspace (also at one split)
    if ((splits > 1 || fast_path(*ap)) &&
        (ap->workspace == nullptr || ap->workspace_bytes < cmt_attn_train_workspace_bytes(ap)))
        return cmt_fail(CMT_EWORKSPACE, "cmt_attn_train_fwd: workspace too small");
    AP p = make_ap(*ap, splits);
    hipStream_t s = (hipStream_t)stream;
    if (fast_path(*ap)) {
        // f16 head-split operands (+ the keys' per-64-row max |k|^2), then the inference core with
        // the row statistic (attention.hip; output rounded to f16 like the flash core's)
        const cmt_attn_train_args& a = *ap;
        const FastWs w = fast_ws(a);
        char* base = (char*)a.workspace;
        f16_t* q16 = (f16_t*)(base + w.q16);
        f16_t* k16 = (f16_t*)(base + w.k16);
        f16_t* v16 = (f16_t*)(base + w.v16);
        float* kmax = (float*)(base + w.kmax);
        to16(a.Q, a.q_bs, a.q_hs, a.q_rs, a.B, a.H, a.Nq, q16, nullptr, s);
        to16(a.K, a.k_bs, a.k_hs, a.k_rs, a.B, a.H, a.Nk, k16, kmax, s);
        to16(a.V, a.v_bs, a.v_hs, a.v_rs, a.B, a.H, a.Nk, v16, nullptr, s);
        if (int rc = cmt_check_launch("cmt_attn_train_fwd (f16 copies)")) return rc;
        cmt_attn_args g = {};
        g.B = a.B; g.H = a.H; g.Nq = a.Nq; g.Nk = a.Nk; g.dtype = CMT_F16;
        g.Q = q16; g.q_bstride = (int64_t)a.H * a.Nq * D; g.q_hstride = (int64_t)a.Nq * D; g.q_rstride = D;
        g.K = k16; g.k_bstride = (int64_t)a.H * a.Nk * D; g.k_hstride = (int64_t)a.Nk * D; g.k_rstride = D;
        g.V = v16; g.v_bstride = g.k_bstride; g.v_hstride = g.k_hstride; g.v_rstride = D;
        g.O = a.O; g.o_bstride = a.o_bs; g.o_rstride = a.o_rs; g.o_dtype = CMT_F32;
        g.scale = a.scale;
        g.flags = CMT_ATTN_ROUND_OUTPUT;
        g.kv_splits = fwd_splits(a);
        g.workspace = base + w.attn;
        g.workspace_bytes = w.total - w.attn;
        g.kmax2 = kmax; g.kmax_ld = a.H; g.kmax_plane0 = 0; g.kmax_rows = 64;
        return cmt_attn_fwd_lse(g, a.LSE, s);
    }
    const dim3 grid(cdiv(ap->Nq, 128), ap->B * ap->H, splits);
    if (ap->fp16_inputs) {
        const bool mask = ap->dn_pad > 0, drop = ap->dropout_p > 0.f;
        if (mask && drop) train16_fwd_kernel<true, true><<<grid, 256, 0, s>>>(p);
        else if (mask) train16_fwd_kernel<true, false><<<grid, 256, 0, s>>>(p);
        else if (drop) train16_fwd_kernel<false, true><<<grid, 256, 0, s>>>(p);
        else train16_fwd_kernel<false, false><<<grid, 256, 0, s>>>(p);
    } else {
        train_fwd_kernel<<<grid, 256, 0, s>>>(p);
    }
    if (splits > 1) {
        const int64_t n = (int64_t)ap->B * ap->H * ap->Nq * D;
        train_combine_kernel<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(p);
    }
    return cmt_check_launch("cmt_attn_train_fwd");
}

extern "C" int cmt_attn_train_bwd(const cmt_attn_train_args* ap, void* stream) {
    CMT_REQUIRE(ap != nullptr, "cmt_attn_train_bwd: null args");
    if (int rc = check_args(*ap, "cmt_attn_train_bwd")) return rc;
    CMT_REQUIRE(ap->dO && ap->dQ && ap->dK && ap->dV && ap->delta, "cmt_attn_train_bwd: null gradient pointer");
    const int ntiles = (ap->Nk + KT - 1) / KT;
    const int base = cdiv(ap->Nq, 128) * ap->B * ap->H;
    int qs = 1;   // key split of the dQ pass (atomics into a zeroed dQ)
    // one round at the kernel's 3 waves per SIMD (3 four-wave workgroups per CU: 768); the
    // power-of-two split ran 1.5 rounds at the coop self-attention shape (r6f: bwd 377 -> 303 us
    // with the dK / dV split below)
    qs = max(1, min(ntiles / 2, 768 / base));
    AP p = make_ap(*ap, qs);
    hipStream_t s = (hipStream_t)stream;
    const int64_t rows = (int64_t)ap->B * ap->H * ap->Nq;
    train_delta_kernel<<<(unsigned)cdiv64(rows, 4), 256, 0, s>>>(p);
    if (fast_path(*ap) && ap->workspace != nullptr && ap->workspace_bytes >= fast_ws(*ap).total) {
        const cmt_attn_train_args& a = *ap;
        const FastWs w = fast_ws(a);
        char* base = (char*)a.workspace;
        f16_t* q16 = (f16_t*)(base + w.q16);
        f16_t* k16 = (f16_t*)(base + w.k16);
        f16_t* v16 = (f16_t*)(base + w.v16);
        f16_t* d16 = (f16_t*)(base + w.d16);
        to16(a.dO, a.o_bs, a.o_hs, a.o_rs, a.B, a.H, a.Nq, d16, nullptr, s);
        if (!a.ws_reuse) {   // ABI 25: else the forward's copies of Q / K / V are still in the workspace
            to16(a.Q, a.q_bs, a.q_hs, a.q_rs, a.B, a.H, a.Nq, q16, nullptr, s);
            to16(a.K, a.k_bs, a.k_hs, a.k_rs, a.B, a.H, a.Nk, k16, nullptr, s);
            to16(a.V, a.v_bs, a.v_hs, a.v_rs, a.B, a.H, a.Nk, v16, nullptr, s);
        }
        // dQ: key splits of 8-wave workgroups, about two per CU
        // (two 8-wave workgroups per CU: about 512 workgroups in one balanced round)
        const int nqb = cdiv(a.Nq, 256);
        const int ds = max(1, min(512 / (nqb * a.B * a.H), ntiles / 8));
        AP pq = make_ap(a, ds);
        if (ds > 1) {
            const bool dense = a.q_hs == D && a.q_rs == (int64_t)a.H * D && a.q_bs == (int64_t)a.Nq * a.H * D;
            if (dense) {
                CMT_REQUIRE(hipMemsetAsync(a.dQ, 0, (size_t)a.B * a.Nq * a.H * D * sizeof(float), s) == hipSuccess,
                            "cmt_attn_train_bwd: dQ zeroing failed");
            } else {
                zero_heads(a.dQ, a.q_bs, a.q_hs, a.q_rs, a.B, a.H, a.Nq, s);
            }
        }
        const int nqp = cdiv(a.Nq, 64) * 64;
        train16_dkv2_kernel<<<dim3((unsigned)cdiv(a.Nk, 256), (unsigned)(a.B * a.H)), 512, 0, s>>>(p, q16, d16, k16,
                                                                                                   v16, nqp);
        // 32 queries per wave (QB = 2, 240 VGPRs at two waves per SIMD: 238 vs 206 us, r4v)
        train16_dq2_kernel<1><<<dim3((unsigned)nqb, (unsigned)(a.B * a.H), (unsigned)ds), 512, 0, s>>>(pq, q16, d16,
                                                                                                       k16, v16);
        return cmt_check_launch("cmt_attn_train_bwd");
    }
    if (qs > 1) {
        // dQ is accumulated: zero it (its [Nq x 32] rows per (b, h), strided)
        zero_heads(ap->dQ, ap->q_bs, ap->q_hs, ap->q_rs, ap->B, ap->H, ap->Nq, s);
    }
    const dim3 gq(cdiv(ap->Nq, 128), ap->B * ap->H, qs), gk(cdiv(ap->Nk, 128), ap->B * ap->H);
    if (ap->fp16_inputs) {
        const bool mask = ap->dn_pad > 0, drop = ap->dropout_p > 0.f;
        if (mask && drop) {
            train16_dq_kernel<true, true><<<gq, 256, 0, s>>>(p);
            train16_dkv_kernel<true, true><<<gk, 256, 0, s>>>(p);
        } else if (mask) {
            train16_dq_kernel<true, false><<<gq, 256, 0, s>>>(p);
            train16_dkv_kernel<true, false><<<gk, 256, 0, s>>>(p);
        } else if (drop) {
            train16_dq_kernel<false, true><<<gq, 256, 0, s>>>(p);
            train16_dkv_kernel<false, true><<<gk, 256, 0, s>>>(p);
        } else {
            train16_dq_kernel<false, false><<<gq, 256, 0, s>>>(p);
            train16_dkv_kernel<false, false><<<gk, 256, 0, s>>>(p);
        }
    } else {
        train_dq_kernel<<<gq, 256, 0, s>>>(p);
        // query splits of the dK / dV pass until the grid covers ~2 workgroups per CU
        const int nqt = cdiv(ap->Nq, KT);
        int ks = 1;
        // one round at the kernel's 2 waves per SIMD (2 four-wave workgroups per CU: 512)
        ks = max(1, min(nqt / 2, (int)(512 / ((int64_t)gk.x * gk.y))));
        if (ks > 1) {
            const cmt_attn_train_args& a = *ap;
            for (int which = 0; which < 2; ++which) {
                float* X = which ? a.dV : a.dK;
                const int64_t bs = which ? a.v_bs : a.k_bs, hs = which ? a.v_hs : a.k_hs, rs = which ? a.v_rs : a.k_rs;
                if (hs == D && rs == (int64_t)a.H * D && bs == (int64_t)a.Nk * a.H * D) {
                    CMT_REQUIRE(hipMemsetAsync(X, 0, (size_t)a.B * a.Nk * a.H * D * sizeof(float), s) == hipSuccess,
                                "cmt_attn_train_bwd: dK / dV zeroing failed");
                } else {
                    zero_heads(X, bs, hs, rs, a.B, a.H, a.Nk, s);
                }
            }
        }
        train_dkv_kernel<<<dim3(gk.x, gk.y, ks), 256, 0, s>>>(p, cdiv(nqt, ks));
    }
    return cmt_check_launch("cmt_attn_train_bwd");
}
