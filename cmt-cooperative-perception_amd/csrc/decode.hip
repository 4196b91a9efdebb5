// NMS-free box decode of the CMT task heads:
// MultiTaskBBoxCoder.decode_single (core/bbox/coders/multi_task_bbox_coder.py:46-100)
// + denormalize_bbox (core/bbox/util.py:37-68), one workgroup per sample.
//
//   scores = sigmoid(logits)  over Nq x ncls  (flattened q-major, class-minor)
//   top-k (k = max_num) by radix select on order-preserving keys in LDS
//   (4 passes of 8 bits; ties at the k-th value resolved by lowest index),
//   bitonic sort of the k survivors (score desc, index asc), then per box:
//   label = idx % ncls, query = idx / ncls, task = class_task[label],
//   box = denormalize(bbox[task * Nq + query]), keep = inside post_center_range
//   (and score > threshold); survivors compacted in rank order.
#include "cmt_common.h"

namespace {

constexpr int DT_THREADS = 1024;
constexpr int MAX_ELEMS = 32768;   // Nq * ncls per sample (LDS keys: 128 KB)
constexpr int MAX_K = 1024;

__device__ __forceinline__ uint32_t order_key(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// block-wide exclusive scan of one int per thread (1024 threads, 16 waves)
__device__ int block_exclusive_scan(int v, int* warp_sums, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) warp_sums[w] = x;
    __syncthreads();
    if (w == 0) {
        int s = lane < DT_THREADS / 64 ? warp_sums[lane] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(s, off);
            if (lane >= off) s += y;
        }
        if (lane < DT_THREADS / 64) warp_sums[lane] = s;   // inclusive over waves
        if (lane == DT_THREADS / 64 - 1) *total = s;
    }
    __syncthreads();
    const int excl = x - v + (w > 0 ? warp_sums[w - 1] : 0);
    __syncthreads();
    return excl;
}

struct DecodeParams {
    const float* logits; int64_t l_bs;      // [B][Nq*ncls]
    const float* bbox; int64_t b_bs;        // [B][T*Nq][code]
    const int* class_task;                  // [ncls]
    int Nq, ncls, code, k;
    float pcr[6];
    float thresh; int use_thresh;
    float* out_boxes; float* out_scores; int* out_labels; int* out_count;   // [B][k][code-1], [B][k], [B][k], [B]
};

__global__ __launch_bounds__(DT_THREADS) void box_decode_kernel(DecodeParams p) {
    extern __shared__ uint32_t keys[];                    // N keys, then sort buffers
    __shared__ int hist[256];
    __shared__ int warp_sums[DT_THREADS / 64];
    __shared__ int s_total;
    __shared__ uint32_t s_prefix;
    __shared__ int s_need;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.Nq * p.ncls;
    const float* lg = p.logits + (int64_t)b * p.l_bs;
    for (int i = tid; i < N; i += DT_THREADS) keys[i] = order_key(lg[i]);
    if (tid == 0) {
        s_prefix = 0u;
        s_need = p.k;
    }
    __syncthreads();
    // ---- radix select: the k-th largest key, 8 bits per pass from the top
    uint32_t mask_hi = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 256; i += DT_THREADS) hist[i] = 0;
        __syncthreads();
        const uint32_t prefix = s_prefix;
        for (int i = tid; i < N; i += DT_THREADS) {
            const uint32_t u = keys[i];
            if ((u & mask_hi) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int need = s_need, cum = 0, bin = 255;
            for (; bin > 0; --bin) {
                if (cum + hist[bin] >= need) break;
                cum += hist[bin];
            }
            s_need = need - cum;
            s_prefix = prefix | ((uint32_t)bin << shift);
        }
        __syncthreads();
        mask_hi |= 255u << shift;
    }
    const uint32_t T = s_prefix;      // k-th largest key
    const int ties_needed = s_need;   // how many keys == T enter the top-k
    // ---- collect: keys > T, and the ties_needed lowest-index keys == T
    const int K = p.k;
    int Kp = 1;
    while (Kp < K) Kp <<= 1;
    uint32_t* skey = keys + N;                      // [Kp]
    int* sidx = (int*)(keys + N + Kp);              // [Kp]
    for (int i = tid; i < Kp; i += DT_THREADS) {
        skey[i] = 0u;                               // padding sorts last
        sidx[i] = 0x7fffffff;
    }
    const int chunk = (N + DT_THREADS - 1) / DT_THREADS;
    const int c0 = tid * chunk, c1 = min(N, c0 + chunk);
    int ng = 0, nt = 0;
    for (int i = c0; i < c1; ++i) {
        ng += keys[i] > T;
        nt += keys[i] == T;
    }
    const int g_off = block_exclusive_scan(ng, warp_sums, &s_total);
    const int n_greater = s_total;
    const int t_off = block_exclusive_scan(nt, warp_sums, &s_total);
    int gi = g_off, ti = t_off;
    for (int i = c0; i < c1; ++i) {
        const uint32_t u = keys[i];
        if (u > T) {
            skey[gi] = u;
            sidx[gi] = i;
            ++gi;
        } else if (u == T) {
            if (ti < ties_needed) {
                skey[n_greater + ti] = u;
                sidx[n_greater + ti] = i;
            }
            ++ti;
        }
    }
    __syncthreads();
    // ---- bitonic sort of Kp (key desc, index asc)
    for (int size = 2; size <= Kp; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < Kp; i += DT_THREADS) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool desc = (i & size) == 0;
                    const uint32_t ki = skey[i], kj = skey[j];
                    const int ii = sidx[i], ij = sidx[j];
                    // "i before j" in the final order: larger key, then smaller index
                    const bool i_first = ki > kj || (ki == kj && ii < ij);
                    if (desc ? !i_first : i_first) {
                        skey[i] = kj; skey[j] = ki;
                        sidx[i] = ij; sidx[j] = ii;
                    }
                }
            }
            __syncthreads();
        }
    }
    // ---- decode, mask, compact in rank order
    float box[9];
    float score = 0.f;
    int label = 0, keep = 0;
    const int nout = p.code - 1;                    // 10-code -> 9 outputs (w,l,h exp'd, rot from sin/cos)
    if (tid < K) {
        const int idx = sidx[tid];
        const float logit = lg[idx];
        score = 1.f / (1.f + expf(-logit));
        label = idx % p.ncls;
        const int q = idx / p.ncls;
        const int task = p.class_task[label];
        const float* bp = p.bbox + (int64_t)b * p.b_bs + ((int64_t)task * p.Nq + q) * p.code;
        box[0] = bp[0];
        box[1] = bp[1];
        box[2] = bp[2];
        box[3] = expf(bp[3]);
        box[4] = expf(bp[4]);
        box[5] = expf(bp[5]);
        box[6] = atan2f(bp[6], bp[7]);
        if (p.code > 8) {
            box[7] = bp[8];
            box[8] = bp[9];
        }
        keep = 1;
#pragma unroll
        for (int a = 0; a < 3; ++a) keep &= (box[a] >= p.pcr[a]) & (box[a] <= p.pcr[3 + a]);
        if (p.use_thresh) keep &= score > p.thresh;
    }
    const int pos = block_exclusive_scan(keep, warp_sums, &s_total);
    if (keep) {
        const int64_t o = (int64_t)b * K + pos;
        p.out_scores[o] = score;
        p.out_labels[o] = label;
        for (int a = 0; a < nout; ++a) p.out_boxes[o * nout + a] = box[a];
    }
    if (tid == 0) p.out_count[b] = s_total;
}

}  // namespace

extern "C" int cmt_box_decode(const float* logits, int64_t logit_bstride, const float* bbox, int64_t bbox_bstride,
                              const int* class_task, int B, int Nq, int ncls, int code, int max_num,
                              const float* post_center_range6, float score_threshold, int use_threshold,
                              float* out_boxes, float* out_scores, int* out_labels, int* out_count, void* stream) {
    CMT_REQUIRE(logits && bbox && class_task && post_center_range6 && out_boxes && out_scores && out_labels &&
                    out_count, "cmt_box_decode: null pointer");
    CMT_REQUIRE(B > 0 && Nq > 0 && ncls > 0 && (code == 8 || code == 10), "cmt_box_decode: bad shape");
    CMT_REQUIRE((int64_t)Nq * ncls <= MAX_ELEMS, "cmt_box_decode: Nq * ncls must be <= 32768");
    CMT_REQUIRE(max_num > 0 && max_num <= MAX_K && max_num <= Nq * ncls, "cmt_box_decode: 0 < max_num <= min(1024, Nq*ncls)");
    DecodeParams p;
    p.logits = logits; p.l_bs = logit_bstride;
    p.bbox = bbox; p.b_bs = bbox_bstride;
    p.class_task = class_task;
    p.Nq = Nq; p.ncls = ncls; p.code = code; p.k = max_num;
    for (int i = 0; i < 6; ++i) p.pcr[i] = post_center_range6[i];
    p.thresh = score_threshold; p.use_thresh = use_threshold;
    p.out_boxes = out_boxes; p.out_scores = out_scores; p.out_labels = out_labels; p.out_count = out_count;
    int Kp = 1;
    while (Kp < max_num) Kp <<= 1;
    const size_t smem = ((size_t)Nq * ncls + 2 * (size_t)Kp) * 4;
    // > 64 KB of dynamic LDS must be opted into (gfx950: 160 KB per workgroup)
    static const hipError_t attr_rc = hipFuncSetAttribute((const void*)box_decode_kernel,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (attr_rc != hipSuccess) return cmt_fail((int)attr_rc, "cmt_box_decode: cannot enable 150 KB of LDS");
    box_decode_kernel<<<B, DT_THREADS, smem, (hipStream_t)stream>>>(p);
    return cmt_check_launch("cmt_box_decode");
}
