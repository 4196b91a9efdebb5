// Shared device helpers for the gfx950 (CDNA4) kernels of libcmt_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/cmt_hip.h"

typedef __bf16 bf16_t;
typedef _Float16 f16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short __attribute__((__vector_size__(4 * sizeof(short)))) s16v4_lds;

#define CMT_LDS __attribute__((address_space(3)))

// ---- error plumbing (host) -------------------------------------------------
void cmt_set_error(const std::string& msg);
int cmt_fail(int code, const std::string& msg);
int cmt_check_launch(const char* what);

#define CMT_REQUIRE(cond, msg)                                   \
    do {                                                         \
        if (!(cond)) return cmt_fail(CMT_EINVAL, std::string(msg)); \
    } while (0)

// ---- element conversion ----------------------------------------------------
template <typename T>
__device__ __forceinline__ float to_f32(T x) { return (float)x; }

template <typename T>
__device__ __forceinline__ T from_f32(float x) { return (T)x; }

// MFMA wrappers: 32x32x16 (f16 / bf16 inputs, 8 elements per lane).
template <typename T> struct mfma_traits;
template <> struct mfma_traits<bf16_t> {
    typedef bf16x8 frag;
    static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct mfma_traits<f16_t> {
    typedef f16x8 frag;
    static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Max helpers.  These must stay compiler-visible (no inline asm): their
// inputs are often MFMA results, and a VALU read of an MFMA destination needs
// hazard wait states that hipcc only inserts for instructions it can see.
// attention.hip is built with -fno-honor-nans, so fmaxf lowers to a single
// v_max/v_max3 without the NaN-canonicalising v_max_f32 x,x per operand.
__device__ __forceinline__ float vmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ float vmax(float a, float b) { return fmaxf(a, b); }
// max of x over the lane pair (l, l ^ 32) via v_permlane32_swap (no LDS round trip)
__device__ __forceinline__ float pair_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Workgroup barrier that is also a compiler memory barrier: LDS-DMA
// (global_load_lds) writes are invisible to the compiler, so ds_reads of a
// freshly DMA'd buffer must not be scheduled above the s_barrier that orders
// them after the other waves' counted vmcnt waits (the bare builtin does not
// prevent that hoisting).  gfx950 has back-off barriers, so the compiler puts
// no wait before an s_barrier it cannot see: the lgkmcnt(0) here makes this
// wave's own ds_writes visible to the waves past the barrier (without it a
// tile staged through LDS was occasionally read before a 16-byte piece of it
// landed -- a 4 x 8 block of wrong outputs in ~1 of 10^6 GEMM tiles).
__device__ __forceinline__ void barrier_mem() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Non-finite sanitiser with torch.nan_to_num defaults.
__device__ __forceinline__ float nan_to_num(float x) {
    if (x != x) return 0.f;
    if (x == __builtin_inff()) return 3.4028234663852886e38f;
    if (x == -__builtin_inff()) return -3.4028234663852886e38f;
    return x;
}

// CMT_F16P split of one fp32 value (cmt_hip.h): x = hi + lo, both f16 (RNE).
typedef f16_t pair_t;
typedef f16x8 pair8_t;
__device__ __forceinline__ void split_pair(float x, pair_t& hi, pair_t& lo) {
    hi = (pair_t)x;
    lo = (pair_t)(x - (float)hi);
}
// Store v as element c of a CMT_F16P row (hi at row[c], lo at row[C + c]).
__device__ __forceinline__ void store_pair(pair_t* row, int C, int c, float v) {
    pair_t h, l;
    split_pair(v, h, l);
    row[c] = h;
    row[C + c] = l;
}
// 4 consecutive elements c..c+3 of a CMT_F16P row (8-byte stores).
__device__ __forceinline__ void store_pair4(pair_t* row, int C, int c, f32x4 v) {
    typedef pair_t p4 __attribute__((ext_vector_type(4)));
    p4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h[j] = (pair_t)v[j];
        l[j] = (pair_t)(v[j] - (float)h[j]);
    }
    *(p4*)(row + c) = h;
    *(p4*)(row + C + c) = l;
}
// 8 consecutive elements c..c+7 (16-byte stores).
__device__ __forceinline__ void store_pair8(pair_t* row, int C, int c, const float* v) {
    pair8_t h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        h[j] = (pair_t)v[j];
        l[j] = (pair_t)(v[j] - (float)h[j]);
    }
    *(pair8_t*)(row + c) = h;
    *(pair8_t*)(row + C + c) = l;
}

// The long-key f16 attention forward (attention.hip, cmt_attn_fwd's bounded-offset path) that
// also writes the row statistic lse[(b * H + h) * Nq + q] = log2(sum_k exp2(c s_qk)) (exp2 units
// of c = scale * log2 e): the training forward's flash-attn fp16 core (attn_train.hip).
int cmt_attn_fwd_lse(const cmt_attn_args& a, float* lse, void* stream);

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// compute units of the current device (cached per device): grids of one workgroup per CU
static inline int cmt_cu_count() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}
static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// f16-operand range guard (ABI 18): an fp32 value the f16 / f16-pair operand formats cannot
// carry -- non-finite, or |x| >= 65520 where the f16 (hi) rounding overflows.  A kernel that
// sees one ORs 1 into the caller's flag word with a vector atomic (rare path only).
__device__ __forceinline__ bool f16_unrepresentable(float x) { return !(__builtin_fabsf(x) < 65520.f); }
__device__ __forceinline__ void raise_range_flag(int* flag, bool bad) {
    if (flag != nullptr && bad) __hip_atomic_fetch_or(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
