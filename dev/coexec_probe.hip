// Co-execution probe (diagnostic, not product code): how do one wave's MFMAs
// and its SIMD partner's VALU / transcendental instructions share a gfx950
// SIMD?  512-thread workgroups, one per CU (waves w and w+4 on one SIMD).
// Waves 0-3 run role A, waves 4-7 role B; each role is one of
//   0 idle, 1 MFMA (32x32x16 f16, 4 independent accumulators),
//   2 v_exp_f32 (8 independent chains), 3 v_fma_f32 (8 chains),
//   4 v_cvt_pk_f16_f32, 5 mixed stream: 1 MFMA + 2 exp + 1 cvt_pk per step
// and the per-wave cycle count (s_memtime) of its loop is written out.
//   hipcc -O3 --offload-arch=gfx950 dev/coexec_probe.hip -o dev/coexec_probe && ./dev/coexec_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int ROLE>
__device__ __forceinline__ float run_role(int n, float seed) {
    if constexpr (ROLE == 1) {
        f16x8 a, b;
        for (int j = 0; j < 8; ++j) {
            a[j] = (_Float16)(seed * (j + 1));
            b[j] = (_Float16)(seed - j);
        }
        f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < n; ++i) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
        }
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
        return s;
    } else if constexpr (ROLE == 2 || ROLE == 3) {
        float x[8];
        for (int j = 0; j < 8; ++j) x[j] = seed * 0.001f * (j + 1);
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    x[j] = ROLE == 2 ? __builtin_amdgcn_exp2f(-x[j]) : __builtin_fmaf(x[j], 0.999f, 0.001f);
        }
        float s = 0.f;
        for (int j = 0; j < 8; ++j) s += x[j];
        return s;
    } else if constexpr (ROLE == 4) {
        float x[16];
        for (int j = 0; j < 16; ++j) x[j] = seed * (j + 1);
        unsigned acc = 0;
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                f16x2 h = {(_Float16)x[j], (_Float16)x[j + 1]};
                acc ^= __builtin_bit_cast(unsigned, h);
                asm volatile("" : "+v"(x[j]), "+v"(x[j + 1]));
            }
        }
        return (float)acc;
    } else if constexpr (ROLE == 5) {
        f16x8 a, b;
        for (int j = 0; j < 8; ++j) {
            a[j] = (_Float16)(seed * (j + 1));
            b[j] = (_Float16)(seed - j);
        }
        f32x16 c0 = {}, c1 = {};
        float x[8];
        for (int j = 0; j < 8; ++j) x[j] = seed * 0.001f * (j + 1);
        for (int i = 0; i < n; ++i) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
            x[0] = __builtin_amdgcn_exp2f(-x[0]);
            x[1] = __builtin_amdgcn_exp2f(-x[1]);
            x[2] = __builtin_amdgcn_exp2f(-x[2]);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
            x[3] = __builtin_amdgcn_exp2f(-x[3]);
            x[4] = __builtin_amdgcn_exp2f(-x[4]);
            x[5] = __builtin_amdgcn_exp2f(-x[5]);
        }
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r];
        for (int j = 0; j < 8; ++j) s += x[j];
        return s;
    }
    return 0.f;
}

template <int A, int B>
__global__ __launch_bounds__(512, 2) void probe(int na, int nb, float* out, long long* cyc) {
    const int wave = threadIdx.x >> 6;
    const float seed = 1.f + threadIdx.x * 1e-3f;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    float r = 0.f;
    if (wave < 4) r = run_role<A>(na, seed);
    else r = run_role<B>(nb, seed);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int A, int B>
void measure(const char* name, int na, int nb, float* out, long long* cyc, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) probe<A, B><<<nblk, 512>>>(na, nb, out, cyc);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) probe<A, B><<<nblk, 512>>>(na, nb, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nblk * 8);
    hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    std::vector<long long> ca, cb;
    for (int i = 0; i < nblk; ++i)
        for (int w = 0; w < 8; ++w) (w < 4 ? ca : cb).push_back(h[i * 8 + w]);
    std::sort(ca.begin(), ca.end());
    std::sort(cb.begin(), cb.end());
    printf("%-28s na=%5d nb=%5d  A cycles %8lld  B cycles %8lld  kernel %8.2f us\n", name, na, nb, ca[ca.size() / 2],
           cb[cb.size() / 2], ms / 5 * 1e3);
}

int main() {
    const int nblk = 256;
    float* out;
    long long* cyc;
    hipMalloc(&out, nblk * 512 * sizeof(float));
    hipMalloc(&cyc, nblk * 8 * sizeof(long long));
    const int N = 2000;
    // alone
    measure<1, 0>("mfma x4 | idle", N, 0, out, cyc, nblk);
    measure<0, 2>("idle | exp x16", 0, N, out, cyc, nblk);
    measure<0, 3>("idle | fma x16", 0, N, out, cyc, nblk);
    measure<0, 4>("idle | cvt_pk x8", 0, N, out, cyc, nblk);
    measure<5, 0>("mixed(2mfma+6exp) | idle", N, 0, out, cyc, nblk);
    // together: MFMA partner beside VALU partner
    measure<1, 2>("mfma x4 | exp x16", N, N, out, cyc, nblk);
    measure<1, 3>("mfma x4 | fma x16", N, N, out, cyc, nblk);
    measure<1, 4>("mfma x4 | cvt_pk x8", N, N, out, cyc, nblk);
    measure<1, 1>("mfma x4 | mfma x4", N, N, out, cyc, nblk);
    measure<2, 2>("exp x16 | exp x16", N, N, out, cyc, nblk);
    measure<5, 5>("mixed | mixed", N, N, out, cyc, nblk);
    measure<5, 2>("mixed | exp x16", N, N, out, cyc, nblk);
    measure<5, 1>("mixed | mfma x4", N, N, out, cyc, nblk);
    hipFree(out);
    hipFree(cyc);
    return 0;
}
