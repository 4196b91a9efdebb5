// Slot-pattern probe (diagnostic, not product code): the cross-attention tile's
// instruction mix on register data, 8 waves per CU (two per SIMD), to see what
// each ingredient costs: per tile 16 MFMAs (8 QK^T as two chains of 4, 4 P.V,
// 4 16x16x32 row sums), 32 v_exp_f32, 16 v_cvt_pk_f16_f32, 12 LDS reads.
//   ROLE 0: MFMAs only
//   ROLE 1: MFMAs + exps + packs interleaved per slot (the attn_sp_kernel order)
//   ROLE 2: ROLE 1 + the 12 LDS fragment reads at the top of each tile
//   ROLE 3: ROLE 2 + one workgroup barrier per tile
//   ROLE 4: exps + packs only (no MFMAs)
//   ROLE 5: ROLE 1 with the exps first, then the MFMAs (no interleave)
//   hipcc -O3 --offload-arch=gfx950 dev/slot_probe.hip -o dev/slot_probe && ./dev/slot_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short __attribute__((__vector_size__(4 * sizeof(short)))) s16v4_lds;

template <int ROLE>
__global__ __launch_bounds__(512, 2) void probe(int iters, float* out, long long* cyc) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[8192];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 8192; i += 512) lds[i] = (_Float16)(i * 1e-3f);
    __syncthreads();
    const float seed = 1.f + tid * 1e-4f;
    f16x8 kf[2][2], vf[2][2], qf[2], ql[2], sel;
    for (int j = 0; j < 8; ++j) {
        qf[0][j] = (_Float16)(seed * j * 0.01f);
        qf[1][j] = (_Float16)(seed * 0.02f);
        ql[0][j] = (_Float16)(seed * 1e-4f);
        ql[1][j] = (_Float16)(seed * 2e-4f);
        sel[j] = (_Float16)((lane & 15) == 0 ? 1.f : 0.f);
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                kf[a][b][j] = (_Float16)(seed * (a + b + j) * 0.01f);
                vf[a][b][j] = (_Float16)(seed * (a - b + j) * 0.01f);
            }
    }
    f32x16 S[2][2] = {}, o = {}, sinit;
    for (int r = 0; r < 16; ++r) sinit[r] = -3.f;
    f32x4 lsum = {};
    f16x8 P[2][2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int c = 0; c < 2; ++c)
                for (int j = 0; j < 8; ++j) P[a][b][c][j] = (_Float16)0.5f;
    const int lofs = (lane * 8) & 2047;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    auto tile = [&](auto par) {
        constexpr int PAR = decltype(par)::value;
        f32x16(&sn)[2] = S[PAR ^ 1];
        const f32x16(&sc)[2] = S[PAR];
        f16x8(&pn)[2][2] = P[PAR];
        const f16x8(&pp)[2][2] = P[PAR ^ 1];
        if constexpr (ROLE >= 2 && ROLE <= 3) {
            const _Float16* base = lds + lofs;
            asm volatile("" : "+v"(base));
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b) kf[a][b] = *(const f16x8*)(base + 512 * (2 * a + b));
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b) {
                    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16v4_lds*)(base + 2048 + 256 * (2 * a + b)));
                    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16v4_lds*)(base + 3072 + 256 * (2 * a + b)));
                    f16x8 v;
                    for (int j = 0; j < 4; ++j) {
                        v[j] = __builtin_bit_cast(_Float16, x[j]);
                        v[4 + j] = __builtin_bit_cast(_Float16, y[j]);
                    }
                    vf[a][b] = v;
                }
        }
        auto mfma = [&](int i) {
            if (i < 4) {
                lsum = __builtin_amdgcn_mfma_f32_16x16x32_f16(sel, pp[i >> 1][i & 1], lsum, 0, 0, 0);
            } else if (i < 12) {
                const int j = i - 4, kb = j / 4, k = j % 4;
                const f16x8& qop = (k >> 1) ? ql[k & 1] : qf[k & 1];
                sn[kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[kb][k & 1], qop, k == 0 ? sinit : sn[kb], 0, 0, 0);
            } else {
                const int j = i - 12;
                o = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[j >> 1][j & 1], pp[j >> 1][j & 1], o, 0, 0, 0);
            }
        };
        float ea = 0.f, eb = 0.f;
        auto pack = [&](int m) {
            h2 v = {(_Float16)ea, (_Float16)eb};
            asm volatile("" : "+v"(v));
            const int kb = m >> 3, r = 2 * (m & 7);
            pn[kb][r >> 3][r & 7] = v[0];
            pn[kb][r >> 3][(r & 7) + 1] = v[1];
        };
        auto exps = [&](int m) {
            const int kb = m >> 3, r = 2 * (m & 7);
            float na, nb;
            asm volatile("v_exp_f32 %0, %1" : "=v"(na) : "v"(sc[kb][r]));
            asm volatile("v_exp_f32 %0, %1" : "=v"(nb) : "v"(sc[kb][r + 1]));
            if (m > 0) pack(m - 1);
            ea = na;
            eb = nb;
        };
        if constexpr (ROLE == 5) {
#pragma unroll
            for (int m = 0; m < 16; ++m) exps(m);
            pack(15);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) mfma(i);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (ROLE != 4) mfma(i);
                if constexpr (ROLE != 0) exps(i);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (ROLE != 0) pack(15);
        }
        if constexpr (ROLE == 3) __syncthreads();
    };
    for (int it = 0; it < iters; it += 2) {
        tile(std::integral_constant<int, 0>{});
        tile(std::integral_constant<int, 1>{});
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float acc = lsum[0] + lsum[1] + o[0] + o[5];
    for (int r = 0; r < 16; ++r) acc += S[0][0][r] + S[1][1][r] + S[0][1][r] + S[1][0][r];
    for (int j = 0; j < 8; ++j) acc += (float)P[0][0][0][j] + (float)P[1][1][1][j];
    out[blockIdx.x * 512 + tid] = acc;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int ROLE>
void measure(const char* name, int iters, float* out, long long* cyc, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 2; ++it) probe<ROLE><<<nblk, 512>>>(iters, out, cyc);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) probe<ROLE><<<nblk, 512>>>(iters, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nblk * 8);
    hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double med = (double)h[h.size() / 2];
    printf("%-44s %8.1f cycles per tile per wave (median wave), kernel %8.2f us\n", name, med / iters,
           ms / 5 * 1e3);
}

int main() {
    const int nblk = 256, iters = 400;
    float* out;
    long long* cyc;
    hipMalloc(&out, nblk * 512 * sizeof(float));
    hipMalloc(&cyc, nblk * 8 * sizeof(long long));
    measure<0>("0 MFMA only (16 per tile)", iters, out, cyc, nblk);
    measure<4>("4 exp + pack only (32 + 16 per tile)", iters, out, cyc, nblk);
    measure<1>("1 slots: MFMA + 2 exp + pack", iters, out, cyc, nblk);
    measure<5>("5 exps first, then MFMAs", iters, out, cyc, nblk);
    measure<2>("2 slots + 12 LDS reads", iters, out, cyc, nblk);
    measure<3>("3 slots + 12 LDS reads + barrier per tile", iters, out, cyc, nblk);
    hipFree(out);
    hipFree(cyc);
    return 0;
}
