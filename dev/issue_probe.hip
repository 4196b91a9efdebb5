// Issue-ceiling probe (diagnostic, not product code) for the d_h = 32 cross-attention core:
// each wave runs the per-tile instruction mix of attn_pb2_kernel<f16, QS> from registers only
// (no LDS, no global memory in the loop), software-pipelined in one stream:
//   QK^T of tile i (8 x v_mfma_f32_32x32x16_f16: two 32-key blocks x (Q hi + Q lo) x 2 k-steps),
//   P of tile i-1 (32 x v_exp_f32 + 16 x v_cvt_pk_f16_f32 per lane),
//   PV + row sums of tile i-2 (4 x 32x32x16 + 4 x 16x16x32),
// at W = 1, 2, 3, 4 waves per SIMD (one 4W-wave workgroup per CU, LDS-pinned), and reports
// SIMD cycles per tile (s_memtime) against the 448-cycle matrix-pipe floor of one tile and the
// issue floor (16 MFMA x 8 + 32 exp x 8 + 16 cvt x 4 = 448).
//   hipcc -O3 --offload-arch=gfx950 dev/issue_probe.hip -o dev/issue_probe && ./dev/issue_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0)
#define MMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0)

template <int MODE>   // 0 full mix (pipelined), 1 MFMA only, 2 exp + cvt only, 3 full mix, one tile at a time
__device__ __forceinline__ void tile_body(f16x8 (&kf)[2][2], const f16x8 (&qf)[2], const f16x8 (&ql)[2],
                                          const f16x8 (&vf)[2][2], const f16x8& sel, f32x16 (&sa)[2],
                                          f32x16 (&sb)[2], f16x8 (&pf)[2][2], f32x16& o, f32x4& l) {
    asm volatile("" : "+v"(kf[0][0]), "+v"(kf[1][1]));   // keep QK^T in the loop
    if (MODE == 3) {
        // QK^T, P and PV of the SAME tile: the overlap has to come from the other waves
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            sa[kb] = MMA32(kf[kb][0], qf[0], f32x16{});
            sa[kb] = MMA32(kf[kb][1], qf[1], sa[kb]);
            sa[kb] = MMA32(kf[kb][0], ql[0], sa[kb]);
            sa[kb] = MMA32(kf[kb][1], ql[1], sa[kb]);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            pf[0][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sa[0][r]);
            pf[1][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sa[1][r]);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                o = MMA32(vf[kb][ss], pf[kb][ss], o);
                l = MMA16(sel, pf[kb][ss], l);
            }
        return;
    }
    if (MODE != 2) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            sa[kb] = MMA32(kf[kb][0], qf[0], f32x16{});
            sa[kb] = MMA32(kf[kb][1], qf[1], sa[kb]);
            sa[kb] = MMA32(kf[kb][0], ql[0], sa[kb]);
            sa[kb] = MMA32(kf[kb][1], ql[1], sa[kb]);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                o = MMA32(vf[kb][ss], pf[kb][ss], o);
                l = MMA16(sel, pf[kb][ss], l);
            }
    }
    if (MODE != 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            pf[0][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sb[0][r]);
            pf[1][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sb[1][r]);
        }
    } else {
        asm volatile("" : "+v"(pf[0][0]), "+v"(pf[1][1]));
    }
    if (MODE == 2) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) sa[kb][r] = sb[kb][r] * 0.999f;
    }
}

// MODE 4: MODE 3's tile with the K fragments (4 x ds_read_b128) and V^T fragments (16 x
// ds_read_b64_tr_b16) read from an LDS ring of 8 tiles each tile, and a workgroup barrier every
// two tiles -- the attention kernel's per-tile LDS traffic and synchronisation, without the DMA
template <int W>
__device__ __forceinline__ void tile_lds(const char* ring, int t, int lane, const f16x8 (&qf)[2], const f16x8 (&ql)[2],
                                         const f16x8& sel, f32x16 (&sa)[2], f16x8 (&pf)[2][2], f32x16& o, f32x4& l) {
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    const char* kt = ring + (t & 7) * 8192;
    const char* vt = kt + 4096;
    const int lr = lane & 31, lh = lane >> 5;
    f16x8 kf[2][2], vf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
            kf[kb][h] = *(const f16x8*)(kt + ((kb * 32 + lr) * 32 + 8 * ((2 * h + lh) ^ ((lr >> 2) & 3))) * 2);
    const int vo = ((4 * lh + ((lane & 15) >> 2)) * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3)) * 2;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            const char* b0 = vt + vo + (kb * 32 + 16 * ss) * 64;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b0);
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b0 + 512));
            short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            vf[kb][ss] = __builtin_bit_cast(f16x8, v8);
        }
    f32x16 sinit;
#pragma unroll
    for (int r = 0; r < 16; ++r) sinit[r] = -4.f;   // the bounded offset enters as the accumulator's start
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        sa[kb] = MMA32(kf[kb][0], qf[0], sinit);
        sa[kb] = MMA32(kf[kb][1], qf[1], sa[kb]);
        sa[kb] = MMA32(kf[kb][0], ql[0], sa[kb]);
        sa[kb] = MMA32(kf[kb][1], ql[1], sa[kb]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        pf[0][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sa[0][r]);
        pf[1][r >> 3][r & 7] = (_Float16)__builtin_amdgcn_exp2f(sa[1][r]);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            o = MMA32(vf[kb][ss], pf[kb][ss], o);
            l = MMA16(sel, pf[kb][ss], l);
        }
}

template <int W>
__global__ __launch_bounds__(256 * W, W) void probe_lds(int nt, float* out, long long* cyc) {
    __shared__ __attribute__((aligned(16))) char ring[8 * 8192];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 8 * 8192 / 4; i += 256 * W) ((float*)ring)[i] = 1e-3f * (float)(i & 255);
    f16x8 qf[2], ql[2], sel, pf[2][2];
    for (int j = 0; j < 8; ++j) {
        const float x = 0.01f * (lane + j);
        qf[0][j] = (_Float16)(0.3f - x); qf[1][j] = (_Float16)(0.2f + x);
        ql[0][j] = (_Float16)(1e-4f * x); ql[1][j] = (_Float16)(-1e-4f * x);
        sel[j] = (_Float16)((lane & 15) < 2 ? 1.f : 0.f);
    }
    f32x16 sa[2], o = {};
    f32x4 l = {};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < nt; i += 2) {
        tile_lds<W>(ring, i + wave, lane, qf, ql, sel, sa, pf, o, l);
        tile_lds<W>(ring, i + wave + 1, lane, qf, ql, sel, sa, pf, o, l);
        __syncthreads();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = l[0] + l[1];
    for (int r = 0; r < 16; ++r) s += o[r];
    out[blockIdx.x * 256 * W + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 * W + wave] = t1 - t0;
}

template <int W, int MODE>
__global__ __launch_bounds__(256 * W, W) void probe(int nt, float* out, long long* cyc) {
    extern __shared__ char pin[];   // dynamic LDS: one workgroup per CU
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f16x8 kf[2][2], vf[2][2], qf[2], ql[2], sel, pf[2][2];
    for (int j = 0; j < 8; ++j) {
        const float x = 0.01f * (lane + j);
        kf[0][0][j] = (_Float16)x; kf[0][1][j] = (_Float16)(x * 0.5f);
        kf[1][0][j] = (_Float16)(-x); kf[1][1][j] = (_Float16)(x * 0.25f);
        vf[0][0][j] = (_Float16)(x + 1.f); vf[0][1][j] = (_Float16)(x - 1.f);
        vf[1][0][j] = (_Float16)(x * 2.f); vf[1][1][j] = (_Float16)(x * 3.f);
        qf[0][j] = (_Float16)(0.3f - x); qf[1][j] = (_Float16)(0.2f + x);
        ql[0][j] = (_Float16)(1e-4f * x); ql[1][j] = (_Float16)(-1e-4f * x);
        sel[j] = (_Float16)((lane & 15) < 2 ? 1.f : 0.f);
        pf[0][0][j] = pf[0][1][j] = pf[1][0][j] = pf[1][1][j] = (_Float16)0.5f;
    }
    f32x16 sa[2], sb[2], o = {};
    f32x4 l = {};
    for (int r = 0; r < 16; ++r) sa[0][r] = sa[1][r] = sb[0][r] = sb[1][r] = -1.f - 0.01f * r;
    if (threadIdx.x == 0) pin[0] = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < nt; i += 2) {
        tile_body<MODE>(kf, qf, ql, vf, sel, sa, sb, pf, o, l);
        tile_body<MODE>(kf, qf, ql, vf, sel, sb, sa, pf, o, l);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = l[0] + l[1];
    for (int r = 0; r < 16; ++r) s += o[r] + sa[0][r] + sb[1][r];
    out[blockIdx.x * 256 * W + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 * W + wave] = t1 - t0;
}

template <int W, int MODE>
void measure(const char* name, int nt, float* out, long long* cyc, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t lds = 96 * 1024;
    hipFuncSetAttribute((const void*)probe<W, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int it = 0; it < 3; ++it) probe<W, MODE><<<nblk, 256 * W, lds>>>(nt, out, cyc);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) probe<W, MODE><<<nblk, 256 * W, lds>>>(nt, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nblk * 4 * W);
    hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double med = (double)h[h.size() / 2];
    // per SIMD: W waves x nt tiles in ~med cycles
    const double per_tile = med / (W * (double)nt);
    const double us = ms / 5 * 1e3;
    // one tile = 32 queries x 64 keys x d 32: 4 * 2048 * 32 = 262144 algorithmic FLOP
    const double tf = 262144.0 * nt * W * 4 * nblk / (us * 1e-6) / 1e12;
    printf("%-26s W=%d  SIMD cycles/tile %7.1f  (floor 448: %.2f)  kernel %8.2f us  %7.1f TF/s algorithmic  clk %.2f GHz\n",
           name, W, per_tile, 448.0 / per_tile, us, tf, med / (us * 1e3));
}

// The LDS loop plus the K/V stream: DMA 0 none; 1 every wave issues 2 LDS-DMA pieces (1 KB) per
// two-tile interval (the tile-at-a-time kernel); 2 waves 0-3 issue 4; 3 a ninth, loader-only wave
// issues all 16 (compute waves issue none).  Pieces come from a 64 MB buffer (HBM / L3 stream),
// each into the ring slot the barrier just freed; vmcnt(8) before each barrier keeps two
// intervals in flight.
typedef const __attribute__((address_space(1))) void* g_addr_t;
typedef __attribute__((address_space(3))) void* l_addr_t;

template <int DMA>
__global__ __launch_bounds__(DMA == 3 ? 576 : 512, 2) void probe_dma(int nt, const char* src, float* out) {
    __shared__ __attribute__((aligned(16))) char ring[8 * 8192];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 8 * 8192 / 4; i += blockDim.x) ((float*)ring)[i] = 1e-3f * (float)(i & 255);
    f16x8 qf[2], ql[2], sel, pf[2][2];
    for (int j = 0; j < 8; ++j) {
        const float x = 0.01f * (lane + j);
        qf[0][j] = (_Float16)(0.3f - x); qf[1][j] = (_Float16)(0.2f + x);
        ql[0][j] = (_Float16)(1e-4f * x); ql[1][j] = (_Float16)(-1e-4f * x);
        sel[j] = (_Float16)((lane & 15) < 2 ? 1.f : 0.f);
    }
    f32x16 sa[2], o = {};
    f32x4 l = {};
    const bool loader = DMA == 3 && wave == 8;
    const int npieces = DMA == 1 ? 2 : DMA == 2 ? (wave < 4 ? 4 : 0) : DMA == 3 ? (loader ? 16 : 0) : 0;
    const char* s0 = src + ((size_t)blockIdx.x * 16 * 1024 + lane * 16) % (60u << 20);
    __syncthreads();
    for (int i = 0; i < nt; i += 2) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __syncthreads();
        for (int k = 0; k < npieces; ++k) {
            const int piece = (wave * npieces + k) & 15;
            const char* g = s0 + ((size_t)(i * 8 + piece) * 1024) % (60u << 20);
            __builtin_amdgcn_global_load_lds((g_addr_t)g, (l_addr_t)(ring + ((i + 6) & 7) * 8192 / 2 + (piece & 7) * 1024),
                                             16, 0, 0);
        }
        if (!loader) {
            tile_lds<2>(ring, i, lane, qf, ql, sel, sa, pf, o, l);
            tile_lds<2>(ring, i + 1, lane, qf, ql, sel, sa, pf, o, l);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = l[0] + l[1];
    for (int r = 0; r < 16; ++r) s += o[r];
    out[blockIdx.x * 576 + threadIdx.x] = s;
}

template <int DMA>
void measure_dma(const char* name, int nt, const char* src, float* out, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t lds = 96 * 1024 - 8 * 8192;
    const int nth = DMA == 3 ? 576 : 512;
    hipFuncSetAttribute((const void*)probe_dma<DMA>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int it = 0; it < 3; ++it) probe_dma<DMA><<<nblk, nth, lds>>>(nt, src, out);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) probe_dma<DMA><<<nblk, nth, lds>>>(nt, src, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms / 5 * 1e3;
    const double tf = 262144.0 * nt * 8 * nblk / (us * 1e-6) / 1e12;
    printf("%-26s kernel %8.2f us  %7.1f TF/s algorithmic  (%.3f of 2.5 PF)\n", name, us, tf, tf / 2500);
}

template <int W>
void measure_lds(const char* name, int nt, float* out, long long* cyc, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t lds = 96 * 1024 - 8 * 8192;   // pin one workgroup per CU
    hipFuncSetAttribute((const void*)probe_lds<W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int it = 0; it < 3; ++it) probe_lds<W><<<nblk, 256 * W, lds>>>(nt, out, cyc);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) probe_lds<W><<<nblk, 256 * W, lds>>>(nt, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms / 5 * 1e3;
    const double tf = 262144.0 * nt * W * 4 * nblk / (us * 1e-6) / 1e12;
    printf("%-26s W=%d  kernel %8.2f us  %7.1f TF/s algorithmic  (%.3f of 2.5 PF)\n", name, W, us, tf, tf / 2500);
}

int main() {
    const int nblk = 256;
    float* out;
    long long* cyc;
    hipMalloc(&out, nblk * 1152 * sizeof(float));
    hipMalloc(&cyc, nblk * 16 * sizeof(long long));
    const int nt = 1000;
    measure<1, 0>("mix", nt, out, cyc, nblk);
    measure<2, 0>("mix", nt, out, cyc, nblk);
    measure<3, 0>("mix", nt, out, cyc, nblk);
    measure<1, 3>("mix, tile at a time", nt, out, cyc, nblk);
    measure<2, 3>("mix, tile at a time", nt, out, cyc, nblk);
    measure<3, 3>("mix, tile at a time", nt, out, cyc, nblk);
    measure<4, 3>("mix, tile at a time", nt, out, cyc, nblk);
    measure_lds<2>("lds + barrier/2 tiles", nt, out, cyc, nblk);
    measure_lds<3>("lds + barrier/2 tiles", nt, out, cyc, nblk);
    measure_lds<4>("lds + barrier/2 tiles", nt, out, cyc, nblk);
    {
        char* src;
        hipMalloc(&src, 64u << 20);
        hipMemset(src, 0, 64u << 20);
        measure_dma<0>("dma none (W=2)", nt, src, out, nblk);
        measure_dma<1>("dma 2/wave/interval", nt, src, out, nblk);
        measure_dma<2>("dma 4/wave, waves 0-3", nt, src, out, nblk);
        measure_dma<3>("dma by a 9th loader wave", nt, src, out, nblk);
        hipFree(src);
    }
    measure<1, 1>("mfma only", nt, out, cyc, nblk);
    measure<2, 1>("mfma only", nt, out, cyc, nblk);
    hipFree(out);
    hipFree(cyc);
    return 0;
}
