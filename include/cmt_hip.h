/*
 * cmt_hip.h -- C ABI of the MI355X-native CMT / CMTCoop decoder-head hot path.
 *
 * Build: libcmt_hip.so (hipcc --offload-arch=gfx950), see
 * cmt-cooperative-perception_amd/csrc/Makefile.  Consumers: the registered
 * Python classes in cmt-cooperative-perception_amd/projects/mmdet3d_plugin
 * (ctypes, native.py) -- the drop-in for the reference's
 * projects/mmdet3d_plugin heads/transformer/attention/voxelization.
 *
 * Contract:
 *   - plain pointers + sizes; every pointer is a device pointer unless noted;
 *   - the caller (PyTorch) owns every buffer; nothing here allocates device
 *     memory -- scratch space is a caller-provided workspace whose size is
 *     returned by the matching *_workspace_bytes query;
 *   - stream-ordered and reentrant: every call takes the stream (a hipStream_t
 *     passed as void*), launches asynchronously on it, never synchronises and
 *     keeps no global mutable state (graph-capturable);
 *   - errors: every entry point returns 0 on success, a CMT_E* argument-check
 *     code, or the hipError_t of a failed launch; cmt_last_error() returns a
 *     thread-local message describing the last failure.
 *
 * Element type codes (dtype arguments).
 */
#ifndef CMT_HIP_H
#define CMT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMT_ABI_VERSION 25

/* CMT_F16P (ABI 12), "f16 pair": an fp32 operand split into two f16 halves,
 * x = hi + lo with hi = f16(x), lo = f16(x - hi).  Representation error:
 * |x - hi - lo| <= max(2^-22 |x|, 2^-25).  The relative 2^-22 (22 significant
 * bits) holds only while lo is itself a normal f16 number, i.e. for |x| >= ~2^-3;
 * below that lo is subnormal and the error is the absolute 2^-25 (the f16
 * subnormal half-step): ~2^-19 relative at |x| ~ 0.05, the scale of xavier
 * weights of a 256-wide layer, ~2^-16 at |x| ~ 0.005.  |x| must stay below
 * 65504.  A row of logical width C is stored as C hi values followed by C lo
 * values ([rows][2C] 16-bit words, leading dimensions in 16-bit elements).  A
 * GEMM whose A and W are both CMT_F16P computes A_hi W_hi + A_lo W_hi + A_hi W_lo
 * with fp32 accumulation (three f16 MFMA passes; the dropped A_lo W_lo term is
 * <= 2^-22 of a product): per product the error is the two operands'
 * representation errors above (tests/test_gpu_split.py::
 * test_gemm_split_small_weights holds the kernel to that bound on xavier-range
 * weights), at 3/16 of the f16 rate instead of the exact-f32 MFMA's 1/16.
 * Producers (LayerNorm, layout, geometry, GEMM epilogues, attention outputs)
 * write this format directly. */
enum cmt_dtype { CMT_F32 = 0, CMT_F16 = 1, CMT_BF16 = 2, CMT_F16P = 3 };

enum cmt_status {
    CMT_OK = 0,
    CMT_EINVAL = 1001,    /* bad argument (shape, alignment, dtype combination) */
    CMT_ENOTSUP = 1002,   /* unsupported configuration */
    CMT_EWORKSPACE = 1003 /* workspace too small */
};

int cmt_abi_version(void);
const char* cmt_last_error(void);

/* sizeof() of each argument struct as compiled into the library: a binding
 * that mirrors a struct (ctypes, cffi) asserts its own size against these
 * before the first call (native.py does; so does the INTEGRATION.md stub). */
int64_t cmt_gemm_args_size(void);
int64_t cmt_attn_args_size(void);
int64_t cmt_ln_args_size(void);
int64_t cmt_chain_args_size(void);
int64_t cmt_gemm_ex_args_size(void);
int64_t cmt_attn_train_args_size(void);
int64_t cmt_ln_train_args_size(void);
int64_t cmt_bn_args_size(void);
int64_t cmt_det_loss_args_size(void);
int64_t cmt_match_cost_args_size(void);
int64_t cmt_adamw_args_size(void);

/* ------------------------------------------------------------------------
 * GEMM with fused prologue/epilogue (MFMA, gfx950).
 *   C[m, n] = act( sum_k Aeff[m, k] * W[n, k] + bias[n] ) + R[m, n]
 * Replaces the cuBLAS GEMMs of the reference:
 *   FlashMHA _in_projection_packed      models/utils/attention.py:21-27,130
 *   FlashMHA out_proj                   models/utils/attention.py:117,138
 *   nn.MultiheadAttention in/out proj   (mmcv MultiheadAttention, attn_cfgs[0])
 *   mmcv FFN fc1/fc2                    (ffn_cfgs, e.g. configs/.../cmt_lidar_voxel0075_cbgs.py:232-239)
 *   bev_embedding / rv_embedding MLPs   models/dense_heads/cmt_head.py:292-301
 *   shared_conv Conv2d 3x3 (+BN fold)   models/dense_heads/cmt_head.py:280-287  (a_mode = CONV3X3)
 *   SeparateTaskHead grouped Conv1d     models/dense_heads/cmt_head.py:136-159  (a_mode = CONV1D3, batch = groups)
 * Output columns n < a2_cols see a modified A (the positional-encoding add
 * `key = key + key_pos`, petr_transformer.py:296-299):
 *   a2_mode CMT_A2_ADD     Aeff = A + A2 (both fp32, added on load);
 *   a2_mode CMT_A2_SELECT  Aeff = A2 (same dtype/strides as A: the caller
 *                          already holds the sum, e.g. written by the LN that
 *                          produced A), so one launch serves Q|K (pos) and V.
 * Compute dtype = w_dtype: CMT_F32 (exact-f32 MFMA 32x32x2), CMT_F16 or
 * CMT_BF16 (MFMA 32x32x16, fp32 accumulate).  With A in the compute dtype the
 * tiles are staged by LDS-DMA (global_load_lds); fp32 A is converted on load.
 * R may be fp32 or the compute dtype (r_dtype).
 * Requirements: N % 64 == 0, K % 32 == 0 (K % 64 for compute-dtype A),
 * 16-byte aligned A/W rows, ldc/ldr multiples of 4.
 * ------------------------------------------------------------------------ */
/* CMT_A_CONV3X3_NCHW (ABI 14): the 3x3 / pad 1 conv straight from an fp32 NCHW map
 * A[b * a_bstride + c * (conv_h * conv_w) + pixel] (lda unused), K = 9 * conv_c tap-major
 * as CONV3X3, M = conv_h * conv_w per batch element; split (CMT_F16P) W (the
 * reference-numerics shared_conv: each input pixel is split into f16 hi / lo once per
 * workgroup and serves all nine taps from LDS; fp32 or CMT_F16P row C) or, since round 6,
 * f16 / bf16 W (one MFMA pass on pixels rounded to W's dtype; fp32 or W-dtype row C);
 * conv_c % 16 == 0, conv_w <= 180, N % 128 == 0.  Optional second output: with A2 (fp32 rows
 * A2[m * lda2 + n], the same for every batch element -- the weight-only BEV position
 * rows) it also writes out + A2 at C + c_split_stride (same layout as C): lowp(memory +
 * pos), the K-projection operand, without a separate GEMM. */
enum cmt_gemm_amode { CMT_A_ROWS = 0, CMT_A_CONV3X3 = 1, CMT_A_CONV1D3 = 2, CMT_A_CONV3X3_NCHW = 3 };
enum cmt_gemm_cmode { CMT_C_ROWS = 0, CMT_C_HEADSPLIT = 1 };
enum cmt_gemm_a2mode { CMT_A2_ADD = 0, CMT_A2_SELECT = 1 };

typedef struct cmt_gemm_args {
    int M, N, K;
    int batch;                 /* grid z; per-batch strides below (elements) */
    const void* A; int64_t lda; int64_t a_bstride; int a_dtype;
    const void* A2; int64_t lda2; int a2_cols; int a2_mode;
    int a_mode;                /* cmt_gemm_amode */
    int conv_h, conv_w, conv_c;/* CONV3X3: NHWC input [M/(h*w)][h][w][c], K = 9*c */
    int seg_len;               /* CONV1D3: rows form segments of seg_len (zero pad), K = 3*C */
    const void* W; int64_t ldw; int64_t w_bstride; int w_dtype;
    const float* bias; int64_t bias_bstride;
    const void* R; int64_t ldr; int64_t r_bstride; int r_dtype;
    void* C; int64_t ldc; int64_t c_bstride; int c_dtype;
    int c_mode;                /* cmt_gemm_cmode; HEADSPLIT: C[(b*(N/32)+n/32)*rows_per_batch + r][32]
                                  (a CMT_F16P C: [..][64], the 32 hi values then the 32 lo values) */
    int rows_per_batch;
    int relu;
    /* optional (HEADSPLIT with a 16-bit C only): plane_max2[(m/64)*(plane_max_cols/32) + n/32]
     * = max over the 64-row block's rows m of sum_{32 cols of head plane n/32} C[m,n]^2
     * (of the stored, rounded values), for n < plane_max_cols; every entry is written
     * (rows >= M count as 0).  Feeds cmt_attn_args.kmax2. */
    float* plane_max2; int plane_max_cols;
    /* optional split-K (ABI 13): k_splits >= 2 splits the logical K into k_splits equal
     * parts (K / k_splits % 64 == 0) run by separate workgroups; part s writes its partial
     * product to C + s * c_split_stride (fp32, row mode, batch 1, no relu), bias and R
     * are added by part 0 only, so the sum of the parts is the GEMM's output.  For the
     * decoder's 900-row GEMMs, whose tile grid alone covers a quarter of the CUs; the
     * LayerNorm after them sums the parts (cmt_ln_args.nparts).  0 or 1: no split. */
    int k_splits; int64_t c_split_stride;
    /* optional f16-operand range guard (ABI 18; the split (CMT_F16P) cmt_gemm kernels: the x3
     * tiles, CMT_A_CONV3X3_NCHW and the 128-wide split tile -- not cmt_kv_proj / cmt_gemm_ln,
     * whose operands are outputs of guarded kernels): when a pre-activation value -- or the second output of
     * CMT_A_CONV3X3_NCHW with A2 -- is non-finite or |x| >= 65520 (outside the f16-pair
     * format: a bad input element makes every output of its 3x3 neighbourhood NaN / inf, since
     * 0 x inf is NaN), the kernel ORs 1 into *range_flag.  Never cleared by the library: the
     * caller zeroes it and reads it after the stream (or a replayed graph) has run.  NULL: off. */
    int* range_flag;
} cmt_gemm_args;

int cmt_gemm(const cmt_gemm_args* args, void* stream);

/* cmt_kv_proj: the cross-attention K/V projection of ALL decoder layers in one
 * launch (kvproj.hip) -- FlashMHA's packed in_proj on the memory side
 * (attention.py:21-27, 126-138; key = key + key_pos at petr_transformer.py:
 * 296-299).  Same cmt_gemm_args contract as cmt_gemm restricted to: K = 256,
 * f16/bf16 A / W / C, row A, head-split C, no R / relu, batch 1, A2 (if any)
 * in select mode on exactly the first N/2 columns, N % (256 * parts) == 0,
 * optional plane_max2.  W is in the FRAGMENT-PACKED layout
 *   Wp[((p * 16 + ks) * 64 + lane) * 8 + e] = W[32 p + (lane & 31)][16 ks + 8 (lane >> 5) + e]
 * (torch: W.view(N/32, 32, 16, 2, 8).permute(0, 2, 3, 1, 4)), ldw unused.
 * c_bstride (16-bit elements, 0: (N/32) * rows_per_batch * 32) is the batch
 * stride of the head-split C, so one layer's K and V planes can be written into
 * a larger [B][planes][Nk][32] buffer (one launch per layer, C pointing at the
 * layer's first plane). */
int cmt_kv_proj(const cmt_gemm_args* args, void* stream);

/* cmt_mlp2_x3 (ABI 15): Linear(K, Hd) + ReLU + Linear(Hd, 256) in one launch at the
 * reference's fp32 numerics (mlp.hip) -- the camera position encoder rv_embedding
 * (cmt_head.py:297-301, applied at 433 on the frustum coordinates of _rv_pe and at
 * 464 on the query coordinates of _rv_query_embed).  Replaces the two cmt_gemm
 * calls (fc1 -> hidden pair rows in HBM -> fc2): the hidden activation never
 * leaves the registers.  Every product is the split-f16 three-pass product of
 * cmt_gemm (hi*hi + lo*hi + hi*lo, fp32 accumulation, fc1 in cmt_gemm's k order,
 * so the hidden values equal the two-GEMM path's bit for bit).
 *   A   CMT_F16P rows [M][2][K] (lda, a_bstride in 16-bit words), K % 16 == 0, K <= 192
 *   W1p / W2p  the fragment packs of the pair weights W1 [Hd][2][K] and W2 [256][2][Hd]
 *       (Hd % 32 == 0):
 *       W1p[(((hb * K/16 + ks) * 2 + pl) * 64 + lane) * 8 + j]
 *           = W1[32 hb + (lane & 31)][pl][16 ks + 8 (lane >> 5) + j]
 *       W2p[((((hb * 8 + ot) * 2 + s) * 2 + pl) * 64 + lane) * 8 + j]
 *           = W2[32 ot + (lane & 31)][pl][32 hb + 16 s + 8 (j >> 2) + 4 (lane >> 5) + (j & 3)]
 *       (the second k order is the hidden accumulator's register order: fc1's
 *       output tile is fc2's operand without leaving the registers)
 *   b1 [Hd] (Hd <= 2048), b2 [256] fp32; out = fc2(relu(fc1(A) + b1)) + b2 (+ R)
 *   R   optional residual rows (CMT_F16P [.][2][256] or fp32), ldr / r_bstride
 *   C   CMT_F16P or fp32 rows, ldc / c_bstride (16-bit words for a pair C, else
 *       elements); batch = grid y. */
typedef struct cmt_mlp2_args {
    int M, K, Hd, N;           /* N must be 256 */
    int batch;
    const void* A; int64_t lda; int64_t a_bstride;
    const void* W1p; const float* b1;
    const void* W2p; const float* b2;
    const void* R; int64_t ldr; int64_t r_bstride; int r_dtype;
    void* C; int64_t ldc; int64_t c_bstride; int c_dtype;
    /* ABI 20, the camera memory rows in one launch (each optional, NULL = off; K == 192):
     * geo_i2l: A is not read but generated -- the _rv_pe frustum coordinates of
     *   cmt_rv_pe_coords (cmt_head.py:417-432, the same arithmetic and f16-pair split): row r of
     *   batch z is pixel r % (geo_h * geo_w) of view v = r / (geo_h * geo_w), V = M / (geo_h *
     *   geo_w) views per batch element, inverse matrix geo_i2l[(z * V + v) * 16], geo_D = K / 3
     *   depths up to geo_depth_max, geo_pc the point-cloud range;
     * rx: the residual R is read from the NCHW fp32 image features instead (the camera memory
     *   rows "(bs v) c h w -> bs (v h w) c", cmt_transformer.py:104-105): element n of row r is
     *   rx[((z * V + v) * 256 + n) * geo_h * geo_w + pixel]; it enters as its f16 pair (the
     *   rounding cmt_nchw_to_rows applies), those pair rows are written to C2 (ldc2 / c2_bstride
     *   in 16-bit words: the memory rows themselves), and a value the pair format cannot carry
     *   ORs 1 into *range_flag (optional) as cmt_nchw_to_rows_ex does. */
    const float* geo_i2l; int geo_h, geo_w, geo_D; float geo_pad_h, geo_pad_w, geo_depth_max;
    float geo_pc[6];
    const float* rx; void* C2; int64_t ldc2; int64_t c2_bstride; int* range_flag;
} cmt_mlp2_args;

int cmt_mlp2_x3(const cmt_mlp2_args* args, void* stream);
int64_t cmt_mlp2_args_size(void);

/* ------------------------------------------------------------------------
 * Multi-head attention core, head_dim = 32 (flash-style, online softmax,
 * f16/bf16 MFMA with fp32 accumulate, or exact-f32 MFMA for dtype CMT_F32;
 * no mask).
 * Replaces flash_attn_unpadded_kvpacked_func (flash-attn 0.2.2) called at
 *   models/utils/attention.py:70-74 (FlashAttention.forward 46-92, fp16 core)
 * and the softmax(QK^T/sqrt(d))V core of nn.MultiheadAttention used by the
 * self-attention (mmcv MultiheadAttention, attn_cfgs[0]).
 * Element (b, h, row, d) of Q/K/V is at X[b*x_bstride + h*x_hstride + row*x_rstride + d]
 * (head-split layout: rstride = 32; token-major [B,S,H*32]: rstride = H*32;
 * sequence-first [S,B,H*32]: rstride = B*H*32).  Row strides must keep
 * 16-byte alignment (multiples of 8 elements).
 * Output O (o_dtype: fp32, or f16/bf16/f16-pair when it only feeds the
 * out-projection GEMM) has the heads concatenated per row (normalised).
 * dtype CMT_F16P (ABI 13, the reference-numerics self-attention): Q/K/V rows
 * are f16 pairs of 64 16-bit elements -- the 32 hi values, then the 32 lo
 * values (cmt_gemm's head-split pair C: rstride = 64) -- every product runs
 * as three f16 MFMAs (~2^-21 relative, fp32 softmax); strides count 16-bit
 * elements; no kv_splits, kmax2 or output rounding.
 * Nk is split into kv_splits chunks processed by separate workgroups and
 * merged by a combine pass (workspace: cmt_attn_workspace_bytes).
 * ------------------------------------------------------------------------ */
/* flags: CMT_ATTN_ROUND_OUTPUT  round O to dtype (flash-attn returns fp16)
 *        CMT_ATTN_FOLD_SCALE    the kernel may fold scale*log2(e) into Q when
 *                               it loads Q (one extra rounding of Q in the
 *                               compute dtype; used by the f16/bf16 policies,
 *                               not by the reference-numerics policy)
 *        CMT_ATTN_FORCE_PINGPONG, CMT_ATTN_FORCE_PIPELINED   reserved, ignored
 *                               (ABI 17 selected a software-pipelined variant
 *                               with the second; it measured slower and was
 *                               removed in round 5)
 *        CMT_ATTN_UNSCALED_Q       f16 long-key core without the fold
 *                               permission: Q enters the QK^T MFMAs unscaled
 *                               and the scores are scaled in fp32 (flash-attn's
 *                               order) instead of Q * scale as hi + lo
 *        CMT_ATTN_KEEP_PARTIALS (ABI 19) a split launch (cmt_attn_splits() > 1) skips its
 *                               combine pass and does not write O: the split partials stay in
 *                               the workspace for cmt_chain's chain B1 (cmt_chain_args.xpart) */
enum { CMT_ATTN_ROUND_OUTPUT = 1, CMT_ATTN_FOLD_SCALE = 2, CMT_ATTN_FORCE_PINGPONG = 256,
       CMT_ATTN_FORCE_PIPELINED = 512, CMT_ATTN_UNSCALED_Q = 1024, CMT_ATTN_KEEP_PARTIALS = 2048 };

typedef struct cmt_attn_args {
    int B, H, Nq, Nk;
    int dtype;                 /* CMT_F32, CMT_F16, CMT_BF16 or CMT_F16P (Q, K, V) */
    const void* Q; int64_t q_bstride, q_hstride, q_rstride;
    const void* K; int64_t k_bstride, k_hstride, k_rstride;
    const void* V; int64_t v_bstride, v_hstride, v_rstride;
    void* O; int64_t o_bstride, o_rstride;   /* O[b*o_bstride + q*o_rstride + h*32 + d] */
    int o_dtype;               /* CMT_F32 / CMT_F16 / CMT_BF16 / CMT_F16P (pair rows [hi H*32 | lo H*32]) */
    float scale;               /* softmax scale, usually 1/sqrt(32) */
    int kv_splits;             /* 0 = choose automatically */
    int flags;                 /* CMT_ATTN_ROUND_OUTPUT | CMT_ATTN_FOLD_SCALE */
    void* workspace; int64_t workspace_bytes;
    /* optional (NULL = off): max squared key-row norms written by the K
     * projection GEMM (cmt_gemm_args.plane_max2): entry [e][kmax_ld] covers key
     * rows e*kmax_rows .. +kmax_rows-1 of the batch-major K rows (b*Nk + row),
     * head h reads column kmax_plane0 + h.  With bf16 the long-key kernel then
     * fixes each query's softmax offset at the Cauchy-Schwarz bound |q|*max|k|
     * (no running max) when that bound is <= 60 in exp2 units. */
    const float* kmax2; int kmax_ld; int kmax_plane0; int kmax_rows;
} cmt_attn_args;

int64_t cmt_attn_workspace_bytes(const cmt_attn_args* args);
int cmt_attn_fwd(const cmt_attn_args* args, void* stream);
/* ABI 19: the key-split count a cmt_attn_fwd launch with these arguments uses (1 = no partials) */
int cmt_attn_splits(const cmt_attn_args* args);

/* ------------------------------------------------------------------------
 * LayerNorm over the last dim C (C % 64 == 0, C <= 1024), eps given.
 *   y = LN(x) * w + b   (nn.LayerNorm; mmcv build_norm_layer LN, eps 1e-5)
 * flags: CMT_LN_NAN_TO_NUM  apply torch.nan_to_num to y (cmt_head.py:499)
 *        CMT_LN_MAX_INTO    y = max(y, Y_old) (coop max-fusion, cmt_head_coop.py:388-389)
 * If W2/B2/Y2 are non-null a second LN is applied to the first LN's output
 * (the decoder post_norm of each layer output, petr_transformer.py:364-368)
 * and written to Y2 with its own flags2.
 * Pointer arguments named *_range6, *3 (voxel geometry) and head_out are HOST
 * arrays (read at launch); all other pointers are device pointers.
 * ------------------------------------------------------------------------ */
enum { CMT_LN_NAN_TO_NUM = 1, CMT_LN_MAX_INTO = 2 };
int cmt_layernorm(const float* X, int64_t ldx, int rows, int C,
                  const float* W, const float* Bv, float eps, float* Y, int64_t ldy, int flags,
                  const float* W2, const float* B2, float* Y2, int64_t ldy2, int flags2,
                  void* stream);

/* cmt_layernorm_ex: cmt_layernorm plus the next GEMMs' operands in the
 * compute dtype (lowp_dtype), written from the same registers:
 *   Yl[row] = lowp(y)            (e.g. the FFN / V-projection input)
 *   Yp[row] = lowp(y + P[row])   (query + query_pos, petr_transformer.py:296-297)
 * Y may be NULL when only the compute-dtype copies are needed. */
typedef struct cmt_ln_args {
    const float* X; int64_t ldx; int rows; int C;
    const float* W; const float* B; float eps;
    float* Y; int64_t ldy; int flags;
    const float* W2; const float* B2; float* Y2; int64_t ldy2; int flags2;
    int lowp_dtype;
    void* Yl; int64_t ldyl;
    void* Yp; int64_t ldyp; const float* P; int64_t ldp;
    /* ABI 13: the LayerNorm input is the sum of nparts (>= 1; 0 = 1) row blocks
     * X + p * part_stride -- the partial products of a split-K cmt_gemm */
    int nparts; int64_t part_stride;
} cmt_ln_args;
int cmt_layernorm_ex(const cmt_ln_args* args, void* stream);

/* cmt_gemm_ln: cmt_gemm followed by cmt_layernorm_ex on its output rows, in
 * one launch (the post-norm "x = LN(x + sublayer(x))" of
 * petr_transformer.py:374-487 for the attention out-projections and FFN fc2):
 * t = A W^T + bias + R is never written; ln->X is ignored and every LN output
 * of ln (Y, Yl, Yp, Y2) is produced.  Needs N == ln->C == 256, compute-dtype
 * A/W, row mode, batch 1.  ABI 14: A and W both CMT_F16P (the reference-numerics
 * out-projections + norms[0] / norms[1]: three f16 passes, fp32 R, pair Yl / Yp). */
int cmt_gemm_ln(const cmt_gemm_args* gemm, const cmt_ln_args* ln, void* stream);

/* ------------------------------------------------------------------------
 * Row-block chains of the decoder layer's query side (rowchain.hip): each
 * workgroup owns 32 complete query rows (C = 256) and runs the layer's GEMMs
 * back to back with their operands in LDS and the post-norm epilogues fused
 * (petr_transformer.py:374-487; mmcv FFN / LN).  Replaces, per layer, the
 * cuBLAS out_proj / in_proj / FFN GEMMs and the three LayerNorms around the
 * two attention cores (attention.py:117, mmcv MultiheadAttention, mmcv FFN).
 *   kind 0 (chain A, after self-attention; 1 workgroup per 32 rows):
 *     Y = norms[0](X Wo^T + bo + R);  Q = lowp(Y + P) Wq^T + bq  (head split [B][8][Nq][32])
 *   kind 1 (chain B1, after cross-attention; 4 workgroups per 32 rows, g = FFN quarter):
 *     o = norms[1](X Wo^T + bo + R);  h_g = relu(lowp(o) W1[256g:256g+256]^T + b1[...]);
 *     WS[g] = lowp(h_g) W2[:, 256g:256g+256]^T  (+ b2 + o for g = 0)     fp32 partials
 *   kind 2 (chain B2; 3 workgroups per 32 rows with Wn, else 1):
 *     Y = norms[2](WS[0] + WS[1] + WS[2] + WS[3])   (the next layer's query)
 *     OUT = post_norm(Y) (+ CMT_LN_NAN_TO_NUM / CMT_LN_MAX_INTO per out_flags)
 *     if Wn: Q = [lowp(Y + P) | lowp(Y + P) | lowp(Y)] Wn^T + bn  (next layer's
 *            self-attn in_proj, head split [B][24][Nq][32])
 * prm: packed fp32 parameter block, layout (floats)
 *   A (1024): bo | norms[0].weight | norms[0].bias | bq
 *   B (3840, the same block for B1 and B2): bo | norms[1].w | norms[1].b | b1 (1024) | b2 |
 *             norms[2].w | norms[2].b | post_norm.w | post_norm.b | bn (768, zeros without Wn)
 * WS: caller workspace of cmt_chain_ws_bytes(rows) bytes = 4 * ceil(rows/32) * 32 * 256
 *     fp32 (B1 writes whole 32-row tiles, B2 reads them; private tile order).
 * One eps for every LayerNorm of the layer.  Weights / X / Q in the compute
 * dtype (f16 / bf16), residuals and outputs fp32; every buffer 16-byte aligned.
 * ------------------------------------------------------------------------ */
typedef struct cmt_chain_args {
    int kind;                  /* 0 = chain A, 1 = chain B1, 2 = chain B2 */
    int rows, Nq;              /* rows = B * Nq */
    int dtype;                 /* CMT_F16 / CMT_BF16 */
    float eps;
    const void* X;             /* A, B1: attention output [rows][256] */
    const float* R;            /* A, B1: residual [rows][256] fp32 (NULL = zeros) */
    const float* P;            /* query_pos [rows][256] fp32 (A; B2 with Wn) */
    const float* prm;          /* packed parameter block */
    const void* Wo;            /* A, B1: out_proj.weight [256][256] */
    const void* W1;            /* A: cross-attn in_proj_weight[:256], FRAGMENT-MAJOR (the Wn layout, g = 0);
                                  B1: fc1.weight [1024][256] row-major */
    const void* W2;            /* B1: fc2.weight [256][1024] as its 4 K blocks [256][256g..256g+256),
                                  each FRAGMENT-MAJOR (the Wn layout, g = K block) */
    const void* Wn;            /* B2: next layer's self-attn in_proj_weight [768][256], FRAGMENT-MAJOR:
                                  element W[256g + 64w + 32nt + r][32kc + 16ks + 8h + e] at
                                  ((((((g*4 + w)*8 + kc)*2 + ks)*2 + nt)*2 + h)*32 + r)*8 + e
                                  (NULL: last layer) */
    float* Y;                  /* A: norms[0] output; B2: norms[2] output; [rows][256] fp32 */
    float* OUT; int out_flags; /* B2: layer output [rows][256] fp32 */
    void* Q;                   /* head-split projection output (A; B2 with Wn) */
    float* WS;                 /* B1 / B2: partials workspace, 4 * ceil(rows/32) * 32 * 256 fp32 (private order) */
    void* OUT16;               /* B2 (optional): the layer output again in dtype (the task-head GEMM operand) */
    int wo_frag;               /* A: 1 = Wo is FRAGMENT-MAJOR (the Wn layout, g = 0) and streams into registers
                                  with W1 (no LDS weight ring); 0 = row-major Wo through the ring (ABI 10) */
    /* ABI 19, B1 with dtype CMT_F16P (optional, NULL = off): the cross-attention output as the split
     * partials a cmt_attn_fwd launch with CMT_ATTN_KEEP_PARTIALS left in its workspace (xpart = that
     * workspace; xsplits = cmt_attn_splits() of the launch, must be 8; B = rows / Nq, 8 heads).
     * Each workgroup combines its 32 rows itself (attn_combine_kernel's arithmetic, rounded to f16
     * when xround, as CMT_ATTN_ROUND_OUTPUT does) and X is not read. */
    const float* xpart; int xsplits; int xround;
} cmt_chain_args;
int cmt_chain(const cmt_chain_args* args, void* stream);
/* bytes of the B1 -> B2 partials workspace WS for `rows` query rows */
int64_t cmt_chain_ws_bytes(int rows);

/* cmt_add_cast: Yl = lowp(X), Yp = lowp(X + P) over rows x C (either output
 * may be NULL; X == NULL reads zeros, the zero target of cmt_transformer.py:114)
 * -- the decoder's first-layer operands from the initial target. */
int cmt_add_cast(const float* X, const float* P, int rows, int C, int lowp_dtype, void* Yl, void* Yp,
                 void* stream);

/* ------------------------------------------------------------------------
 * Coordinate encodings.
 * cmt_pos2embed: cmt_head.py:40-50.  pos [n, pos_stride] (x, y in the first two
 *   fp32 lanes), out [n, 2F] of odtype (F = num_pos_feats); mode 1 applies
 *   sigmoid(inverse_sigmoid(p)) first (query_embed, cmt_head.py:470).
 *   If pos == NULL the BEV grid centres (coords_bev, cmt_head.py:324-337) of a
 *   grid_h x grid_w map are generated in place of the input.
 * cmt_rv_pe_coords: _rv_pe geometry (cmt_head.py:417-432): out [BV*h*w, 3*D] (odtype)
 *   normalised lidar coordinates of D depth samples per image token; i2l is a
 *   [BV,4,4] fp32 device array of inv(lidar2img) (fp64 host inverse).
 * cmt_rv_query_coords: _rv_query_embed geometry (cmt_head.py:446-463):
 *   ref [B,Nq,3] (raw reference points; clamped + sigmoid(inverse_sigmoid)),
 *   l2i / i2l [B,V,4,4] fp32 -> out [B,V,Nq,3*D], mask [B,V,Nq] fp32 {0,1}.
 * cmt_masked_view_sum: (rv * mask).sum(dim=1) (cmt_head.py:466) added into Y:
 *   Y[b,q,:] += sum_v X[b,v,q,:] * mask[b,v,q].
 * cmt_rv_query_coords_ex (ABI 11): cmt_rv_query_coords with out in odtype
 *   (f16/bf16 rounded RNE: the operand of the rv_embedding GEMM without a cast pass).
 * cmt_masked_view_sum_ex (ABI 11): Y[b,q,:] = base[q,:] + sum_v ... (base [Nq,C]
 *   fp32, the BEV half of query_pos shared by every batch element; NULL: Y += ...),
 *   and optionally the decoder's first operands Yp = lowp(Y) = lowp(0 + query_pos)
 *   and Yl = lowp(0) (the zero target, cmt_transformer.py:114) in lowp_dtype.
 * ------------------------------------------------------------------------ */
int cmt_pos2embed(const float* pos, int64_t pos_stride, int n, int F, int mode,
                  int grid_h, int grid_w, void* out, int odtype, int64_t ldo, void* stream);
int cmt_rv_pe_coords(int BV, int h, int w, int D, float pad_h, float pad_w, float depth_max,
                     const float* i2l, const float* pc_range6, void* out, int odtype, void* stream);
int cmt_rv_query_coords(const float* ref, int B, int V, int Nq, int D, float pad_h, float pad_w,
                        const float* l2i, const float* i2l, const float* pc_range6,
                        float* out, float* mask, void* stream);
int cmt_masked_view_sum(const float* X, const float* mask, int B, int V, int Nq, int C,
                        float* Y, void* stream);
int cmt_rv_query_coords_ex(const float* ref, int B, int V, int Nq, int D, float pad_h, float pad_w,
                           const float* l2i, const float* i2l, const float* pc_range6,
                           void* out, int odtype, float* mask, void* stream);
int cmt_masked_view_sum_ex(const float* X, const float* mask, int B, int V, int Nq, int C,
                           const float* base, float* Y, void* Yl, void* Yp, int lowp_dtype, void* stream);

/* ------------------------------------------------------------------------
 * Layout / dtype plumbing.
 * cmt_nchw_to_rows: X [B, C, H*W] (optionally grouped as B = nb*nv images)
 *   -> rows: Y[(b_outer*rows_per_batch + row_offset + v*H*W + p)*ldy + c],
 *   i.e. rearrange "(bs v) c h w -> bs (v h w) c" (cmt_transformer.py:104-105),
 *   output dtype ydtype (CMT_F32/F16/BF16).
 * cmt_cast: elementwise dtype conversion of n elements.
 * ------------------------------------------------------------------------ */
int cmt_nchw_to_rows(const float* X, int nb, int nv, int C, int HW, void* Y, int ydtype,
                     int64_t ldy, int64_t rows_per_batch, int64_t row_offset, void* stream);
/* cmt_nchw_to_rows_ex (ABI 18): the same with the f16-operand range guard of
 * cmt_gemm_args.range_flag: for a CMT_F32 / CMT_F16 / CMT_F16P ydtype, an input element
 * that is non-finite or |x| >= 65520 ORs 1 into *range_flag (NULL: off; CMT_F32 with a flag:
 * rows a split-f16 consumer reads as pairs next, e.g. the training shared_conv). */
int cmt_nchw_to_rows_ex(const float* X, int nb, int nv, int C, int HW, void* Y, int ydtype,
                        int64_t ldy, int64_t rows_per_batch, int64_t row_offset, int* range_flag, void* stream);
int cmt_cast(const void* X, int xdtype, void* Y, int ydtype, int64_t n, void* stream);
/* cmt_split_rows (ABI 12): fp32 rows X[r * ldx + c] -> CMT_F16P rows Y [rows][2C]
 * (the split f16 GEMM operand of an fp32 tensor, e.g. the module-level API's inputs). */
int cmt_split_rows(const float* X, int64_t ldx, int64_t rows, int C, void* Y, void* stream);

/* ------------------------------------------------------------------------
 * SeparateTaskHead tail (cmt_head.py:136-203) + box epilogue (501-513).
 * H1 [L, B*Nq, nheads*hc] is the output of the first grouped conv (one GEMM
 * for all heads).  For every head: GroupLayerNorm1d over its hc channels
 * (eps 1e-6, biased var, cmt_head.py:56-66) -> ReLU -> grouped Conv1d
 * (kernel k along queries, zero pad) with weights W2 [L][out_total][k][hc]
 * packed per head, bias B2 [L][out_total].  Outputs are written to
 * OUT[L, B, Nq, out_total] (heads concatenated in order, widths head_out[]).
 * Columns listed by center_col/height_col receive the box epilogue:
 * sigmoid(x + inverse_sigmoid(ref)) * (max - min) + min.  H1 is only read;
 * the norm is applied to the LDS copy (one launch).
 * ------------------------------------------------------------------------ */
int cmt_task_head_tail(const float* H1, int L, int B, int Nq, int nheads, int hc,
                       const float* gln_w, const float* gln_b, const float* W2, const float* B2,
                       const int* head_out, int out_total, int k,
                       const float* ref, int center_col, int height_col, const float* pc_range6,
                       float* OUT, void* stream);

/* ------------------------------------------------------------------------
 * Point -> voxel scatter-mean (SPConvVoxelization + HardSimpleVFE).
 * Replaces spconv PointToVoxel at mmcv_custom/ops/voxel/spconv_voxelize.py:25-32,58-61
 * (called per sample at models/detectors/cmt.py:101-105) and mmdet3d
 * HardSimpleVFE.  Deterministic CPU semantics: voxels in first-appearance
 * order of their points, each keeps its first max_points points in input
 * order, at most max_voxels voxels, coordinates z,y,x.
 * points [N, F] fp32 (F >= nfeat_mean); outputs sized for max_voxels:
 *   voxels [max_voxels, max_points, F] (zero padded), coors [max_voxels, 3],
 *   num_points [max_voxels], means [max_voxels, nfeat_mean],
 *   num_voxels [1] (device int, M; -1 if the in-kernel scan gave up).
 * Three launches, no host synchronisation (graph-capturable).
 * Workspace (ABI 9): cmt_voxelize_workspace_bytes(N, .) bytes, filled once by
 * cmt_voxelize_workspace_init; every call leaves it clean again, so one
 * workspace serves any number of calls with N up to its capacity (the
 * largest power of two >= 1024 whose layout fits workspace_bytes), on one
 * stream at a time.
 * ------------------------------------------------------------------------ */
int64_t cmt_voxelize_workspace_bytes(int N, int max_voxels);
int cmt_voxelize_workspace_init(void* workspace, int64_t workspace_bytes, void* stream);
int cmt_voxelize(const float* points, int N, int F, const float* voxel_size3,
                 const float* coors_range6, const int* grid3, int max_points, int max_voxels,
                 int nfeat_mean, float* voxels, int* coors, int* num_points, float* means,
                 int* num_voxels, void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * NMS-free box decode.  Replaces
 * MultiTaskBBoxCoder.decode_single (core/bbox/coders/multi_task_bbox_coder.py:46-100)
 * + denormalize_bbox (core/bbox/util.py:37-68) for every sample b < B:
 *   logits [B][Nq*ncls] (last decoder layer, tasks' classes concatenated),
 *   bbox   [B][T*Nq][code] (center2, height1, dim3, rot2, vel2 per task block),
 *   class_task [ncls] = task index of each class label (device int32).
 * top-k (k = max_num) of sigmoid(logits), ties at the k-th value by lowest
 * index, score-descending; boxes denormalised (exp dims, atan2 yaw) to
 * code-1 values; kept if the center lies in post_center_range6 (HOST array)
 * and, when use_threshold, score > score_threshold.  Outputs are compacted in
 * rank order: out_boxes [B][max_num][code-1], out_scores/out_labels
 * [B][max_num], out_count [B] (device).  Nq*ncls <= 32768, max_num <= 1024.
 * ------------------------------------------------------------------------ */
int cmt_box_decode(const float* logits, int64_t logit_bstride, const float* bbox, int64_t bbox_bstride,
                   const int* class_task, int B, int Nq, int ncls, int code, int max_num,
                   const float* post_center_range6, float score_threshold, int use_threshold,
                   float* out_boxes, float* out_scores, int* out_labels, int* out_count, void* stream);

/* ========================================================================
 * TRAINING PATH (BASELINE configs[3] DDP training).
 * Exact-f32 kernels (the reference trains the head in fp32), used by the
 * torch.autograd Functions of projects/mmdet3d_plugin/models/utils/train_ops.py.
 * ======================================================================== */

/* cmt_gemm_f32_ex: C[z][m][n] = alpha * sum_k A(m,k) B(n,k) (+ bias[n]) + beta * C
 *   A(m,k) = A[z*a_bs + m*a_sm + k*a_sk],  B(n,k) = B[z*b_bs + n*b_sn + k*b_sk]
 * Any operand may be transposed (strides); k- or row-contiguous operands with
 * 16-byte alignment are staged by 16-byte loads.  ksplit > 1 splits K over
 * workgroups that add their partial sums into C with f32 atomics (beta = 1,
 * the caller initialises C).  Replaces the cuBLAS GEMMs of every nn.Linear
 * forward and backward (dX = dY W, dW = dY^T X) in the reference's training step. */
typedef struct cmt_gemm_ex_args {
    int M, N, K, batch;
    float alpha, beta;
    const float* A; int64_t a_sm, a_sk, a_bs;
    const float* B; int64_t b_sn, b_sk, b_bs;
    float* C; int64_t ldc, c_bs;
    const float* bias;         /* optional [N] per batch entry, at bias + z * bias_bs */
    int ksplit;
    int64_t bias_bs;           /* ABI 16: batch stride of bias (0: one bias for every z) */
    float* a_rowsum;           /* ABI 17, optional [batch][M], zero-initialised by the caller:
                                * += sum over this launch's k of A(m, k) in fp32 (cmt_gemm_bf16x3_ex
                                * only; a Linear's bias gradient from its weight-gradient GEMM) */
} cmt_gemm_ex_args;
int cmt_gemm_f32_ex(const cmt_gemm_ex_args* args, void* stream);
/* cmt_gemm_bf16x3_ex: the same contract, each fp32 operand split into a bf16
 * pair (hi + lo, RNE) and multiplied in three bf16 MFMA passes (lo*hi + hi*lo +
 * hi*hi, fp32 accumulate): ~2^-16 relative per product, fp32 exponent range --
 * the training step's Linear forward / dX / dW (the reference's fp32 cuBLAS
 * GEMMs, which torch 1.9.1 runs as TF32, ~2^-11, on Ampere by default). */
int cmt_gemm_bf16x3_ex(const cmt_gemm_ex_args* args, void* stream);
/* A Linear's backward in one call (ABI 23) on cmt_gemm_bf16x3_ex's arithmetic:
 * dX[M][K] = dY W (dX optional), dW[N][K] = dY^T X and dB[N] = the column sums of
 * dY (both optional; dB needs dW), with dY [M][N] and W [N][K] contiguous and X
 * [M][K] of row stride ldx.  dW and dB are overwritten: when the weight-gradient
 * reduction is split (ksplit > 1) or dB is asked for, they are zeroed on the
 * stream first and accumulated with f32 atomics.  Replaces, per call, the two
 * GEMM launches and the zero fill a caller of cmt_gemm_bf16x3_ex issues. */
int cmt_linear_bwd_bf16x3(const float* dY, const float* X, const float* W, float* dX, float* dW, float* dB,
                          int M, int K, int N, int64_t ldx, int ksplit, void* stream);
/* cmt_linear_bwd_bf16x3_ex (ABI 24): the same with flags.  CMT_LINEAR_BWD_ACCUMULATE: dW and dB
 * already hold a sum (a parameter's gradient) and the call ADDS to it -- no zero fill, the weight
 * gradient read-modify-written (unsplit) or f32-atomically added (split), the bias gradient added
 * atomically: the training step writes each Linear's weight gradient straight into the
 * parameter's .grad instead of returning it for autograd to add. */
#define CMT_LINEAR_BWD_ACCUMULATE 1
int cmt_linear_bwd_bf16x3_ex(const float* dY, const float* X, const float* W, float* dX, float* dW, float* dB,
                             int M, int K, int N, int64_t ldx, int ksplit, int flags, void* stream);

/* Attention forward with row statistics, and its backward (attn_train.hip),
 * exact f32, head_dim 32.  Replaces, in the training step, the fp32
 * self-attention core of nn.MultiheadAttention (with the DN mask of
 * cmt_head.py:386-398 and attn_drop) and the flash-attn 0.2.2 cross core
 * (attention.py:46-92; fp16_inputs = 1 rounds q, k, v, P and O to fp16 like
 * that core).  Element (b, h, row, d) of X at X[b*x_bs + h*x_hs + row*x_rs + d];
 * dQ / dK / dV use the strides of Q / K / V, dO those of O.
 * fwd writes O and LSE[b][h][q] = log2 sum_k exp2(c s_qk) (c = scale log2 e);
 * bwd reads Q, K, V, O, dO, LSE and writes dQ, dK, dV (delta: [B*H*Nq] scratch).
 * DN mask (dn_pad > 0): key k < dn_pad is hidden from query q if q >= dn_pad or
 * k / dn_group != q / dn_group.  dropout_p > 0: keep(q, k) from a counter hash
 * of (seed, b, h, q, k), identical in fwd and bwd (training only). */
typedef struct cmt_attn_train_args {
    int B, H, Nq, Nk;
    const float* Q; int64_t q_bs, q_hs, q_rs;
    const float* K; int64_t k_bs, k_hs, k_rs;
    const float* V; int64_t v_bs, v_hs, v_rs;
    float* O; int64_t o_bs, o_hs, o_rs;
    float* LSE;
    const float* dO; float* dQ; float* dK; float* dV; float* delta;
    float scale;
    int dn_pad, dn_group;
    int fp16_inputs;
    float dropout_p; uint32_t seed;
    int kv_splits;             /* fwd: 0 = automatic */
    void* workspace; int64_t workspace_bytes;
    const uint32_t* seed_dev;  /* ABI 22, optional: the dropout seed is seed + *seed_dev, read on the
                                * device (a graph-replayed step draws a fresh seed without re-capture) */
    int ws_reuse;              /* ABI 25, backward of the long-key path: nonzero = the workspace is the one
                                * the forward ran with on the same Q / K / V, so its f16 copies of them are
                                * reused and only dO is converted */
} cmt_attn_train_args;
/* Long-key fp16 path (ABI 15; fp16_inputs, no DN mask, no dropout, Nk >= 4096,
 * 128 < Nq <= 1152, heads contiguous in O (o_hs == 32), kv_splits 0 -- the
 * cross-attention of the training step): the forward runs cmt_attn_fwd's
 * bounded long-key core with the row statistic, the backward the dK/dV kernel
 * with the head's Q / dO resident in LDS and a K/V-streaming dQ kernel, all on
 * f16 copies of the operands held in the workspace.  cmt_attn_train_workspace_bytes
 * covers both directions; the forward returns CMT_EWORKSPACE on this path
 * with a smaller workspace, the backward runs the general kernels with less. */
int64_t cmt_attn_train_workspace_bytes(const cmt_attn_train_args* args);
int cmt_attn_train_fwd(const cmt_attn_train_args* args, void* stream);
int cmt_attn_train_bwd(const cmt_attn_train_args* args, void* stream);

/* Row LayerNorm with saved statistics (C = 64 or 256): nn.LayerNorm
 * (mmcv LN, eps 1e-5) of the decoder and, with C = 64, eps 1e-6 and one weight
 * set per rows_per_wset rows, GroupLayerNorm1d (cmt_head.py:53-94) whose
 * custom backward (68-81) is the LayerNorm backward:
 *   dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy w;
 *   dW[set] += sum dy xhat, dB[set] += sum dy (f32 atomics; zero them first). */
typedef struct cmt_ln_train_args {
    int rows, C;
    const float* X; int64_t ldx;
    const float* W; const float* B; float eps;
    int rows_per_wset;         /* 0 = one weight set */
    float* Y; int64_t ldy;     /* fwd output; bwd: dY reads ldy */
    float* mean; float* rstd;  /* [rows] saved by fwd, read by bwd */
    const float* dY; float* dX; int64_t lddx; int accumulate;
    float* dW; float* dB;
} cmt_ln_train_args;
int cmt_ln_train_fwd(const cmt_ln_train_args* args, void* stream);
int cmt_ln_train_bwd(const cmt_ln_train_args* args, void* stream);

/* BatchNorm2d in training mode (batch statistics over all NHWC rows, running
 * stats updated with momentum, unbiased running var) fused with ReLU: the
 * shared_conv ConvModule (cmt_head.py:280-287) after its 3x3 conv; and its
 * backward (dX, dW, dB).  workspace: cmt_bn_workspace_bytes(C). */
typedef struct cmt_bn_args {
    int rows, C;
    const float* X; float* Y;
    const float* W; const float* B; float eps; float momentum;
    float* running_mean; float* running_var;   /* optional */
    float* mean_save; float* rstd_save;        /* [C] */
    const float* dY; float* dX; float* dW; float* dB;
    void* workspace;
} cmt_bn_args;
int64_t cmt_bn_workspace_bytes(int C);
int cmt_bn_relu_train_fwd(const cmt_bn_args* args, void* stream);
int cmt_bn_relu_train_bwd(const cmt_bn_args* args, void* stream);

/* im2col of the 3x3 / pad 1 conv on NHWC rows (the weight-gradient operand of
 * shared_conv): out[(img*H+y)*W+x][tap*C + c], tap = 3*dy + dx. */
int cmt_im2col3x3(const float* X, int nimg, int H, int W, int C, float* out, void* stream);
/* The same weight gradient without the im2col matrix (ABI 21): dW[cout][tap*Cin + c]
 * = sum over the nimg*H*W rows r of dY[r][cout] * im2col(X)[r][tap*Cin + c], the
 * im2col elements gathered inside cmt_gemm_bf16x3_ex's kernel (its arithmetic);
 * ksplit > 1 adds into dW with f32 atomics (zero it first), 1 overwrites it.
 * Cin, Cout multiples of 4; X, dY 16-byte aligned. */
int cmt_conv3x3_wgrad_bf16x3(const float* X, const float* dY, float* dW, int nimg, int H, int W, int Cin,
                             int Cout, int ksplit, void* stream);

/* FocalLoss(use_sigmoid, gamma, alpha) + L1Loss of one task / decoder layer
 * (mmdet 2.28.2; cmt_head.py:702-720, 777-812): out[0] = cls loss, out[1] =
 * box loss; dlogits / dboxes (optional) receive d(loss)/d(input) * gscale.
 * labels == ncls is background.  One workgroup, fixed reduction order. */
typedef struct cmt_det_loss_args {
    int R, ncls;
    const float* logits; int64_t ld_logits;
    const int* labels; const float* label_w;
    int Rb;
    const float* boxes; int64_t ld_boxes;
    const float* targets; const float* box_w;  /* [Rb][10] */
    float gamma, alpha, cls_weight, box_weight, cls_avg, box_avg, gscale;
    float* out;                                 /* [2] */
    float* dlogits; float* dboxes;
} cmt_det_loss_args;
int cmt_det_loss(const cmt_det_loss_args* args, void* stream);

/* Hungarian cost matrix of HungarianAssigner3D (hungarian_assigner_3d.py:
 * 120-136): FocalLossCost (eps 1e-12) * cls_weight + BBox3DL1Cost over the
 * first 8 code-weighted box channels * reg_weight.  cost [Nq][ngt]. */
typedef struct cmt_match_cost_args {
    int Nq, ngt;
    const float* logits; int64_t ld_logits;
    const float* boxes; int64_t ld_boxes;
    const float* gt; const int* gt_labels;      /* gt [ngt][10] normalized */
    const float* code_w;                         /* [10] device */
    float gamma, alpha, cls_weight, reg_weight;
    float* cost;
} cmt_match_cost_args;
int cmt_match_cost(const cmt_match_cost_args* args, void* stream);

/* cmt_sumsq: *out += sum x^2 (zero *out first).  cmt_adamw_step:
 * torch.optim.AdamW over a flat buffer; if max_norm > 0 the gradient is scaled
 * by min(1, max_norm / (sqrt(*sumsq) + 1e-6)) (clip_grad_norm_, mmcv
 * OptimizerHook grad_clip). */
int cmt_sumsq(const float* x, int64_t n, float* out, void* stream);
typedef struct cmt_adamw_args {
    int64_t n; int step;
    float lr, beta1, beta2, eps, weight_decay, max_norm;
    float* param; const float* grad; float* exp_avg; float* exp_avg_sq;
    const float* sumsq;
} cmt_adamw_args;
int cmt_adamw_step(const cmt_adamw_args* args, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CMT_HIP_H */
