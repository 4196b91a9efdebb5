"""ctypes binding of libcmt_hip.so (the C ABI declared in include/cmt_hip.h).

This is the ONLY way the product path computes: every wrapper below checks
that its tensors live on a HIP device and raises if the library is missing --
there is no CPU or eager-PyTorch fallback.  PyTorch provides device memory,
the current stream and graph capture (plumbing); the arithmetic happens in the
hand-written gfx950 kernels.
"""
import ctypes
import os

import torch

__all__ = ["lib", "available", "gemm", "split_rows", "width", "lstride", "F16P", "gemm_ln", "chain", "kv_proj", "kv_pack", "attention", "layernorm", "layernorm_ex", "add_cast", "pos2embed",
           "rv_pe_coords",
           "rv_query_coords", "masked_view_sum", "nchw_to_rows", "cast", "task_head_tail",
           "voxelize", "box_decode", "DT", "dtype_code", "LN_NAN_TO_NUM", "LN_MAX_INTO"]

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_DEFAULT_LIB = os.path.join(_PKG_ROOT, "lib", "libcmt_hip.so")

F32, F16, BF16, F16P = 0, 1, 2, 3
# torch.uint16 (runtime.SPLIT) carries the split pair format CMT_F16P: a logical
# [..., C] operand stored as [..., 2, C] (f16 hi values, then f16 lo values)
DT = {torch.float32: F32, torch.float16: F16, torch.bfloat16: BF16, torch.uint16: F16P}
LN_NAN_TO_NUM, LN_MAX_INTO = 1, 2
A_ROWS, A_CONV3X3, A_CONV1D3, A_CONV3X3_NCHW = 0, 1, 2, 3
C_ROWS, C_HEADSPLIT = 0, 1
A2_ADD, A2_SELECT = 0, 1
ATTN_KEEP_PARTIALS = 2048   # cmt_hip.h CMT_ATTN_KEEP_PARTIALS (ABI 19)
LINEAR_BWD_ACCUMULATE = 1   # cmt_hip.h CMT_LINEAR_BWD_ACCUMULATE (ABI 24)
CHAIN_XSPLITS = 8           # the split count chain B1 combines (cmt_chain_args.xsplits)
ABI_VERSION = 25
PLANE_MAX_ROWS = 64   # key rows per plane_max2 / kmax2 entry (cmt_hip.h)

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_flt = ctypes.c_float


class GemmArgs(ctypes.Structure):
    _fields_ = [("M", _int), ("N", _int), ("K", _int), ("batch", _int),
                ("A", _vp), ("lda", _i64), ("a_bstride", _i64), ("a_dtype", _int),
                ("A2", _vp), ("lda2", _i64), ("a2_cols", _int), ("a2_mode", _int),
                ("a_mode", _int), ("conv_h", _int), ("conv_w", _int), ("conv_c", _int), ("seg_len", _int),
                ("W", _vp), ("ldw", _i64), ("w_bstride", _i64), ("w_dtype", _int),
                ("bias", _vp), ("bias_bstride", _i64),
                ("R", _vp), ("ldr", _i64), ("r_bstride", _i64), ("r_dtype", _int),
                ("C", _vp), ("ldc", _i64), ("c_bstride", _i64), ("c_dtype", _int),
                ("c_mode", _int), ("rows_per_batch", _int), ("relu", _int),
                ("plane_max2", _vp), ("plane_max_cols", _int),
                ("k_splits", _int), ("c_split_stride", _i64), ("range_flag", _vp)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("B", _int), ("H", _int), ("Nq", _int), ("Nk", _int), ("dtype", _int),
                ("Q", _vp), ("q_bstride", _i64), ("q_hstride", _i64), ("q_rstride", _i64),
                ("K", _vp), ("k_bstride", _i64), ("k_hstride", _i64), ("k_rstride", _i64),
                ("V", _vp), ("v_bstride", _i64), ("v_hstride", _i64), ("v_rstride", _i64),
                ("O", _vp), ("o_bstride", _i64), ("o_rstride", _i64), ("o_dtype", _int), ("scale", _flt),
                ("kv_splits", _int),
                ("flags", _int),
                ("workspace", _vp), ("workspace_bytes", _i64),
                ("kmax2", _vp), ("kmax_ld", _int), ("kmax_plane0", _int), ("kmax_rows", _int)]


class ChainArgs(ctypes.Structure):
    _fields_ = [("kind", _int), ("rows", _int), ("Nq", _int), ("dtype", _int), ("eps", _flt),
                ("X", _vp), ("R", _vp), ("P", _vp), ("prm", _vp),
                ("Wo", _vp), ("W1", _vp), ("W2", _vp), ("Wn", _vp),
                ("Y", _vp), ("OUT", _vp), ("out_flags", _int), ("Q", _vp), ("WS", _vp),
                ("OUT16", _vp), ("wo_frag", _int),
                ("xpart", _vp), ("xsplits", _int), ("xround", _int)]


class LnArgs(ctypes.Structure):
    _fields_ = [("X", _vp), ("ldx", _i64), ("rows", _int), ("C", _int),
                ("W", _vp), ("B", _vp), ("eps", _flt),
                ("Y", _vp), ("ldy", _i64), ("flags", _int),
                ("W2", _vp), ("B2", _vp), ("Y2", _vp), ("ldy2", _i64), ("flags2", _int),
                ("lowp_dtype", _int),
                ("Yl", _vp), ("ldyl", _i64),
                ("Yp", _vp), ("ldyp", _i64), ("P", _vp), ("ldp", _i64),
                ("nparts", _int), ("part_stride", _i64)]


class GemmExArgs(ctypes.Structure):
    _fields_ = [("M", _int), ("N", _int), ("K", _int), ("batch", _int), ("alpha", _flt), ("beta", _flt),
                ("A", _vp), ("a_sm", _i64), ("a_sk", _i64), ("a_bs", _i64),
                ("B", _vp), ("b_sn", _i64), ("b_sk", _i64), ("b_bs", _i64),
                ("C", _vp), ("ldc", _i64), ("c_bs", _i64), ("bias", _vp), ("ksplit", _int),
                ("bias_bs", _i64), ("a_rowsum", _vp)]


class AttnTrainArgs(ctypes.Structure):
    _fields_ = [("B", _int), ("H", _int), ("Nq", _int), ("Nk", _int),
                ("Q", _vp), ("q_bs", _i64), ("q_hs", _i64), ("q_rs", _i64),
                ("K", _vp), ("k_bs", _i64), ("k_hs", _i64), ("k_rs", _i64),
                ("V", _vp), ("v_bs", _i64), ("v_hs", _i64), ("v_rs", _i64),
                ("O", _vp), ("o_bs", _i64), ("o_hs", _i64), ("o_rs", _i64),
                ("LSE", _vp), ("dO", _vp), ("dQ", _vp), ("dK", _vp), ("dV", _vp), ("delta", _vp),
                ("scale", _flt), ("dn_pad", _int), ("dn_group", _int), ("fp16_inputs", _int),
                ("dropout_p", _flt), ("seed", ctypes.c_uint32), ("kv_splits", _int),
                ("workspace", _vp), ("workspace_bytes", _i64), ("seed_dev", _vp), ("ws_reuse", _int)]


class LnTrainArgs(ctypes.Structure):
    _fields_ = [("rows", _int), ("C", _int), ("X", _vp), ("ldx", _i64), ("W", _vp), ("B", _vp), ("eps", _flt),
                ("rows_per_wset", _int), ("Y", _vp), ("ldy", _i64), ("mean", _vp), ("rstd", _vp),
                ("dY", _vp), ("dX", _vp), ("lddx", _i64), ("accumulate", _int), ("dW", _vp), ("dB", _vp)]


class BnArgs(ctypes.Structure):
    _fields_ = [("rows", _int), ("C", _int), ("X", _vp), ("Y", _vp), ("W", _vp), ("B", _vp), ("eps", _flt),
                ("momentum", _flt), ("running_mean", _vp), ("running_var", _vp), ("mean_save", _vp),
                ("rstd_save", _vp), ("dY", _vp), ("dX", _vp), ("dW", _vp), ("dB", _vp), ("workspace", _vp)]


class DetLossArgs(ctypes.Structure):
    _fields_ = [("R", _int), ("ncls", _int), ("logits", _vp), ("ld_logits", _i64), ("labels", _vp), ("label_w", _vp),
                ("Rb", _int), ("boxes", _vp), ("ld_boxes", _i64), ("targets", _vp), ("box_w", _vp),
                ("gamma", _flt), ("alpha", _flt), ("cls_weight", _flt), ("box_weight", _flt), ("cls_avg", _flt),
                ("box_avg", _flt), ("gscale", _flt), ("out", _vp), ("dlogits", _vp), ("dboxes", _vp)]


class MatchCostArgs(ctypes.Structure):
    _fields_ = [("Nq", _int), ("ngt", _int), ("logits", _vp), ("ld_logits", _i64), ("boxes", _vp), ("ld_boxes", _i64),
                ("gt", _vp), ("gt_labels", _vp), ("code_w", _vp), ("gamma", _flt), ("alpha", _flt),
                ("cls_weight", _flt), ("reg_weight", _flt), ("cost", _vp)]


class AdamwArgs(ctypes.Structure):
    _fields_ = [("n", _i64), ("step", _int), ("lr", _flt), ("beta1", _flt), ("beta2", _flt), ("eps", _flt),
                ("weight_decay", _flt), ("max_norm", _flt), ("param", _vp), ("grad", _vp), ("exp_avg", _vp),
                ("exp_avg_sq", _vp), ("sumsq", _vp)]


class Mlp2Args(ctypes.Structure):
    _fields_ = [("M", _int), ("K", _int), ("Hd", _int), ("N", _int), ("batch", _int),
                ("A", _vp), ("lda", _i64), ("a_bstride", _i64),
                ("W1p", _vp), ("b1", _vp), ("W2p", _vp), ("b2", _vp),
                ("R", _vp), ("ldr", _i64), ("r_bstride", _i64), ("r_dtype", _int),
                ("C", _vp), ("ldc", _i64), ("c_bstride", _i64), ("c_dtype", _int),
                ("geo_i2l", _vp), ("geo_h", _int), ("geo_w", _int), ("geo_D", _int), ("geo_pad_h", _flt),
                ("geo_pad_w", _flt), ("geo_depth_max", _flt), ("geo_pc", _flt * 6),
                ("rx", _vp), ("C2", _vp), ("ldc2", _i64), ("c2_bstride", _i64), ("range_flag", _vp)]


STRUCTS = {"gemm": GemmArgs, "attn": AttnArgs, "ln": LnArgs, "chain": ChainArgs, "gemm_ex": GemmExArgs,
           "attn_train": AttnTrainArgs, "ln_train": LnTrainArgs, "bn": BnArgs, "det_loss": DetLossArgs,
           "match_cost": MatchCostArgs, "adamw": AdamwArgs, "mlp2": Mlp2Args}

_LIB = None


def _load():
    path = os.environ.get("CMT_HIP_LIB", _DEFAULT_LIB)
    if not os.path.exists(path):
        raise RuntimeError(
            f"libcmt_hip.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C cmt-cooperative-perception_amd/csrc`).  There is no fallback path.")
    torch.cuda.init() if torch.cuda.is_available() else None  # share torch's HIP runtime (same soname)
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    sig = {
        "cmt_abi_version": ([], _int),
        "cmt_last_error": ([], ctypes.c_char_p),
        "cmt_gemm": ([P(GemmArgs), _vp], _int),
        "cmt_attn_workspace_bytes": ([P(AttnArgs)], _i64),
        "cmt_attn_splits": ([P(AttnArgs)], _int),
        "cmt_attn_fwd": ([P(AttnArgs), _vp], _int),
        "cmt_layernorm": ([_vp, _i64, _int, _int, _vp, _vp, _flt, _vp, _i64, _int, _vp, _vp, _vp, _i64, _int, _vp],
                          _int),
        "cmt_layernorm_ex": ([P(LnArgs), _vp], _int),
        "cmt_gemm_ln": ([P(GemmArgs), P(LnArgs), _vp], _int),
        "cmt_chain": ([P(ChainArgs), _vp], _int),
        "cmt_kv_proj": ([P(GemmArgs), _vp], _int),
        "cmt_mlp2_x3": ([P(Mlp2Args), _vp], _int),
        "cmt_mlp2_args_size": ([], _i64),
        "cmt_add_cast": ([_vp, _vp, _int, _int, _int, _vp, _vp, _vp], _int),
        "cmt_pos2embed": ([_vp, _i64, _int, _int, _int, _int, _int, _vp, _int, _i64, _vp], _int),
        "cmt_rv_pe_coords": ([_int, _int, _int, _int, _flt, _flt, _flt, _vp, P(_flt), _vp, _int, _vp], _int),
        "cmt_rv_query_coords": ([_vp, _int, _int, _int, _int, _flt, _flt, _vp, _vp, P(_flt), _vp, _vp, _vp], _int),
        "cmt_masked_view_sum": ([_vp, _vp, _int, _int, _int, _int, _vp, _vp], _int),
        "cmt_rv_query_coords_ex": ([_vp, _int, _int, _int, _int, _flt, _flt, _vp, _vp, P(_flt), _vp, _int, _vp, _vp],
                                   _int),
        "cmt_masked_view_sum_ex": ([_vp, _vp, _int, _int, _int, _int, _vp, _vp, _vp, _vp, _int, _vp], _int),
        "cmt_nchw_to_rows": ([_vp, _int, _int, _int, _int, _vp, _int, _i64, _i64, _i64, _vp], _int),
        "cmt_nchw_to_rows_ex": ([_vp, _int, _int, _int, _int, _vp, _int, _i64, _i64, _i64, _vp, _vp], _int),
        "cmt_cast": ([_vp, _int, _vp, _int, _i64, _vp], _int),
        "cmt_split_rows": ([_vp, _i64, _i64, _int, _vp, _vp], _int),
        "cmt_task_head_tail": ([_vp, _int, _int, _int, _int, _int, _vp, _vp, _vp, _vp, P(_int), _int, _int, _vp,
                                _int, _int, P(_flt), _vp, _vp], _int),
        "cmt_box_decode": ([_vp, _i64, _vp, _i64, _vp, _int, _int, _int, _int, _int, P(_flt), _flt, _int,
                            _vp, _vp, _vp, _vp, _vp], _int),
        "cmt_voxelize_workspace_bytes": ([_int, _int], _i64),
        "cmt_voxelize_workspace_init": ([_vp, _i64, _vp], _int),
        "cmt_voxelize": ([_vp, _int, _int, P(_flt), P(_flt), P(_int), _int, _int, _int, _vp, _vp, _vp, _vp, _vp,
                          _vp, _i64, _vp], _int),
        "cmt_gemm_args_size": ([], _i64),
        "cmt_attn_args_size": ([], _i64),
        "cmt_ln_args_size": ([], _i64),
        "cmt_chain_args_size": ([], _i64),
        "cmt_chain_ws_bytes": ([_int], _i64),
        "cmt_gemm_ex_args_size": ([], _i64),
        "cmt_attn_train_args_size": ([], _i64),
        "cmt_ln_train_args_size": ([], _i64),
        "cmt_bn_args_size": ([], _i64),
        "cmt_det_loss_args_size": ([], _i64),
        "cmt_match_cost_args_size": ([], _i64),
        "cmt_adamw_args_size": ([], _i64),
        "cmt_gemm_f32_ex": ([P(GemmExArgs), _vp], _int),
        "cmt_gemm_bf16x3_ex": ([P(GemmExArgs), _vp], _int),
        "cmt_linear_bwd_bf16x3": ([_vp, _vp, _vp, _vp, _vp, _vp, _int, _int, _int, _i64, _int, _vp], _int),
        "cmt_linear_bwd_bf16x3_ex": ([_vp, _vp, _vp, _vp, _vp, _vp, _int, _int, _int, _i64, _int, _int, _vp], _int),
        "cmt_attn_train_workspace_bytes": ([P(AttnTrainArgs)], _i64),
        "cmt_attn_train_fwd": ([P(AttnTrainArgs), _vp], _int),
        "cmt_attn_train_bwd": ([P(AttnTrainArgs), _vp], _int),
        "cmt_ln_train_fwd": ([P(LnTrainArgs), _vp], _int),
        "cmt_ln_train_bwd": ([P(LnTrainArgs), _vp], _int),
        "cmt_bn_workspace_bytes": ([_int], _i64),
        "cmt_bn_relu_train_fwd": ([P(BnArgs), _vp], _int),
        "cmt_bn_relu_train_bwd": ([P(BnArgs), _vp], _int),
        "cmt_im2col3x3": ([_vp, _int, _int, _int, _int, _vp, _vp], _int),
        "cmt_conv3x3_wgrad_bf16x3": ([_vp, _vp, _vp, _int, _int, _int, _int, _int, _int, _vp], _int),
        "cmt_det_loss": ([P(DetLossArgs), _vp], _int),
        "cmt_match_cost": ([P(MatchCostArgs), _vp], _int),
        "cmt_sumsq": ([_vp, _i64, _vp, _vp], _int),
        "cmt_adamw_step": ([P(AdamwArgs), _vp], _int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.cmt_abi_version() != ABI_VERSION:
        raise RuntimeError("libcmt_hip.so ABI version mismatch")
    for name, st in STRUCTS.items():
        got = getattr(L, f"cmt_{name}_args_size")()
        if got != ctypes.sizeof(st):
            raise RuntimeError(f"cmt_{name}_args: library struct is {got} bytes, the ctypes mirror "
                               f"{ctypes.sizeof(st)} (stale binding)")
    return L


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _load()
    return _LIB


def available():
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


def _check(rc, name):
    if rc != 0:
        msg = lib().cmt_last_error().decode("utf-8", "replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("CMT HIP ops need tensors on a HIP device (no CPU fallback)")


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_cur_device = torch._C._cuda_getDevice
_cur_raw_stream = torch._C._cuda_getCurrentRawStream


def _stream():
    """the current HIP stream of the current device (torch.cuda.current_stream() costs ~10 us of
    device-index bookkeeping per call: a training step launches ~3 000 native kernels)"""
    return ctypes.c_void_p(_cur_raw_stream(_cur_device()))


def dtype_code(dt):
    return DT[dt]


def _farr(vals, n):
    arr = (ctypes.c_float * n)(*[float(v) for v in vals])
    return arr


# ---------------------------------------------------------------------------
def gemm(A, W, C, *, M, N, K, lda, ldw, ldc, bias=None, relu=False, R=None, ldr=0, A2=None, lda2=0, a2_cols=0,
         a_mode=A_ROWS, conv=(0, 0, 0), seg_len=0, batch=1, a_bstride=0, w_bstride=0, bias_bstride=0,
         r_bstride=0, c_bstride=0, headsplit_rows=0, a_offset=0, c_offset=0, r_offset=0, a2_offset=0,
         plane_max2=None, plane_max_cols=0, k_splits=0, c2=None, range_flag=None):
    """C = act(A W^T + bias) + R with the fused prologue/epilogue of cmt_gemm.
    Offsets are in elements of the respective tensor.  A2 of A's dtype selects
    (replaces A for output columns < a2_cols); an fp32 A2 beside fp32 A is
    added on load.  plane_max2 (fp32 [ceil(M/64), plane_max_cols/32], head-split
    16-bit C only) receives the per-64-row max squared row norm of each head plane.
    k_splits >= 2: C holds k_splits fp32 partial blocks of M * ldc elements whose sum
    is the output (bias and R in the first); a layernorm_ex(nparts=k_splits) reduces them.
    c2 (a_mode A_CONV3X3_NCHW with fp32 A2 rows): a second output out + A2, laid out like C.
    range_flag (int32 device word; split x3 kernels): set to 1 by the kernel when a value
    falls outside the f16-pair format (cmt_hip.h cmt_gemm_args.range_flag)."""
    if k_splits > 1 and C.numel() < k_splits * M * ldc:
        raise RuntimeError("gemm: a split-K C needs k_splits blocks of M * ldc elements")
    g = _gemm_args(A, W, C, M=M, N=N, K=K, lda=lda, ldw=ldw, ldc=ldc, bias=bias, relu=relu, R=R, ldr=ldr, A2=A2,
                   lda2=lda2, a2_cols=a2_cols, a_mode=a_mode, conv=conv, seg_len=seg_len, batch=batch,
                   a_bstride=a_bstride, w_bstride=w_bstride, bias_bstride=bias_bstride, r_bstride=r_bstride,
                   c_bstride=c_bstride, headsplit_rows=headsplit_rows, a_offset=a_offset, c_offset=c_offset,
                   r_offset=r_offset, a2_offset=a2_offset)
    if plane_max2 is not None:
        _dev(plane_max2)
        if plane_max2.dtype != torch.float32 or plane_max2.numel() < -(-M // PLANE_MAX_ROWS) * (plane_max_cols // 32):
            raise RuntimeError("plane_max2 must be fp32 with ceil(M/64) * plane_max_cols/32 entries")
        g.plane_max2, g.plane_max_cols = plane_max2.data_ptr(), plane_max_cols
    if k_splits > 1:
        g.k_splits, g.c_split_stride = k_splits, M * ldc
    if range_flag is not None:
        _dev(range_flag)
        if range_flag.dtype != torch.int32:
            raise RuntimeError("gemm: range_flag must be an int32 device word")
        g.range_flag = range_flag.data_ptr()
    if c2 is not None:
        # a second output (A_CONV3X3_NCHW with A2): C's layout, at c_offset elements into c2
        _dev(c2)
        if c2.dtype != C.dtype or k_splits > 1:
            raise RuntimeError("gemm: c2 must have C's dtype (and no split-K)")
        es = C.element_size()
        d = c2.data_ptr() + c_offset * _ps(C) * es - g.C
        if d % es:
            raise RuntimeError("gemm: c2 misaligned against C")
        g.c_split_stride = d // es
    _check(lib().cmt_gemm(ctypes.byref(g), _stream()), "cmt_gemm")


def kv_pack(W):
    """Fragment-packed copy of a [N][256] K/V projection weight for cmt_kv_proj
    (cmt_hip.h): plane p, k-step ks, lane -> 8 consecutive k of row 32p + lane % 32."""
    n, k = W.shape
    if n % 32 or k != 256:
        raise RuntimeError("kv_pack: W must be [N % 32 == 0][256]")
    return W.reshape(n // 32, 32, 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()


def kv_proj(A, Wp, C, *, M, N, bias=None, A2=None, headsplit_rows, plane_max2=None, plane_max_cols=0,
            c_offset=0, c_bstride=0):
    """Cross-attention K/V projection (cmt_kv_proj): columns < N/2 read A2
    (lowp(mem + pos)) when given, the rest A (lowp(mem)); Wp from kv_pack;
    head-split C starting ``c_offset`` elements in, batch stride ``c_bstride``
    elements (0: the launch's own N/32 planes); optional per-64-row key-norm
    maxima (as cmt_gemm)."""
    g = _gemm_args(A, Wp, C, M=M, N=N, K=256, lda=256, ldw=256, ldc=0, bias=bias, A2=A2,
                   lda2=256 if A2 is not None else 0, a2_cols=N // 2 if A2 is not None else 0,
                   headsplit_rows=headsplit_rows, c_offset=c_offset, c_bstride=c_bstride)
    if C.numel() < c_offset + (M // headsplit_rows - 1) * (c_bstride or N * headsplit_rows) + N * headsplit_rows:
        raise RuntimeError("kv_proj: C is too small for the launch's planes")
    if plane_max2 is not None:
        _dev(plane_max2)
        if plane_max2.dtype != torch.float32 or plane_max2.numel() < -(-M // PLANE_MAX_ROWS) * (plane_max_cols // 32):
            raise RuntimeError("plane_max2 must be fp32 with ceil(M/64) * plane_max_cols/32 entries")
        g.plane_max2, g.plane_max_cols = plane_max2.data_ptr(), plane_max_cols
    _check(lib().cmt_kv_proj(ctypes.byref(g), _stream()), "cmt_kv_proj")


def mlp2_pack(W1, W2):
    """Fragment packs of the pair weights of Linear(K, Hd) -> ReLU -> Linear(Hd, 256)
    for cmt_mlp2_x3 (cmt_hip.h): W1 [Hd, 2, K], W2 [256, 2, Hd] (runtime.SPLIT)
    -> (W1p, W2p).  W2p orders each 16-unit k-step of a 32-unit hidden block as
    the hidden accumulator's registers: position 8 lh + j holds unit
    8 (j >> 2) + 4 lh + (j & 3)."""
    if W1.dtype != torch.uint16 or W2.dtype != torch.uint16 or W1.dim() != 3 or W2.dim() != 3:
        raise RuntimeError("mlp2_pack: W1 / W2 must be split pair weights [N, 2, K]")
    hd, _, k = W1.shape
    n, _, hd2 = W2.shape
    if hd2 != hd or n != 256 or hd % 32 or k % 16:
        raise RuntimeError("mlp2_pack: W1 [Hd, 2, K] and W2 [256, 2, Hd] with Hd % 32 == 0, K % 16 == 0")
    # W1p[hb][ks][pl][lh][lr][j] = W1[32 hb + lr][pl][16 ks + 8 lh + j]
    w1p = W1.view(hd // 32, 32, 2, k // 16, 2, 8).permute(0, 3, 2, 4, 1, 5).contiguous()
    # W2p[hb][ot][s][pl][lh][lr][jh][jl] = W2[32 ot + lr][pl][32 hb + 16 s + 8 jh + 4 lh + jl]
    w2p = W2.view(8, 32, 2, hd // 32, 2, 2, 2, 4).permute(3, 0, 4, 2, 6, 1, 5, 7).contiguous()
    return w1p, w2p


def mlp2(A, W1p, b1, W2p, b2, C, *, M, K, Hd, R=None, batch=1, a_bstride=0, c_offset=0, c_bstride=0,
         r_offset=0, r_bstride=0, geo=None, rx=None, C2=None, c2_offset=0, c2_bstride=0, range_flag=None):
    """C = Linear2(ReLU(Linear1(A) + b1)) + b2 (+ R) in one launch (cmt_mlp2_x3):
    A pair rows [.., 2, K]; packs from mlp2_pack; C / R fp32 [.., 256] or pair
    [.., 2, 256] rows.  Offsets and strides are LOGICAL (rows of the operand).
    ABI 20, the camera memory rows in one launch: geo = dict(i2l, h, w, D, pad_h, pad_w,
    depth_max, pc_range) generates A (the _rv_pe frustum coordinates; A is then None), rx (NCHW
    fp32 image features) replaces R, and C2 (pair rows) receives the memory rows themselves."""
    _dev(A, W1p, b1, W2p, b2, C, R, rx, C2, range_flag)
    if (A is not None and A.dtype != torch.uint16) or W1p.dtype != torch.uint16 or W2p.dtype != torch.uint16:
        raise RuntimeError("mlp2: A and the packs must be split pairs (torch.uint16)")
    if (geo is None) != (rx is None) or (geo is None) != (C2 is None) or (geo is None) == (A is None):
        raise RuntimeError("mlp2: give A, or geo + rx + C2 (the fused camera-row form)")
    g = Mlp2Args()
    g.M, g.K, g.Hd, g.N, g.batch = M, K, Hd, 256, batch
    if A is not None:
        g.A, g.lda, g.a_bstride = A.data_ptr(), lstride(A) * 2, a_bstride * 2
    else:
        _dev(geo["i2l"])
        if rx.dtype != torch.float32 or not rx.is_contiguous() or C2.dtype != torch.uint16:
            raise RuntimeError("mlp2: rx must be contiguous NCHW fp32, C2 pair rows")
        g.geo_i2l = geo["i2l"].data_ptr()
        g.geo_h, g.geo_w, g.geo_D = geo["h"], geo["w"], geo["D"]
        g.geo_pad_h, g.geo_pad_w, g.geo_depth_max = geo["pad_h"], geo["pad_w"], geo["depth_max"]
        for i in range(6):
            g.geo_pc[i] = float(geo["pc_range"][i])
        g.rx = rx.data_ptr()
        g.C2 = C2.data_ptr() + c2_offset * 2 * C2.element_size()   # logical elements (pair: 2 words each)
        g.ldc2, g.c2_bstride = lstride(C2) * 2, c2_bstride * 2
        if range_flag is not None:
            if range_flag.dtype != torch.int32:
                raise RuntimeError("mlp2: range_flag must be an int32 device word")
            g.range_flag = range_flag.data_ptr()
    g.W1p, g.b1, g.W2p, g.b2 = W1p.data_ptr(), b1.data_ptr(), W2p.data_ptr(), b2.data_ptr()
    sc = _ps(C)
    g.C = C.data_ptr() + c_offset * sc * C.element_size()
    g.ldc, g.c_bstride, g.c_dtype = lstride(C) * sc, c_bstride * sc, DT[C.dtype]
    if R is not None:
        sr = _ps(R)
        g.R = R.data_ptr() + r_offset * sr * R.element_size()
        g.ldr, g.r_bstride, g.r_dtype = lstride(R) * sr, r_bstride * sr, DT[R.dtype]
    else:
        g.R, g.ldr, g.r_bstride, g.r_dtype = None, 0, 0, F32
    _check(lib().cmt_mlp2_x3(ctypes.byref(g), _stream()), "cmt_mlp2_x3")


def _ps(t):
    """Physical 16-bit words per logical element: 2 for a split f16 pair
    tensor, else 1.  Strides and offsets of the wrappers below are LOGICAL
    (elements of the [..., C] operand) and scaled by this; pair offsets must
    be whole rows."""
    return 2 if t is not None and t.dtype == torch.uint16 else 1


def width(t):
    """Logical row width of an operand tensor (pair tensors are [..., 2, C])."""
    return t.shape[-1]


def lstride(t):
    """Logical row stride of a 2-D (or pair [rows, 2, C]) operand tensor."""
    return t.stride(0) // _ps(t)


def _gemm_args(A, W, C, *, M, N, K, lda, ldw, ldc, bias=None, relu=False, R=None, ldr=0, A2=None, lda2=0,
               a2_cols=0, a_mode=A_ROWS, conv=(0, 0, 0), seg_len=0, batch=1, a_bstride=0, w_bstride=0,
               bias_bstride=0, r_bstride=0, c_bstride=0, headsplit_rows=0, a_offset=0, c_offset=0, r_offset=0,
               a2_offset=0):
    _dev(A, W, C, bias, R, A2)
    g = GemmArgs()
    g.M, g.N, g.K, g.batch = M, N, K, batch
    sa, sw, sr, sc, s2 = _ps(A), _ps(W), _ps(R), _ps(C), _ps(A2)
    g.A = A.data_ptr() + a_offset * sa * A.element_size()
    g.lda, g.a_bstride, g.a_dtype = lda * sa, a_bstride * sa, DT[A.dtype]
    g.A2 = None if A2 is None else A2.data_ptr() + a2_offset * s2 * A2.element_size()
    g.lda2, g.a2_cols = lda2 * s2, a2_cols
    g.a2_mode = A2_ADD if (A2 is None or A.dtype == torch.float32) else A2_SELECT
    g.a_mode = a_mode
    g.conv_h, g.conv_w, g.conv_c = conv
    g.seg_len = seg_len
    g.W, g.ldw, g.w_bstride, g.w_dtype = W.data_ptr(), ldw * sw, w_bstride * sw, DT[W.dtype]
    g.bias = None if bias is None else bias.data_ptr()
    g.bias_bstride = bias_bstride
    g.R = None if R is None else R.data_ptr() + r_offset * sr * R.element_size()
    g.ldr, g.r_bstride = ldr * sr, r_bstride * sr
    g.r_dtype = F32 if R is None else DT[R.dtype]
    g.C = None if C is None else C.data_ptr() + c_offset * sc * C.element_size()
    g.ldc, g.c_bstride, g.c_dtype = ldc * sc, c_bstride * sc, DT[C.dtype] if C is not None else F32
    g.c_mode = C_HEADSPLIT if headsplit_rows else C_ROWS
    g.rows_per_batch = headsplit_rows
    g.relu = int(bool(relu))
    return g


def linear(X, W, bias=None, *, relu=False, R=None, out=None, out_dtype=torch.float32, A2=None, a2_cols=0,
           headsplit_rows=0):
    """Row-major linear layer: X [M, K] (f32 or compute dtype; pair [M, 2, K]),
    W [N, K] (pair [N, 2, K]).  A split W with an fp32 X splits X first."""
    if W.dtype == torch.uint16 and X.dtype == torch.float32:
        X = split_rows(X)
    M, K = X.shape[0], width(X)
    N = W.shape[0]
    if out is None:
        out = torch.empty((M, 2, N) if out_dtype == torch.uint16 else (M, N), device=X.device, dtype=out_dtype)
    gemm(X, W, out, M=M, N=N, K=K, lda=lstride(X), ldw=lstride(W), ldc=N, bias=bias, relu=relu, R=R,
         ldr=(lstride(R) if R is not None else 0), A2=A2, lda2=(lstride(A2) if A2 is not None else 0),
         a2_cols=a2_cols, headsplit_rows=headsplit_rows)
    return out


def split_rows(X, out=None):
    """fp32 rows X [M, C] (any row stride) -> split f16 pair rows [M, 2, C] (cmt_split_rows)."""
    _dev(X, out)
    M, C = X.shape
    if out is None:
        out = torch.empty((M, 2, C), dtype=torch.uint16, device=X.device)
    _check(lib().cmt_split_rows(_p(X), X.stride(0), M, C, _p(out), _stream()), "cmt_split_rows")
    return out


_WS_CACHE = {}


def attention(Q, K, V, O, *, B, H, Nq, Nk, q_strides, k_strides, v_strides, o_strides, scale, q_offset=0,
              k_offset=0, v_offset=0, o_offset=0, kv_splits=0, workspace=None, round_output=False,
              fold_scale=False, kmax2=None, kmax_ld=0, kmax_plane0=0, keep_partials=False, _diag_flags=0):
    """Strides are (batch, head, row) in elements; o_strides = (batch, row).
    f16-pair Q/K/V (torch.uint16, the split self-attention): strides and offsets
    count 16-bit elements, a pair row being 64 of them (32 hi, 32 lo).
    fold_scale lets the kernel fold scale*log2(e) into Q on load (one extra
    rounding of Q; the f16/bf16 policies only).  kmax2: the K projection's
    plane_max2 partials (see gemm) -- lets the bf16 long-key kernel fix each
    query's softmax offset at |q| max|k| instead of tracking a running max.
    keep_partials (ABI 19): a launch with CHAIN_XSPLITS key splits leaves its
    partials in ``workspace`` (which must then be given) for chain B1 and does
    not write O.  Returns the number of partials kept (0: O written)."""
    _dev(Q, K, V, O, kmax2)
    a = AttnArgs()
    a.B, a.H, a.Nq, a.Nk, a.dtype = B, H, Nq, Nk, DT[Q.dtype]
    es = Q.element_size()
    a.Q = Q.data_ptr() + q_offset * es
    a.q_bstride, a.q_hstride, a.q_rstride = q_strides
    a.K = K.data_ptr() + k_offset * es
    a.k_bstride, a.k_hstride, a.k_rstride = k_strides
    a.V = V.data_ptr() + v_offset * es
    a.v_bstride, a.v_hstride, a.v_rstride = v_strides
    so = _ps(O)
    a.O = O.data_ptr() + o_offset * so * O.element_size()
    a.o_bstride, a.o_rstride = o_strides[0] * so, o_strides[1] * so
    a.o_dtype = DT[O.dtype]
    a.scale, a.kv_splits = scale, kv_splits
    a.flags = (1 if round_output else 0) | (2 if fold_scale else 0) | _diag_flags
    if kmax2 is not None:
        a.kmax2, a.kmax_ld, a.kmax_plane0, a.kmax_rows = kmax2.data_ptr(), kmax_ld, kmax_plane0, PLANE_MAX_ROWS
    kept = 0
    if keep_partials and int(lib().cmt_attn_splits(ctypes.byref(a))) == CHAIN_XSPLITS:
        a.flags |= ATTN_KEEP_PARTIALS
        kept = CHAIN_XSPLITS
    need = lib().cmt_attn_workspace_bytes(ctypes.byref(a))
    if need > 0:
        if workspace is None or workspace.numel() < need:
            if keep_partials:
                raise RuntimeError("cmt_attn_fwd: keep_partials needs a caller workspace of "
                                   "cmt_attn_workspace_bytes (the partials' consumer reads it)")
            workspace = torch.empty(need, dtype=torch.uint8, device=O.device)
        a.workspace, a.workspace_bytes = workspace.data_ptr(), workspace.numel()
    _check(lib().cmt_attn_fwd(ctypes.byref(a), _stream()), "cmt_attn_fwd")
    return kept


def attn_workspace_bytes(*, B, H, Nq, Nk, kv_splits=0):
    a = AttnArgs()
    a.B, a.H, a.Nq, a.Nk, a.kv_splits = B, H, Nq, Nk, kv_splits
    return int(lib().cmt_attn_workspace_bytes(ctypes.byref(a)))


def layernorm(X, W, Bv, Y, *, rows, C, ldx, ldy, eps=1e-5, flags=0, W2=None, B2=None, Y2=None, ldy2=0,
              flags2=0, x_offset=0, y_offset=0, y2_offset=0):
    _dev(X, W, Bv, Y, W2, B2, Y2)
    _check(lib().cmt_layernorm(X.data_ptr() + 4 * x_offset, ldx, rows, C, _p(W), _p(Bv), eps,
                               Y.data_ptr() + 4 * y_offset, ldy, flags, _p(W2), _p(B2),
                               None if Y2 is None else Y2.data_ptr() + 4 * y2_offset, ldy2, flags2, _stream()),
           "cmt_layernorm")


def layernorm_ex(X, W, Bv, *, rows, C, ldx, eps=1e-5, Y=None, ldy=0, flags=0, W2=None, B2=None, Y2=None, ldy2=0,
                 flags2=0, Yl=None, Yp=None, P=None, y2_offset=0, nparts=1):
    """LayerNorm with optional second LN (Y2) and compute-dtype copies
    Yl = lowp(y), Yp = lowp(y + P) (rows of width C, contiguous).  nparts >= 2:
    the input is the sum of nparts blocks X + p * rows * ldx (a split-K gemm's C)."""
    a = _ln_args(X, W, Bv, rows=rows, C=C, ldx=ldx, eps=eps, Y=Y, ldy=ldy, flags=flags, W2=W2, B2=B2, Y2=Y2,
                 ldy2=ldy2, flags2=flags2, Yl=Yl, Yp=Yp, P=P, y2_offset=y2_offset)
    if nparts > 1:
        if X.numel() < nparts * rows * ldx:
            raise RuntimeError("layernorm_ex: X holds fewer than nparts blocks of rows * ldx")
        a.nparts, a.part_stride = nparts, rows * ldx
    _check(lib().cmt_layernorm_ex(ctypes.byref(a), _stream()), "cmt_layernorm_ex")


def _ln_args(X, W, Bv, *, rows, C, ldx, eps=1e-5, Y=None, ldy=0, flags=0, W2=None, B2=None, Y2=None, ldy2=0,
             flags2=0, Yl=None, Yp=None, P=None, y2_offset=0):
    _dev(X, W, Bv, Y, W2, B2, Y2, Yl, Yp, P)
    a = LnArgs()
    a.X, a.ldx, a.rows, a.C = _p(X), ldx, rows, C
    a.W, a.B, a.eps = W.data_ptr(), Bv.data_ptr(), eps
    a.Y, a.ldy, a.flags = _p(Y), ldy, flags
    a.W2, a.B2 = _p(W2), _p(B2)
    a.Y2 = None if Y2 is None else Y2.data_ptr() + 4 * y2_offset
    a.ldy2, a.flags2 = ldy2, flags2
    low = Yl if Yl is not None else Yp
    a.lowp_dtype = DT[low.dtype] if low is not None else BF16
    a.Yl, a.ldyl = _p(Yl), C * _ps(Yl)
    a.Yp, a.ldyp, a.P, a.ldp = _p(Yp), C * _ps(Yp), _p(P), C
    return a


def gemm_ln(A, W, *, M, K, lda, ldw, bias=None, R=None, ldr=0, ln_w, ln_b, eps=1e-5, Y=None, flags=0,
            W2=None, B2=None, Y2=None, flags2=0, Yl=None, Yp=None, P=None, y2_offset=0):
    """One launch of  y = LN(A W^T + bias + R)  with cmt_layernorm_ex's
    outputs (N = C = 256, compute-dtype A/W, contiguous [M, 256] rows)."""
    N = W.shape[0]
    g = _gemm_args(A, W, None, M=M, N=N, K=K, lda=lda, ldw=ldw, ldc=0, bias=bias, R=R, ldr=ldr)
    a = _ln_args(None, ln_w, ln_b, rows=M, C=N, ldx=0, eps=eps, Y=Y, ldy=N, flags=flags, W2=W2, B2=B2, Y2=Y2,
                 ldy2=N, flags2=flags2, Yl=Yl, Yp=Yp, P=P, y2_offset=y2_offset)
    _check(lib().cmt_gemm_ln(ctypes.byref(g), ctypes.byref(a), _stream()), "cmt_gemm_ln")


CHAIN_PRM = {0: 1024, 1: 3840, 2: 3840}


def chain_ws_numel(rows):
    """fp32 elements of the chain B1 -> B2 partials workspace (4 partials of
    whole 32-row blocks, in the chains' private tile order)."""
    return 4 * ((rows + 31) // 32) * 32 * 256


def pack_chain_wn(W):
    """Row-major weight [256 G, 256] -> the fragment-major 1-D layout the chains
    stream into registers (cmt_hip.h cmt_chain_args.Wn; chain A's W1 is G = 1):
    index (g, wave, kc, ks, nt, lh, lr, e)."""
    if W.dim() != 2 or W.shape[1] != 256 or W.shape[0] % 256:
        raise RuntimeError("pack_chain_wn: weight must be [256 G, 256]")
    G = W.shape[0] // 256
    return W.reshape(G, 4, 2, 32, 8, 2, 2, 8).permute(0, 1, 4, 5, 2, 6, 3, 7).contiguous().view(-1)


def pack_chain_fc2(W2):
    """fc2.weight [256, 1024] -> its four K blocks [256, 256] stacked and packed
    fragment-major (cmt_hip.h cmt_chain_args.W2)."""
    if W2.shape != (256, 1024):
        raise RuntimeError("pack_chain_fc2: fc2.weight must be [256, 1024]")
    return pack_chain_wn(torch.cat([W2[:, 256 * g:256 * (g + 1)] for g in range(4)], 0))


def pack_chain_pair(Wp):
    """Split-f16 weight (uint16 [256 G, 2, 256], the CMT_F16P rows to_dtype
    writes) -> the split chains' fragment-major pair pack: pack_chain_wn of the
    hi halves, then of the lo halves (cmt_hip.h cmt_chain_args, dtype CMT_F16P)."""
    if Wp.dtype != torch.uint16 or Wp.dim() != 3 or Wp.shape[1] != 2:
        raise RuntimeError("pack_chain_pair: weight must be split-f16 rows [R, 2, C]")
    h = Wp.view(torch.float16)
    return torch.cat([pack_chain_wn(h[:, 0].contiguous()), pack_chain_wn(h[:, 1].contiguous())]).view(torch.uint16)


def pack_chain_fc2_pair(W2p):
    """Split-f16 fc2.weight [256, 2, 1024] -> its four K blocks packed as
    pack_chain_fc2 does, hi halves then lo halves."""
    if W2p.dtype != torch.uint16 or tuple(W2p.shape) != (256, 2, 1024):
        raise RuntimeError("pack_chain_fc2_pair: fc2.weight must be split-f16 [256, 2, 1024]")
    h = W2p.view(torch.float16)
    return torch.cat([pack_chain_fc2(h[:, 0].contiguous()), pack_chain_fc2(h[:, 1].contiguous())]).view(torch.uint16)


def chain(kind, X, P, prm, Wo, W1, Y, *, rows, Nq, eps, R=None, W2=None, Wn=None, OUT=None, out_offset=0,
          out_flags=0, Q=None, WS=None, OUT16=None, xpart=None, xsplits=0, xround=False):
    """One row-block chain of a decoder layer's query side (cmt_chain): kind 0
    after self-attention; kinds 1 then 2 after cross-attention (cmt_hip.h).
    Split-f16 operands (torch.uint16: the 'ref' policy) select the split chains:
    X / OUT16 pair rows, every weight a fragment-major pair pack
    (pack_chain_pair / pack_chain_fc2_pair; chain B1's W1 is fc1's), chain A's
    Q f16 head-split, chain B2's Q head-split pairs.  xpart (ABI 19, split chain
    B1): the cross-attention workspace a keep_partials attention() left its
    ``xsplits`` partials in, combined inside the chain (X is then not read)."""
    _dev(X, P, prm, Wo, W1, Y, R, W2, Wn, OUT, Q, WS, OUT16, xpart)
    split = any(t is not None and t.dtype == torch.uint16 for t in (X, Wo, W1, W2, Wn, Q, OUT16))
    pw = 2 if split else 1   # a pair pack holds the hi pack, then the lo pack
    if Wn is not None and (Wn.dim() != 1 or Wn.numel() != pw * 768 * 256):
        raise RuntimeError("cmt_chain: Wn must be fragment-major (pack_chain_wn / pack_chain_pair)")
    if kind == 1 and (W2 is None or W2.dim() != 1 or W2.numel() != pw * 256 * 1024):
        raise RuntimeError("cmt_chain: chain B1's W2 must be fragment-major (pack_chain_fc2 / pack_chain_fc2_pair)")
    if kind == 0 and (W1 is None or W1.dim() != 1 or W1.numel() != pw * 256 * 256):
        raise RuntimeError("cmt_chain: chain A's W1 must be fragment-major (pack_chain_wn / pack_chain_pair)")
    # chain A's Wo: row-major [256, 256] (LDS weight ring) or fragment-major 1-D (pack_chain_wn: registers)
    wo_frag = int(kind == 0 and Wo is not None and Wo.dim() == 1)
    if wo_frag and Wo.numel() != pw * 256 * 256:
        raise RuntimeError("cmt_chain: a fragment-major Wo must be pack_chain_wn / pack_chain_pair of [256, 256]")
    if prm.dtype != torch.float32 or prm.numel() != CHAIN_PRM[kind]:
        raise RuntimeError(f"cmt_chain: parameter block must be {CHAIN_PRM[kind]} fp32 values")
    if WS is not None and (WS.dtype != torch.float32 or WS.numel() < chain_ws_numel(rows)):
        raise RuntimeError("cmt_chain: WS must hold chain_ws_numel(rows) fp32")
    a = ChainArgs()
    a.kind, a.rows, a.Nq, a.eps = kind, rows, Nq, eps
    if split:
        if kind != 2 and xpart is None and (X is None or X.dtype != torch.uint16):
            raise RuntimeError("cmt_chain: the split chains take pair-row X")
        if any(t is not None and (t.dtype != torch.uint16 or t.dim() != 1) for t in (Wo, W1, W2, Wn)):
            raise RuntimeError("cmt_chain: the split chains take fragment-major pair weights")
        if kind == 1 and (W1.numel() != 2 * 1024 * 256 or Wo.numel() != 2 * 256 * 256):
            raise RuntimeError("cmt_chain: split chain B1 takes fragment-major pair packs of Wo and fc1")
        if kind == 0 and not wo_frag:
            raise RuntimeError("cmt_chain: split chain A takes a fragment-major pair pack of Wo")
        if Q is not None and Q.dtype != (torch.float16 if kind == 0 else torch.uint16):
            raise RuntimeError("cmt_chain: split chain A writes an f16 Q, chain B2 head-split pairs")
        if OUT16 is not None and (OUT is None or OUT16.dtype != torch.uint16):
            raise RuntimeError("cmt_chain: split OUT16 is the pair copy of OUT")
        a.dtype = F16P
    else:
        if OUT16 is not None and (OUT is None or OUT16.dtype not in (torch.float16, torch.bfloat16)):
            raise RuntimeError("cmt_chain: OUT16 must be a 16-bit copy target beside OUT")
        lows = [t for t in (X, Wo, W1, W2, Wn, Q, OUT16) if t is not None]
        if any(t.dtype != lows[0].dtype for t in lows) or (lows and lows[0].dtype not in (torch.float16,
                                                                                          torch.bfloat16)):
            raise RuntimeError("cmt_chain: X, Wo, W1, W2, Wn, Q and OUT16 must share one 16-bit dtype (f16 or bf16)")
        a.dtype = DT[lows[0].dtype] if lows else BF16   # B2 without in_proj: no 16-bit operand

    def ptr(t):
        return None if t is None else t.data_ptr()
    a.X, a.R, a.P, a.prm = ptr(X), ptr(R), ptr(P), ptr(prm)
    a.Wo, a.W1, a.W2, a.Wn = ptr(Wo), ptr(W1), ptr(W2), ptr(Wn)
    a.Y = ptr(Y)
    a.OUT = None if OUT is None else OUT.data_ptr() + 4 * out_offset
    a.out_flags = out_flags
    a.Q = ptr(Q)
    a.WS = ptr(WS)
    # OUT16 holds the layer outputs like OUT: 2 bytes per element, 4 for a pair (hi and lo)
    a.OUT16 = None if OUT16 is None else OUT16.data_ptr() + (4 if split else 2) * out_offset
    a.wo_frag = wo_frag
    if xpart is not None:
        if kind != 1 or not split:
            raise RuntimeError("cmt_chain: xpart feeds the split chain B1 only")
        a.xpart, a.xsplits, a.xround = xpart.data_ptr(), xsplits, int(bool(xround))
    _check(lib().cmt_chain(ctypes.byref(a), _stream()), "cmt_chain")


def add_cast(X, *, rows, C, Yl=None, Yp=None, P=None):
    """Yl = lowp(X), Yp = lowp(X + P); X None = zeros."""
    _dev(X, Yl, Yp, P)
    low = Yl if Yl is not None else Yp
    _check(lib().cmt_add_cast(_p(X), _p(P), rows, C, DT[low.dtype], _p(Yl), _p(Yp), _stream()),
           "cmt_add_cast")


def pos2embed(pos, out, *, n, F, mode=0, pos_stride=2, grid=(0, 0), ldo=None):
    _dev(pos, out)
    _check(lib().cmt_pos2embed(_p(pos), pos_stride, n, F, mode, grid[0], grid[1], _p(out), DT[out.dtype],
                               (ldo if ldo is not None else 2 * F) * _ps(out), _stream()), "cmt_pos2embed")


def rv_pe_coords(i2l, out, *, BV, h, w, D, pad_h, pad_w, depth_max, pc_range):
    _dev(i2l, out)
    _check(lib().cmt_rv_pe_coords(BV, h, w, D, pad_h, pad_w, depth_max, _p(i2l), _farr(pc_range, 6), _p(out),
                                  DT[out.dtype], _stream()), "cmt_rv_pe_coords")


def rv_query_coords(ref, l2i, i2l, out, mask, *, B, V, Nq, D, pad_h, pad_w, pc_range):
    _dev(ref, l2i, i2l, out, mask)
    _check(lib().cmt_rv_query_coords(_p(ref), B, V, Nq, D, pad_h, pad_w, _p(l2i), _p(i2l), _farr(pc_range, 6),
                                     _p(out), _p(mask), _stream()), "cmt_rv_query_coords")


def masked_view_sum(X, mask, Y, *, B, V, Nq, C, base=None, Yl=None, Yp=None):
    """Y += sum_v X * mask; with ``base`` [Nq, C]: Y = base + sum; Yp / Yl (f16/bf16):
    lowp(Y) and lowp(0) -- the decoder's first operands."""
    _dev(X, mask, Y, base, Yl, Yp)
    if base is None and Yl is None and Yp is None:
        _check(lib().cmt_masked_view_sum(_p(X), _p(mask), B, V, Nq, C, _p(Y), _stream()), "cmt_masked_view_sum")
        return
    low = Yp if Yp is not None else Yl
    _check(lib().cmt_masked_view_sum_ex(_p(X), _p(mask), B, V, Nq, C, _p(base), _p(Y), _p(Yl), _p(Yp),
                                        DT[low.dtype] if low is not None else 0, _stream()),
           "cmt_masked_view_sum_ex")


def rv_query_coords_lowp(ref, l2i, i2l, out, mask, *, B, V, Nq, D, pad_h, pad_w, pc_range):
    """cmt_rv_query_coords with the coordinates written in out's dtype (RNE)."""
    _dev(ref, l2i, i2l, out, mask)
    _check(lib().cmt_rv_query_coords_ex(_p(ref), B, V, Nq, D, pad_h, pad_w, _p(l2i), _p(i2l), _farr(pc_range, 6),
                                        _p(out), DT[out.dtype], _p(mask), _stream()), "cmt_rv_query_coords_ex")


def nchw_to_rows(X, Y, *, nb, nv, C, HW, ldy, rows_per_batch, row_offset=0, range_flag=None):
    """NCHW fp32 -> rows of Y's dtype; range_flag: int32 device word set to 1 when an f16 /
    f16-pair output meets a value outside that format (cmt_nchw_to_rows_ex)."""
    _dev(X, Y, range_flag)
    if range_flag is not None and range_flag.dtype != torch.int32:
        raise RuntimeError("nchw_to_rows: range_flag must be an int32 device word")
    _check(lib().cmt_nchw_to_rows_ex(_p(X), nb, nv, C, HW, _p(Y), DT[Y.dtype], ldy * _ps(Y), rows_per_batch,
                                     row_offset, _p(range_flag) if range_flag is not None else None, _stream()),
           "cmt_nchw_to_rows")


def cast(X, Y):
    _dev(X, Y)
    _check(lib().cmt_cast(_p(X), DT[X.dtype], _p(Y), DT[Y.dtype], X.numel(), _stream()), "cmt_cast")


def task_head_tail(H1, gw, gb, W2, B2, ref, out, *, L, B, Nq, nheads, hc, head_out, k, center_col, height_col,
                   pc_range):
    _dev(H1, gw, gb, W2, B2, ref, out)
    ho = (ctypes.c_int * len(head_out))(*head_out)
    _check(lib().cmt_task_head_tail(_p(H1), L, B, Nq, nheads, hc, _p(gw), _p(gb), _p(W2), _p(B2), ho,
                                    int(sum(head_out)), k, _p(ref), center_col, height_col, _farr(pc_range, 6),
                                    _p(out), _stream()), "cmt_task_head_tail")


def box_decode(logits, bbox, class_task, *, Nq, ncls, max_num, post_center_range, score_threshold=None):
    """logits [B, Nq*ncls] f32, bbox [B, T*Nq, code] f32, class_task [ncls] int32 (device) ->
    (boxes [B, max_num, code-1], scores [B, max_num], labels [B, max_num] int32, count [B] int32),
    rows [:count[b]] valid, in descending score order."""
    _dev(logits, bbox, class_task)
    B = logits.shape[0]
    code = bbox.shape[-1]
    dev = logits.device
    boxes = torch.empty((B, max_num, code - 1), dtype=torch.float32, device=dev)
    scores = torch.empty((B, max_num), dtype=torch.float32, device=dev)
    labels = torch.empty((B, max_num), dtype=torch.int32, device=dev)
    count = torch.empty((B,), dtype=torch.int32, device=dev)
    thr = 0.0 if score_threshold is None else float(score_threshold)
    _check(lib().cmt_box_decode(_p(logits), logits.stride(0), _p(bbox), bbox.stride(0), _p(class_task), B, Nq, ncls,
                                code, max_num, _farr(post_center_range, 6), thr, int(bool(score_threshold)),
                                _p(boxes), _p(scores), _p(labels), _p(count), _stream()), "cmt_box_decode")
    return boxes, scores, labels, count


def voxelize_workspace(n_points, device, max_voxels=1):
    """A clean voxelizer workspace for up to ``n_points`` points (cmt_hip.h:
    cmt_voxelize_workspace_init); calls leave it clean, so it is reused."""
    wsb = int(lib().cmt_voxelize_workspace_bytes(int(n_points), int(max_voxels)))
    ws = torch.empty((wsb,), dtype=torch.uint8, device=device)
    _check(lib().cmt_voxelize_workspace_init(_p(ws), wsb, _stream()), "cmt_voxelize_workspace_init")
    return ws


def voxelize(points, *, voxel_size, coors_range, grid, max_points, max_voxels, nfeat_mean, workspace=None):
    """points [N, F] f32 on device -> (voxels, coors, num_points, means, num_voxels_dev) sized max_voxels.
    Three launches, no host sync (graph-capturable).  ``workspace``: from
    voxelize_workspace (capacity >= N); a fresh one is made when None."""
    _dev(points)
    points = points.contiguous()
    N, F = points.shape
    dev = points.device
    voxels = torch.empty((max_voxels, max_points, F), dtype=torch.float32, device=dev)
    coors = torch.empty((max_voxels, 3), dtype=torch.int32, device=dev)
    num = torch.empty((max_voxels,), dtype=torch.int32, device=dev)
    means = torch.empty((max_voxels, nfeat_mean), dtype=torch.float32, device=dev)
    nvox = torch.empty((1,), dtype=torch.int32, device=dev)
    ws = workspace if workspace is not None else voxelize_workspace(N, dev, max_voxels)
    _dev(ws)
    g = (ctypes.c_int * 3)(*[int(x) for x in grid])
    _check(lib().cmt_voxelize(_p(points), N, F, _farr(voxel_size, 3), _farr(coors_range, 6), g, max_points,
                              max_voxels, nfeat_mean, _p(voxels), _p(coors), _p(num), _p(means), _p(nvox), _p(ws),
                              ws.numel(), _stream()), "cmt_voxelize")
    return voxels, coors, num, means, nvox
