"""ctypes wrappers of the training-path kernels (include/cmt_hip.h "TRAINING
PATH": train.hip, attn_train.hip).  Same contract as native.py: device
tensors only, the current torch stream, no CPU or eager-PyTorch fallback."""
import ctypes
import threading

import torch

from . import native as N

__all__ = ["gemm_ex", "set_train_gemm", "linear_fwd", "linear_bwd", "attn_train_fwd", "attn_train_bwd", "ln_train_fwd", "ln_train_bwd",
           "bn_relu_train_fwd", "bn_relu_train_bwd", "im2col3x3", "conv3x3_wgrad", "det_loss", "match_cost", "sumsq", "adamw_step"]


def _ptr(t):
    return None if t is None else t.data_ptr()


def _f32(*ts):
    N._dev(*ts)
    for t in ts:
        if t is not None and t.dtype != torch.float32:
            raise RuntimeError("training kernels take fp32 tensors")


# Arithmetic of the training step's GEMMs: "bf16x3" (cmt_gemm_bf16x3_ex, three bf16 MFMA
# passes on split operands, ~2^-16 relative per product) or "f32" (cmt_gemm_f32_ex, the
# exact-f32 MFMA at 1/16 of the bf16 rate).  The reference's fp32 GEMMs ran as TF32
# (~2^-11) under torch 1.9.1's defaults on its Ampere GPUs.
_GEMM_ENTRY = {"bf16x3": "cmt_gemm_bf16x3_ex", "f32": "cmt_gemm_f32_ex"}
_gemm_mode = "bf16x3"


def set_train_gemm(mode):
    """Select the training GEMM arithmetic ("bf16x3" or "f32"); returns the previous mode."""
    global _gemm_mode
    if mode not in _GEMM_ENTRY:
        raise ValueError(f"train gemm mode must be one of {sorted(_GEMM_ENTRY)}")
    old, _gemm_mode = _gemm_mode, mode
    return old


_tls = threading.local()


def gemm_ex(A, a_strides, B, b_strides, C, *, M, N_, K, ldc, alpha=1.0, beta=0.0, bias=None, batch=1, a_bs=0,
            b_bs=0, c_bs=0, ksplit=1, a_offset=0, b_offset=0, c_offset=0, mode=None, bias_bs=0, a_rowsum=None):
    """C[z][m][n] = alpha sum_k A(m,k) B(n,k) (+bias) + beta C; strides in elements:
    a_strides = (s_m, s_k), b_strides = (s_n, s_k).  ``mode``: see set_train_gemm."""
    _f32(A, B, C, bias)
    # one argument struct per thread (the library copies it at the call; autograd runs the
    # backward on its own thread): no ctypes allocation per launch
    g = getattr(_tls, "gemm_args", None)
    if g is None:
        g = _tls.gemm_args = N.GemmExArgs()
    g.a_rowsum = None
    g.M, g.N, g.K, g.batch, g.alpha, g.beta = M, N_, K, batch, alpha, beta
    g.A, (g.a_sm, g.a_sk), g.a_bs = A.data_ptr() + 4 * a_offset, a_strides, a_bs
    g.B, (g.b_sn, g.b_sk), g.b_bs = B.data_ptr() + 4 * b_offset, b_strides, b_bs
    g.C, g.ldc, g.c_bs = C.data_ptr() + 4 * c_offset, ldc, c_bs
    g.bias, g.ksplit, g.bias_bs = _ptr(bias), ksplit, bias_bs
    entry = _GEMM_ENTRY[mode or _gemm_mode]
    if a_rowsum is not None:
        if entry != "cmt_gemm_bf16x3_ex":
            raise ValueError("a_rowsum: bf16x3 GEMM only")
        g.a_rowsum = a_rowsum.data_ptr()
    N._check(getattr(N.lib(), entry)(ctypes.byref(g), N._stream()), entry)


def _ksplit(k, m, n):
    """split the reduction when the output tile grid alone cannot fill the chip"""
    tiles = -(-m // 64) * -(-n // 64)
    s = 1
    while tiles * s < 512 and k // (2 * s) >= 256:
        s *= 2
    return s


def linear_fwd(X, W, b=None):
    """Y = X W^T + b, X [M, K] (row stride X.stride(0)), W [N, K] contiguous."""
    M, K = X.shape
    Nn = W.shape[0]
    Y = torch.empty((M, Nn), dtype=torch.float32, device=X.device)
    gemm_ex(X, (X.stride(0), 1), W, (W.stride(0), 1), Y, M=M, N_=Nn, K=K, ldc=Nn, bias=b)
    return Y


def linear_bwd(dY, X, W, need_dx=True, need_dw=True, need_db=True, dw_into=None, db_into=None):
    """(dX, dW, dB) of Y = X W^T + b.  dw_into / db_into (a parameter's .grad, or a view of it):
    the weight / bias gradient is ADDED there (ABI 24: no zero fill, no temporary) and returned
    as None."""
    M, K = X.shape
    Nn = W.shape[0]
    dY = dY.contiguous()
    dX = dW = dB = None
    if dw_into is not None or db_into is not None:
        if not need_dw or dw_into is None or (need_db and db_into is None):
            raise ValueError("linear_bwd: accumulate the weight gradient, and the bias one with it")
        _f32(dY, X, W, dw_into, db_into)
        if X.stride(1) != 1 or not W.is_contiguous() or not dw_into.is_contiguous() or \
                dw_into.shape != W.shape or (db_into is not None and not db_into.is_contiguous()):
            raise RuntimeError("linear_bwd: contiguous X rows, W and gradient targets of W's shape")
        if need_dx:
            dX = torch.empty((M, K), dtype=torch.float32, device=X.device)
        if _gemm_mode == "bf16x3":
            N._check(N.lib().cmt_linear_bwd_bf16x3_ex(dY.data_ptr(), X.data_ptr(), W.data_ptr(), _ptr(dX),
                                                       dw_into.data_ptr(), _ptr(db_into if need_db else None), M, K,
                                                       Nn, X.stride(0), _ksplit(M, Nn, K),
                                                       N.LINEAR_BWD_ACCUMULATE, N._stream()),
                     "cmt_linear_bwd_bf16x3_ex")
        else:
            if need_dx:
                gemm_ex(dY, (Nn, 1), W, (1, W.stride(0)), dX, M=M, N_=K, K=Nn, ldc=K)
            gemm_ex(dY, (1, Nn), X, (1, X.stride(0)), dw_into, M=Nn, N_=K, K=M, ldc=K, beta=1.0,
                    ksplit=_ksplit(M, Nn, K))
            if need_db:
                db_into.add_(dY.sum(0))
        return dX, None, None
    if _gemm_mode == "bf16x3" and (need_dx or need_dw):
        # one native call: both GEMMs, the split-K / bias-gradient zeroing on the stream (ABI 23)
        _f32(dY, X, W)
        if X.stride(1) != 1 or not W.is_contiguous():
            raise RuntimeError("linear_bwd: X rows and W must be contiguous")
        dev = X.device
        if need_dx:
            dX = torch.empty((M, K), dtype=torch.float32, device=dev)
        if need_dw:
            dW = torch.empty((Nn, K), dtype=torch.float32, device=dev)
            if need_db:
                dB = torch.empty((Nn,), dtype=torch.float32, device=dev)
        N._check(N.lib().cmt_linear_bwd_bf16x3(dY.data_ptr(), X.data_ptr(), W.data_ptr(), _ptr(dX), _ptr(dW),
                                                _ptr(dB), M, K, Nn, X.stride(0),
                                                _ksplit(M, Nn, K) if need_dw else 1, N._stream()),
                 "cmt_linear_bwd_bf16x3")
        if need_db and dB is None:
            dB = dY.sum(0)
        return dX, dW, dB
    if need_dx:
        dX = torch.empty((M, K), dtype=torch.float32, device=X.device)
        gemm_ex(dY, (Nn, 1), W, (1, W.stride(0)), dX, M=M, N_=K, K=Nn, ldc=K)
    if need_dw:
        ks = _ksplit(M, Nn, K)
        # the bias gradient (column sums of dY = row sums of the GEMM's A = dY^T) comes out of the
        # weight-gradient GEMM itself (a_rowsum); split-K dW and dB share one zero fill
        fuse_db = need_db and _gemm_mode == "bf16x3"
        nz, nb = (Nn * K if ks > 1 else 0), (Nn if fuse_db else 0)
        buf = torch.zeros((nz + nb,), dtype=torch.float32, device=X.device) if nz + nb else None
        dW = buf[:nz].view(Nn, K) if ks > 1 else torch.empty((Nn, K), dtype=torch.float32, device=X.device)
        if fuse_db:
            dB = buf[nz:]
        gemm_ex(dY, (1, Nn), X, (1, X.stride(0)), dW, M=Nn, N_=K, K=M, ldc=K, beta=1.0 if ks > 1 else 0.0, ksplit=ks,
                a_rowsum=dB)
    if need_db and dB is None:
        dB = dY.sum(0)
    return dX, dW, dB


def linear_fwd_batched(X, W, b=None):
    """Y[l] = X[l] W[l]^T + b[l] for every l in one launch: X [L, M, K], W [L, N, K], b [L, N]
    (all contiguous) -> Y [L, M, N]."""
    L, M, K = X.shape
    Nn = W.shape[1]
    Y = torch.empty((L, M, Nn), dtype=torch.float32, device=X.device)
    gemm_ex(X, (K, 1), W, (K, 1), Y, M=M, N_=Nn, K=K, ldc=Nn, bias=b, batch=L, a_bs=M * K, b_bs=Nn * K,
            c_bs=M * Nn, bias_bs=Nn)
    return Y


def linear_bwd_batched(dY, X, W, need_dx=True, need_dw=True, need_db=True):
    """(dX, dW, dB) of linear_fwd_batched, one launch each."""
    L, M, K = X.shape
    Nn = W.shape[1]
    dY = dY.contiguous()
    dX = dW = dB = None
    if need_dx:
        dX = torch.empty((L, M, K), dtype=torch.float32, device=X.device)
        gemm_ex(dY, (Nn, 1), W, (1, K), dX, M=M, N_=K, K=Nn, ldc=K, batch=L, a_bs=M * Nn, b_bs=Nn * K, c_bs=M * K)
    if need_dw:
        dW = torch.empty((L, Nn, K), dtype=torch.float32, device=X.device)
        if need_db and _gemm_mode == "bf16x3":
            dB = torch.zeros((L, Nn), dtype=torch.float32, device=X.device)
        gemm_ex(dY, (1, Nn), X, (1, K), dW, M=Nn, N_=K, K=M, ldc=K, batch=L, a_bs=M * Nn, b_bs=M * K, c_bs=Nn * K,
                a_rowsum=dB)
    if need_db and dB is None:
        dB = dY.sum(1)
    return dX, dW, dB


def _attn_args(Q, K, V, O, LSE, *, B, H, Nq, Nk, q_strides, k_strides, v_strides, o_strides, scale, dn_pad=0,
               dn_group=0, fp16_inputs=False, dropout_p=0.0, seed=0, seed_dev=None):
    """seed_dev: optional int32 device tensor [1]; the kernels' dropout seed is seed + seed_dev[0]"""
    a = N.AttnTrainArgs()
    a.B, a.H, a.Nq, a.Nk = B, H, Nq, Nk
    a.Q, (a.q_bs, a.q_hs, a.q_rs) = Q.data_ptr(), q_strides
    a.K, (a.k_bs, a.k_hs, a.k_rs) = K.data_ptr(), k_strides
    a.V, (a.v_bs, a.v_hs, a.v_rs) = V.data_ptr(), v_strides
    a.O, (a.o_bs, a.o_hs, a.o_rs) = O.data_ptr(), o_strides
    a.LSE = LSE.data_ptr()
    a.scale, a.dn_pad, a.dn_group = scale, dn_pad, dn_group
    a.fp16_inputs, a.dropout_p, a.seed = int(bool(fp16_inputs)), dropout_p, seed & 0xFFFFFFFF
    if seed_dev is not None:
        if seed_dev.dtype != torch.int32 or not seed_dev.is_cuda:
            raise RuntimeError("seed_dev must be an int32 device tensor")
        a.seed_dev = seed_dev.data_ptr()
    return a


def attn_train_fwd(Q, K, V, O, LSE, **kw):
    """Returns the workspace (or None): handed to attn_train_bwd(ws=...) for the same Q / K / V,
    the backward reuses the forward's f16 copies of them (ABI 25 ws_reuse)."""
    _f32(Q, K, V, O, LSE)
    a = _attn_args(Q, K, V, O, LSE, **kw)
    need = N.lib().cmt_attn_train_workspace_bytes(ctypes.byref(a))
    ws = None
    if need > 0:
        ws = torch.empty(need, dtype=torch.uint8, device=O.device)
        a.workspace, a.workspace_bytes = ws.data_ptr(), need
    N._check(N.lib().cmt_attn_train_fwd(ctypes.byref(a), N._stream()), "cmt_attn_train_fwd")
    return ws


def attn_train_bwd(Q, K, V, O, LSE, dO, dQ, dK, dV, ws=None, **kw):
    """ws: the workspace attn_train_fwd returned for these Q / K / V (unchanged since), or None"""
    _f32(Q, K, V, O, LSE, dO, dQ, dK, dV)
    a = _attn_args(Q, K, V, O, LSE, **kw)
    delta = torch.empty(kw["B"] * kw["H"] * kw["Nq"], dtype=torch.float32, device=O.device)
    a.dO, a.dQ, a.dK, a.dV, a.delta = dO.data_ptr(), dQ.data_ptr(), dK.data_ptr(), dV.data_ptr(), delta.data_ptr()
    # the long-key fp16 path takes f16 copies of Q, dO, K, V in the workspace (cmt_hip.h)
    need = N.lib().cmt_attn_train_workspace_bytes(ctypes.byref(a))
    if need > 0:
        if ws is not None and ws.numel() >= need:
            a.ws_reuse = 1
        else:
            ws = torch.empty(need, dtype=torch.uint8, device=O.device)
        a.workspace, a.workspace_bytes = ws.data_ptr(), need
    N._check(N.lib().cmt_attn_train_bwd(ctypes.byref(a), N._stream()), "cmt_attn_train_bwd")


def _ln_args(X, W, Bv, *, C, eps, rows_per_wset=0):
    a = N.LnTrainArgs()
    a.rows, a.C = X.shape[0], C
    a.X, a.ldx = X.data_ptr(), X.stride(0)
    a.W, a.B, a.eps, a.rows_per_wset = W.data_ptr(), Bv.data_ptr(), eps, rows_per_wset
    return a


def ln_train_fwd(X, W, Bv, *, eps, rows_per_wset=0):
    """y, mean, rstd of a row LayerNorm over the last dim (C = 64 / 256)."""
    _f32(X, W, Bv)
    rows, C = X.shape
    Y = torch.empty((rows, C), dtype=torch.float32, device=X.device)
    mean = torch.empty(rows, dtype=torch.float32, device=X.device)
    rstd = torch.empty_like(mean)
    a = _ln_args(X, W, Bv, C=C, eps=eps, rows_per_wset=rows_per_wset)
    a.Y, a.ldy, a.mean, a.rstd = Y.data_ptr(), C, mean.data_ptr(), rstd.data_ptr()
    N._check(N.lib().cmt_ln_train_fwd(ctypes.byref(a), N._stream()), "cmt_ln_train_fwd")
    return Y, mean, rstd


def ln_train_bwd(dY, X, W, mean, rstd, *, eps, rows_per_wset=0, wsets=1, dw_into=None, db_into=None):
    """(dX, dW, dB); dw_into / db_into (both or neither: the parameters' .grad): the weight and
    bias gradients are added there (the kernel's per-column sums are atomic adds) and returned
    as None."""
    _f32(dY, X, W, mean, rstd)
    rows, C = X.shape
    dY = dY.contiguous()
    dX = torch.empty((rows, C), dtype=torch.float32, device=X.device)
    if dw_into is not None or db_into is not None:
        _f32(dw_into, db_into)
        if dw_into is None or db_into is None or dw_into.numel() != wsets * C or db_into.numel() != wsets * C or \
                not (dw_into.is_contiguous() and db_into.is_contiguous()):
            raise ValueError("ln_train_bwd: contiguous weight and bias gradient targets")
        a = _ln_args(X, W, W, C=C, eps=eps, rows_per_wset=rows_per_wset)
        a.ldy, a.mean, a.rstd = C, mean.data_ptr(), rstd.data_ptr()
        a.dY, a.dX, a.lddx, a.accumulate = dY.data_ptr(), dX.data_ptr(), C, 0
        a.dW, a.dB = dw_into.data_ptr(), db_into.data_ptr()
        N._check(N.lib().cmt_ln_train_bwd(ctypes.byref(a), N._stream()), "cmt_ln_train_bwd")
        return dX, None, None
    dWB = torch.zeros((2, wsets, C), dtype=torch.float32, device=X.device)   # one fill for both sums
    dW, dB = dWB[0], dWB[1]
    a = _ln_args(X, W, W, C=C, eps=eps, rows_per_wset=rows_per_wset)
    a.ldy, a.mean, a.rstd = C, mean.data_ptr(), rstd.data_ptr()
    a.dY, a.dX, a.lddx, a.accumulate, a.dW, a.dB = dY.data_ptr(), dX.data_ptr(), C, 0, dW.data_ptr(), dB.data_ptr()
    N._check(N.lib().cmt_ln_train_bwd(ctypes.byref(a), N._stream()), "cmt_ln_train_bwd")
    return dX, dW.view(-1), dB.view(-1)


def _bn_args(X, W, Bv, mean_save, rstd_save, ws, eps=1e-5, momentum=0.1):
    a = N.BnArgs()
    a.rows, a.C = X.shape
    a.X, a.W, a.B, a.eps, a.momentum = X.data_ptr(), W.data_ptr(), Bv.data_ptr(), eps, momentum
    a.mean_save, a.rstd_save, a.workspace = mean_save.data_ptr(), rstd_save.data_ptr(), ws.data_ptr()
    return a


def bn_relu_train_fwd(X, W, Bv, running_mean=None, running_var=None, *, eps=1e-5, momentum=0.1):
    """relu(BatchNorm2d-train(X)) over rows [B*H*W, C]; returns (Y, mean, rstd)."""
    _f32(X, W, Bv, running_mean, running_var)
    rows, C = X.shape
    Y = torch.empty_like(X)
    mean = torch.empty(C, dtype=torch.float32, device=X.device)
    rstd = torch.empty_like(mean)
    ws = torch.empty(int(N.lib().cmt_bn_workspace_bytes(C)), dtype=torch.uint8, device=X.device)
    a = _bn_args(X, W, Bv, mean, rstd, ws, eps, momentum)
    a.Y = Y.data_ptr()
    a.running_mean, a.running_var = _ptr(running_mean), _ptr(running_var)
    N._check(N.lib().cmt_bn_relu_train_fwd(ctypes.byref(a), N._stream()), "cmt_bn_relu_train_fwd")
    return Y, mean, rstd


def bn_relu_train_bwd(dY, X, Y, W, mean, rstd):
    _f32(dY, X, Y, W, mean, rstd)
    C = X.shape[1]
    dX = torch.empty_like(X)
    dW = torch.empty(C, dtype=torch.float32, device=X.device)
    dB = torch.empty_like(dW)
    ws = torch.empty(int(N.lib().cmt_bn_workspace_bytes(C)), dtype=torch.uint8, device=X.device)
    a = _bn_args(X, W, W, mean, rstd, ws)
    a.Y, a.dY, a.dX, a.dW, a.dB = Y.data_ptr(), dY.contiguous().data_ptr(), dX.data_ptr(), dW.data_ptr(), dB.data_ptr()
    N._check(N.lib().cmt_bn_relu_train_bwd(ctypes.byref(a), N._stream()), "cmt_bn_relu_train_bwd")
    return dX, dW, dB


def im2col3x3(X, nimg, H, W, C):
    _f32(X)
    out = torch.empty((nimg * H * W, 9 * C), dtype=torch.float32, device=X.device)
    N._check(N.lib().cmt_im2col3x3(X.data_ptr(), nimg, H, W, C, out.data_ptr(), N._stream()), "cmt_im2col3x3")
    return out


def conv3x3_wgrad(X, dY, nimg, H, W, Cin, ksplit):
    """dW [Cout, 9 Cin] (tap-major) of the 3x3 / pad 1 conv on NHWC rows X [nimg*H*W, Cin] given
    dY [nimg*H*W, Cout]: the bf16x3 GEMM with the im2col operand gathered in the kernel."""
    _f32(X, dY)
    X, dY = X.contiguous(), dY.contiguous()
    Cout = dY.shape[1]
    dW = (torch.zeros if ksplit > 1 else torch.empty)((Cout, 9 * Cin), dtype=torch.float32, device=X.device)
    N._check(N.lib().cmt_conv3x3_wgrad_bf16x3(X.data_ptr(), dY.data_ptr(), dW.data_ptr(), nimg, H, W, Cin, Cout,
                                              ksplit, N._stream()), "cmt_conv3x3_wgrad_bf16x3")
    return dW


def det_loss(logits, labels, label_w, boxes, targets, box_w, *, gamma, alpha, cls_weight, box_weight, cls_avg,
             box_avg, need_grad=True, out=None):
    """(loss [2] device tensor, dlogits, dboxes) of FocalLoss + L1Loss; out: a caller's [2] slot."""
    _f32(logits, boxes, targets, box_w, label_w)
    N._dev(labels)
    if out is None:
        out = torch.empty(2, dtype=torch.float32, device=logits.device)
    elif out.dtype != torch.float32 or out.numel() != 2 or not out.is_contiguous():
        raise RuntimeError("det_loss: out must be a contiguous fp32 [2] tensor")
    # the kernel writes every gradient element (rows x ncls, rows x 10): no fill for dense operands
    dl = (torch.empty_like if logits.is_contiguous() else torch.zeros_like)(logits) if need_grad else None
    db = (torch.empty_like if boxes.is_contiguous() else torch.zeros_like)(boxes) if need_grad else None
    a = N.DetLossArgs()
    a.R, a.ncls = logits.shape
    a.logits, a.ld_logits, a.labels, a.label_w = logits.data_ptr(), logits.stride(0), labels.data_ptr(), _ptr(label_w)
    a.Rb = boxes.shape[0]
    a.boxes, a.ld_boxes, a.targets, a.box_w = boxes.data_ptr(), boxes.stride(0), targets.data_ptr(), box_w.data_ptr()
    a.gamma, a.alpha, a.cls_weight, a.box_weight = gamma, alpha, cls_weight, box_weight
    a.cls_avg, a.box_avg, a.gscale = cls_avg, box_avg, 1.0
    a.out, a.dlogits, a.dboxes = out.data_ptr(), _ptr(dl), _ptr(db)
    N._check(N.lib().cmt_det_loss(ctypes.byref(a), N._stream()), "cmt_det_loss")
    return out, dl, db


def match_cost(logits, boxes, gt, gt_labels, code_w, *, gamma, alpha, cls_weight, reg_weight):
    _f32(logits, boxes, gt, code_w)
    N._dev(gt_labels)
    Nq, ngt = logits.shape[0], gt.shape[0]
    cost = torch.empty((Nq, ngt), dtype=torch.float32, device=logits.device)
    a = N.MatchCostArgs()
    a.Nq, a.ngt = Nq, ngt
    a.logits, a.ld_logits, a.boxes, a.ld_boxes = logits.data_ptr(), logits.stride(0), boxes.data_ptr(), boxes.stride(0)
    a.gt, a.gt_labels, a.code_w = gt.data_ptr(), gt_labels.data_ptr(), code_w.data_ptr()
    a.gamma, a.alpha, a.cls_weight, a.reg_weight, a.cost = gamma, alpha, cls_weight, reg_weight, cost.data_ptr()
    N._check(N.lib().cmt_match_cost(ctypes.byref(a), N._stream()), "cmt_match_cost")
    return cost


def sumsq(x, out):
    _f32(x, out)
    N._check(N.lib().cmt_sumsq(x.data_ptr(), x.numel(), out.data_ptr(), N._stream()), "cmt_sumsq")


def adamw_step(param, grad, exp_avg, exp_avg_sq, *, step, lr, beta1, beta2, eps, weight_decay, max_norm=0.0,
               sumsq_buf=None):
    _f32(param, grad, exp_avg, exp_avg_sq, sumsq_buf)
    a = N.AdamwArgs()
    a.n, a.step, a.lr, a.beta1, a.beta2, a.eps = param.numel(), step, lr, beta1, beta2, eps
    a.weight_decay, a.max_norm = weight_decay, max_norm
    a.param, a.grad, a.exp_avg, a.exp_avg_sq = param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr()
    a.sumsq = _ptr(sumsq_buf)
    N._check(N.lib().cmt_adamw_step(ctypes.byref(a), N._stream()), "cmt_adamw_step")
