"""torch.autograd Functions of the training path: forward AND backward run on
the gfx950 kernels of train.hip / attn_train.hip (native_train.py).  Autograd
is only the bookkeeping (which gradient goes where); reshapes, residual adds,
ReLU masks and the few-element box epilogue between these ops are plain
tensor glue on the device.

Reference semantics (training step of CmtHead / CmtHeadCoop):
  Linear          nn.Linear / the packed in_proj of nn.MultiheadAttention and
                  FlashMHA (attention.py:21-27), mmcv FFN, the MLPs
  attention       nn.MultiheadAttention core (fp32, DN mask cmt_head.py:386-398,
                  attn_drop) and the flash-attn 0.2.2 fp16 cross core
  LayerNorm       nn.LayerNorm (eps 1e-5) and GroupLayerNorm1d (cmt_head.py:53-94)
  BN + ReLU       shared_conv's BatchNorm2d (training statistics) + ReLU
  conv3x3         shared_conv's Conv2d (no bias): forward on cmt_gemm's exact-f32
                  implicit-GEMM path, weight gradient = dY^T im2col(X), input
                  gradient = the same implicit conv on the flipped weights
  nchw_rows       the memory-row layout of the feature maps (gradient back to NCHW)
"""
import contextlib
import math

import torch

from ... import native
from ... import native_train as T
from ...runtime import SPLIT

__all__ = ["linear", "linear_batched", "taps3", "attention", "layer_norm", "group_layer_norm", "bn_relu", "conv3x3", "nchw_rows", "det_loss",
           "direct_param_grads", "kv_all", "cross_attention", "layer_loss"]


# ---- parameter gradients written in place (ABI 24).  Inside direct_param_grads() the backward of
# a Linear / LayerNorm whose weight (and bias) is a leaf parameter -- or a contiguous view of one,
# like the chunks of nn.MultiheadAttention's packed in_proj -- adds its weight / bias gradient
# straight into that parameter's .grad (allocated zeroed on first use, as autograd would) and
# returns None for it: no gradient temporary, no zero fill of a split-K reduction, no
# AccumulateGrad add per parameter and use.  Only the Trainer's backward() turns it on, and only
# where nothing hooks the accumulation (world size 1: the bucketed all-reduce counts
# post-accumulate-grad hooks) and no graph is being captured; .grad then holds exactly what
# autograd would have accumulated (tests/test_gpu_train_head.py::test_direct_param_grads_match).
# A process-wide switch, not a thread-local one: autograd runs a GPU backward on its own device
# thread.  ``writes`` counts the gradients added in place (tests check the path ran).
class _DirectState:
    on = False
    writes = 0


_direct = _DirectState()


@contextlib.contextmanager
def direct_param_grads(enabled=True):
    prev = _direct.on
    _direct.on = bool(enabled)
    try:
        yield
    finally:
        _direct.on = prev


def _grad_target(t):
    """The tensor t's gradient should be added to in place (a view of its parameter's .grad), or
    None when t's gradient must go back through autograd."""
    if t is None or not _direct.on or not t.requires_grad:
        return None
    p = t if t.is_leaf else t._base
    if p is None or not p.is_leaf or not t.is_contiguous() or getattr(p, "_post_accumulate_grad_hooks", None):
        return None
    if not t.is_leaf and (t._base._base is not None or t.grad_fn is None):
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    g = p.grad
    if not g.is_contiguous() or g.dtype != t.dtype:
        return None
    _direct.writes += 1
    if t is p:
        return g
    # t is a contiguous view of the contiguous parameter p: the same elements of its .grad
    return g.reshape(-1)[t.storage_offset() - p.storage_offset():][:t.numel()].view(t.shape)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.wb = (w, b)
        return T.linear_fwd(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        need_db = ctx.has_b and ctx.needs_input_grad[2]
        gw = gb = None
        if ctx.needs_input_grad[1]:
            gw = _grad_target(ctx.wb[0])
            gb = _grad_target(ctx.wb[1]) if need_db else None
            if gw is None or (need_db and gb is None):
                gw = gb = None
        if gw is not None:
            dx, _, _ = T.linear_bwd(dy, x, w, need_dx=ctx.needs_input_grad[0], need_dw=True, need_db=need_db,
                                    dw_into=gw, db_into=gb)
            return dx, None, None
        dx, dw, db = T.linear_bwd(dy, x, w, need_dx=ctx.needs_input_grad[0], need_dw=ctx.needs_input_grad[1],
                                  need_db=need_db)
        return dx, dw, db


def linear(x, w, b=None):
    """x [..., K] -> [..., N] (rows flattened, fp32)."""
    shape = x.shape
    y = _Linear.apply(x.reshape(-1, shape[-1]).contiguous(), w.contiguous(), b)
    return y.view(*shape[:-1], w.shape[0])


class _LinearBatched(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return T.linear_fwd_batched(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        return T.linear_bwd_batched(dy, x, w, need_dx=ctx.needs_input_grad[0], need_dw=ctx.needs_input_grad[1],
                                    need_db=ctx.has_b and ctx.needs_input_grad[2])


def linear_batched(x, w, b=None):
    """x [L, ..., K], w [L, N, K], b [L, N] -> [L, ..., N]: one Linear per leading index (the task
    heads' per-layer grouped Conv1d) in one launch, forward and backward."""
    shape = x.shape
    y = _LinearBatched.apply(x.reshape(shape[0], -1, shape[-1]).contiguous(), w.contiguous(),
                             None if b is None else b.contiguous())
    return y.view(*shape[:-1], w.shape[1])


class _Attention(torch.autograd.Function):
    """q [B, Nq, H*32], k / v [B, Nk, H*32] (contiguous rows) -> o [B, Nq, H*32]."""

    @staticmethod
    def forward(ctx, q, k, v, H, scale, dn_pad, dn_group, fp16, dropout_p, seed, seed_dev):
        B, Nq, C = q.shape
        Nk = k.shape[1]
        o = torch.empty_like(q)
        lse = torch.empty((B * H * Nq,), dtype=torch.float32, device=q.device)
        kw = dict(B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(Nq * C, 32, C), k_strides=(Nk * C, 32, C),
                  v_strides=(Nk * C, 32, C), o_strides=(Nq * C, 32, C), scale=scale, dn_pad=dn_pad,
                  dn_group=dn_group, fp16_inputs=fp16, dropout_p=dropout_p, seed=seed, seed_dev=seed_dev)
        ctx.ws = T.attn_train_fwd(q, k, v, o, lse, **kw)
        ctx.kw = kw
        ctx.save_for_backward(q, k, v, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        T.attn_train_bwd(q, k, v, o, lse, do.contiguous(), dq, dk, dv, ws=ctx.ws, **ctx.kw)
        ctx.ws = None
        return dq, dk, dv, None, None, None, None, None, None, None, None


class KVAll:
    """One agent's cross-attention keys / values of EVERY decoder layer (kv_all) and the arena
    their gradients are written into by the layers' attention backward (cross_attention)."""

    def __init__(self):
        self.K = self.V = self.dK = self.dV = None
        self.written = set()


class _KVAll(torch.autograd.Function):
    """K_l = (mem + pos) Wk_l^T + bk_l and V_l = mem Wv_l^T + bv_l of all L layers as TWO Linears of
    width L C (FlashMHA's packed in_proj, attention.py:21-27, per layer): [B, Nk, L C] each, layer l
    in columns [l C, (l + 1) C).  Its output is a 0-dim token the layers' cross_attention calls
    take as input; their backward writes dK_l / dV_l straight into the holder's arena (strided,
    no per-layer gradient tensor, no accumulation), and this backward runs the two Linears'
    backward once: d(mem + pos) = dK Wk (reduction over L C), dW = dK^T (mem + pos) -- instead
    of 2 L projection GEMMs each way, L per-layer weight-gradient GEMMs of a 256 x 256 output
    split over the ~40 k key rows, and 2 L - 2 [Nk, C] gradient additions."""

    @staticmethod
    def forward(ctx, memk, mem, holder, nl, *wb):
        B, Nk, C = memk.shape
        wk, bk, wv, bv = wb[:nl], wb[nl:2 * nl], wb[2 * nl:3 * nl], wb[3 * nl:]
        ctx.has_b = bk[0] is not None
        Wk, Wv = torch.cat(wk, 0), torch.cat(wv, 0)
        bkc = torch.cat(bk, 0) if ctx.has_b else None
        bvc = torch.cat(bv, 0) if ctx.has_b else None
        xk, xv = memk.reshape(B * Nk, C), mem.reshape(B * Nk, C)
        holder.K = T.linear_fwd(xk, Wk, bkc).view(B, Nk, nl * C)
        holder.V = T.linear_fwd(xv, Wv, bvc).view(B, Nk, nl * C)
        holder.dK = holder.dV = None
        holder.written = set()
        ctx.save_for_backward(xk, xv, Wk, Wv)
        ctx.holder, ctx.nl, ctx.shape = holder, nl, (B, Nk, C)
        ctx.set_materialize_grads(False)
        return memk.new_zeros(())

    @staticmethod
    def backward(ctx, _token_grad):
        xk, xv, Wk, Wv = ctx.saved_tensors
        h, nl, (B, Nk, C) = ctx.holder, ctx.nl, ctx.shape
        if h.dK is None:
            return (None,) * (4 + 4 * nl)
        for l in set(range(nl)) - h.written:      # a layer whose attention got no gradient
            h.dK[..., l * C:(l + 1) * C].zero_()
            h.dV[..., l * C:(l + 1) * C].zero_()
        gin = ctx.needs_input_grad
        outs = []
        for x, W, d, need_x, off in ((xk, Wk, h.dK, gin[0], 4), (xv, Wv, h.dV, gin[1], 4 + 2 * nl)):
            need_w = any(gin[off:off + nl])
            need_b = ctx.has_b and any(gin[off + nl:off + 2 * nl])
            dx, dw, db = T.linear_bwd(d.view(B * Nk, nl * C), x, W, need_dx=need_x, need_dw=need_w or need_b,
                                      need_db=need_b)
            dws = list(dw.split(C, 0)) if need_w else [None] * nl
            dbs = list(db.split(C, 0)) if need_b else [None] * nl
            outs.append((None if dx is None else dx.view(B, Nk, C), dws, dbs))
        h.K = h.V = h.dK = h.dV = None            # the step's K / V and their gradients are done
        (dmk, dwk, dbk), (dm, dwv, dbv) = outs
        return (dmk, dm, None, None, *dwk, *dbk, *dwv, *dbv)


def kv_all(memk, mem, layers_kv):
    """layers_kv: per layer (wk, bk, wv, bv) -- the K / V chunks of its packed in_proj.  Returns
    (holder, token) for cross_attention."""
    holder = KVAll()
    nl = len(layers_kv)
    wb = [t[0] for t in layers_kv] + [t[1] for t in layers_kv] + [t[2] for t in layers_kv] + \
         [t[3] for t in layers_kv]
    token = _KVAll.apply(memk.contiguous(), mem.contiguous(), holder, nl, *[w.contiguous() if w is not None else None
                                                                           for w in wb])
    return holder, token


_ZERO_TOKEN = {}


class _CrossAttn(torch.autograd.Function):
    """The cross-attention core of layer l on the all-layer K / V of kv_all (columns [l C, (l+1) C),
    strided rows: no copy); its backward writes dK_l / dV_l into the holder's arena."""

    @staticmethod
    def forward(ctx, q, token, holder, l, H, scale, fp16):
        B, Nq, C = q.shape
        K, V = holder.K[..., l * C:(l + 1) * C], holder.V[..., l * C:(l + 1) * C]
        Nk, ld = K.shape[1], K.stride(1)
        o = torch.empty_like(q)
        lse = torch.empty((B * H * Nq,), dtype=torch.float32, device=q.device)
        kw = dict(B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(Nq * C, 32, C), k_strides=(K.stride(0), 32, ld),
                  v_strides=(V.stride(0), 32, V.stride(1)), o_strides=(Nq * C, 32, C), scale=scale, dn_pad=0,
                  dn_group=0, fp16_inputs=fp16, dropout_p=0.0, seed=0, seed_dev=None)
        # the workspace holds the f16 copies of q / K / V the backward reuses (ABI 25)
        ctx.ws = T.attn_train_fwd(q, K, V, o, lse, **kw)
        ctx.kw, ctx.holder, ctx.l = kw, holder, l
        ctx.save_for_backward(q, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        q, o, lse = ctx.saved_tensors
        h, l = ctx.holder, ctx.l
        C = q.shape[2]
        if h.dK is None:
            h.dK, h.dV = torch.empty_like(h.K), torch.empty_like(h.V)
        K, V = h.K[..., l * C:(l + 1) * C], h.V[..., l * C:(l + 1) * C]
        dK, dV = h.dK[..., l * C:(l + 1) * C], h.dV[..., l * C:(l + 1) * C]
        dq = torch.empty_like(q)
        T.attn_train_bwd(q, K, V, o, lse, do.contiguous(), dq, dK, dV, ws=ctx.ws, **ctx.kw)
        ctx.ws = None
        h.written.add(l)
        z = _ZERO_TOKEN.get(q.device)
        if z is None:
            z = _ZERO_TOKEN[q.device] = torch.zeros((), dtype=torch.float32, device=q.device)
        return dq, z, None, None, None, None, None


def cross_attention(q, token, holder, l, num_heads, *, fp16=True):
    return _CrossAttn.apply(q.contiguous(), token, holder, l, num_heads, 1.0 / math.sqrt(q.shape[-1] // num_heads),
                            fp16)


def attention(q, k, v, num_heads, *, dn_pad=0, dn_group=0, fp16=False, dropout_p=0.0, seed=0, seed_dev=None):
    """seed_dev: optional int32 device tensor [1] added to seed on the device (graph-replayed steps)"""
    return _Attention.apply(q.contiguous(), k.contiguous(), v.contiguous(), num_heads,
                            1.0 / math.sqrt(q.shape[-1] // num_heads), dn_pad, dn_group, fp16, dropout_p, seed,
                            seed_dev)


class _Taps3(torch.autograd.Function):
    """x [..., Nq, C] -> [..., Nq, 3C]: the three taps q - 1, q, q + 1 of a kernel-3 Conv1d along
    the queries (zero padded), as the GEMM operand of the task heads' grouped convs; the backward
    sums the three shifted gradient slices (one fill + three adds, where the autograd of pad +
    three slices + cat took a zero fill, a copy and an add per slice)."""

    @staticmethod
    def forward(ctx, x):
        Nq = x.shape[-2]
        xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
        return torch.cat([xp[..., 0:Nq, :], xp[..., 1:Nq + 1, :], xp[..., 2:Nq + 2, :]], -1)

    @staticmethod
    def backward(ctx, g):
        Nq, C = g.shape[-2], g.shape[-1] // 3
        gp = g.new_zeros(g.shape[:-2] + (Nq + 2, C))
        gp[..., 0:Nq, :] += g[..., 0:C]
        gp[..., 1:Nq + 1, :] += g[..., C:2 * C]
        gp[..., 2:Nq + 2, :] += g[..., 2 * C:]
        return gp[..., 1:Nq + 1, :]


def taps3(x):
    return _Taps3.apply(x)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps, rows_per_wset, wsets):
        y, mean, rstd = T.ln_train_fwd(x, w, b, eps=eps, rows_per_wset=rows_per_wset)
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.eps, ctx.rpw, ctx.wsets = eps, rows_per_wset, wsets
        ctx.wb = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        if ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            gw, gb = _grad_target(ctx.wb[0]), _grad_target(ctx.wb[1])
            if gw is not None and gb is not None:
                dx, _, _ = T.ln_train_bwd(dy, x, w, mean, rstd, eps=ctx.eps, rows_per_wset=ctx.rpw, wsets=ctx.wsets,
                                          dw_into=gw, db_into=gb)
                return dx, None, None, None, None, None
        dx, dw, db = T.ln_train_bwd(dy, x, w, mean, rstd, eps=ctx.eps, rows_per_wset=ctx.rpw, wsets=ctx.wsets)
        return dx, dw.view(w.shape), db.view(w.shape), None, None, None


def layer_norm(x, w, b, eps=1e-5):
    shape = x.shape
    return _LayerNorm.apply(x.reshape(-1, shape[-1]).contiguous(), w, b, eps, 0, 1).view(shape)


def group_layer_norm(x, w, b, eps=1e-6):
    """x [G, R, 64]: LayerNorm over the 64 channels of every row with weight set
    g for rows of group g (GroupLayerNorm1d, cmt_head.py:53-94); w, b [G*64]."""
    G, R, Cg = x.shape
    return _LayerNorm.apply(x.reshape(G * R, Cg).contiguous(), w, b, eps, R, G).view(G, R, Cg)


class _BnRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, running_mean, running_var, eps, momentum):
        y, mean, rstd = T.bn_relu_train_fwd(x, w, b, running_mean, running_var, eps=eps, momentum=momentum)
        # the kernel updated the running statistics through their pointers: bump the versions so
        # weight packs built from them (the BN fold of the inference engine) are rebuilt
        for t in (running_mean, running_var):
            if t is not None:
                torch.autograd.graph.increment_version(t)
        ctx.save_for_backward(x, y, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = T.bn_relu_train_bwd(dy, x, y, w, mean, rstd)
        return dx, dw, db, None, None, None, None


def bn_relu(x, bn):
    """relu(bn(x)) with training statistics; x rows [B*H*W, C]."""
    return _BnRelu.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum)


class _Conv3x3(torch.autograd.Function):
    """NHWC rows [B*H*W, Cin] -> [B*H*W, Cout]; weight [Cout, 9*Cin] tap-major."""

    @staticmethod
    def forward(ctx, x, w, geom):
        B, H, W, Cin = geom
        Cout = w.shape[0]
        y = torch.empty((B * H * W, Cout), dtype=torch.float32, device=x.device)
        if T._gemm_mode == "f32" or Cout % 128 or Cin % 32:
            native.gemm(x, w, y, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout,
                        a_mode=native.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin,
                        c_bstride=H * W * Cout)
        else:
            # the split-f16 implicit-GEMM conv of the inference path (three f16 MFMA passes on pair
            # operands, ~2^-21 relative per product): 3x the exact-f32 MFMA's speed at this size.
            # Its input operand is range-checked where it is laid out (nchw_rows(range_flag=...):
            # the head's device word, CmtHead.check_input_range(); no host sync in the step); the
            # conv OUTPUT stays fp32 into BatchNorm, so a large but valid output is not flagged
            xs = native.split_rows(x)
            wh = w.detach().half()                                   # pair weights (no host range check:
            ws = torch.stack([wh, (w.detach() - wh.float()).half()], dim=-2).contiguous().view(SPLIT)   # no sync)
            native.gemm(xs, ws, y, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout,
                        a_mode=native.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin,
                        c_bstride=H * W * Cout)
        ctx.save_for_backward(x, w)
        ctx.geom = geom
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        B, H, W, Cin = ctx.geom
        Cout = w.shape[0]
        dw = None
        if ctx.needs_input_grad[1]:
            rows = B * H * W
            ks = max(T._ksplit(rows, Cout, 9 * Cin), 2)
            if T._gemm_mode == "bf16x3" and Cin % 4 == 0 and Cout % 4 == 0:
                # the im2col operand gathered inside the GEMM (no [rows, 9 Cin] matrix)
                dw = T.conv3x3_wgrad(x, dy, B, H, W, Cin, ks)
            else:
                col = T.im2col3x3(x, B, H, W, Cin)                 # [rows, 9*Cin]
                dw = torch.zeros((Cout, 9 * Cin), dtype=torch.float32, device=x.device)
                T.gemm_ex(dy.contiguous(), (1, Cout), col, (1, 9 * Cin), dw, M=Cout, N_=9 * Cin, K=rows,
                          ldc=9 * Cin, beta=1.0, ksplit=ks)
        dx = None
        if ctx.needs_input_grad[0]:
            # dX = conv3x3(dY, W'), W'[cin][tap][cout] = W[cout][8 - tap][cin]: the transposed conv is the
            # same implicit GEMM on the spatially flipped, transposed weights (zero padding included)
            wt = w.view(Cout, 9, Cin).flip(1).permute(2, 1, 0).reshape(Cin, 9 * Cout).contiguous()
            dx = torch.empty((B * H * W, Cin), dtype=torch.float32, device=x.device)
            native.gemm(dy.contiguous(), wt, dx, M=H * W, N=Cin, K=9 * Cout, lda=Cout, ldw=9 * Cout, ldc=Cin,
                        a_mode=native.A_CONV3X3, conv=(H, W, Cout), batch=B, a_bstride=H * W * Cout,
                        c_bstride=H * W * Cin)
        return dx, dw, None


def conv3x3(x_rows, w_tap_major, geom):
    return _Conv3x3.apply(x_rows, w_tap_major, geom)


class _NchwRows(torch.autograd.Function):
    """Feature maps [B*V, C, H, W] -> memory rows [B*V*H*W, C] ("(bs v) c h w ->
    bs (v h w) c", cmt_transformer.py:104-105) on the native layout kernel;
    the backward is the transpose back, so the backbone / neck that produced
    the maps receives its gradient as in the reference."""

    @staticmethod
    def forward(ctx, x, B, range_flag=None):
        BV, C, H, W = x.shape
        y = torch.empty((BV * H * W, C), dtype=torch.float32, device=x.device)
        native.nchw_to_rows(x.contiguous().float(), y, nb=B, nv=BV // B, C=C, HW=H * W, ldy=C,
                            rows_per_batch=BV // B * H * W, range_flag=range_flag)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        BV, C, H, W = ctx.shape
        return dy.view(BV, H * W, C).transpose(1, 2).reshape(BV, C, H, W), None, None


def nchw_rows(x, B, range_flag=None):
    """range_flag: the head's f16-operand range word (int32 device tensor), set when an input
    value cannot be carried as an f16 pair (|x| >= 65520, non-finite) -- for rows a split-f16
    kernel reads next (the training shared_conv)."""
    return _NchwRows.apply(x, B, range_flag)


class _DetLoss(torch.autograd.Function):
    """FocalLoss + L1Loss of one (layer, task): returns a [2] tensor (cls, box);
    the kernel computes the input gradients in the same launch."""

    @staticmethod
    def forward(ctx, logits, boxes, labels, label_w, targets, box_w, cfg):
        lg, bx = logits.contiguous(), boxes.contiguous()
        out, dl, db = T.det_loss(lg, labels, label_w, bx, targets, box_w, **cfg)
        ctx.save_for_backward(dl, db)
        return out

    @staticmethod
    def backward(ctx, dout):
        dl, db = ctx.saved_tensors
        return dl * dout[0], db * dout[1], None, None, None, None, None


def det_loss(logits, boxes, labels, label_w, targets, box_w, **cfg):
    return _DetLoss.apply(logits, boxes, labels, label_w, targets, box_w, cfg)


class _LayerLoss(torch.autograd.Function):
    """The loss terms of one (decoder layer, task) in ONE autograd node (cmt_head.py:815-903):
    the matching queries' FocalLoss + L1Loss (loss_single) and, with DN queries, the DN
    classification term over every DN row and the box term over the task's rows
    (dn_loss_single) -- one cmt_det_loss launch each, the DN one with dn_weight folded into the
    loss weights -- each term through torch.nan_to_num as the reference applies it.  Returns the
    [2] or [4] term vector; its backward scales the kernels' input gradients by the incoming
    gradient where the raw term was finite (NanToNumBackward)."""

    @staticmethod
    def forward(ctx, pl, pb, dpl, dpb, labels, lw, nt, w, cfg, dn):
        n = 4 if dpl is not None else 2
        raw = torch.empty(n, dtype=torch.float32, device=pl.device)
        _, dl, db = T.det_loss(pl.contiguous(), labels, lw, pb.contiguous(), nt, w, out=raw[0:2], **cfg)
        grads = [dl, db]
        if dpl is not None:
            kl, dlw, ntg, dw, dcfg = dn
            _, dlc, dbb = T.det_loss(dpl.contiguous(), kl, dlw, dpb.contiguous(), ntg, dw, out=raw[2:4], **dcfg)
            grads += [dlc, dbb]
        ctx.save_for_backward(raw, *grads)
        ctx.n = n
        return torch.nan_to_num(raw)

    @staticmethod
    def backward(ctx, dv):
        raw, *grads = ctx.saved_tensors
        g = dv * torch.isfinite(raw)
        out = [grads[i] * g[i] for i in range(ctx.n)]
        if ctx.n == 2:
            out += [None, None]
        return (*out, None, None, None, None, None, None)


def layer_loss(pl, pb, labels, lw, nt, w, cfg, dpl=None, dpb=None, kl=None, dlw=None, ntg=None, dw=None, dcfg=None):
    """-> tuple of the (layer, task)'s loss terms: (loss_cls, loss_bbox[, dn_loss_cls, dn_loss_bbox])."""
    dn = (kl, dlw, ntg, dw, dcfg) if dpl is not None else None
    return _LayerLoss.apply(pl, pb, dpl, dpb, labels, lw, nt, w, cfg, dn).unbind(0)
