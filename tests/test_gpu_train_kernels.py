"""Training-path kernels (train.hip, attn_train.hip) against float64 PyTorch CPU
autograd of the same math: general-stride GEMM (every transpose), attention
forward statistics + backward (DN mask, ragged shapes, fp16-core rounding,
hash dropout), LayerNorm / GroupLayerNorm1d, BatchNorm2d+ReLU (training
statistics), im2col, FocalLoss+L1Loss, the Hungarian cost matrix and AdamW
with gradient-norm clipping."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _T():
    from projects.mmdet3d_plugin import native_train as T
    return T


@pytest.mark.parametrize("mode", ["f32", "bf16x3"])
@pytest.mark.parametrize("M,N,K,ta,tb", [(100, 70, 50, False, False), (256, 256, 900, True, True),
                                         (33, 257, 64, False, True), (64, 64, 4000, True, False),
                                         # 128 x 128 tiles: a very large ragged product (>= 1 536 tiles, no
                                         # split) and a long reduction whose split-K the launcher re-chooses
                                         (12300, 2060, 40, False, False), (12300, 2060, 40, True, True),
                                         (256, 256, 70000, True, False)])
def test_gemm_ex_transposes(dev, M, N, K, ta, tb, mode):
    """cmt_gemm_f32_ex (exact f32) and cmt_gemm_bf16x3_ex (three bf16 passes on split
    operands) against float64, every transpose, split-K; the bf16x3 form also on
    operands scaled by 2^-30 (gradient-sized values keep their relative accuracy:
    bf16 pairs have the fp32 exponent range)."""
    T = _T()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g) if tb else torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    ref = (A.double().t() if ta else A.double()) @ (B.double() if tb else B.double().t()) * 0.5 + bias.double()
    Ad, Bd = A.to(dev), B.to(dev)
    C = torch.empty(M, N, device=dev)
    a_str = (1, M) if ta else (K, 1)
    b_str = (1, N) if tb else (K, 1)
    T.gemm_ex(Ad, a_str, Bd, b_str, C, M=M, N_=N, K=K, ldc=N, alpha=0.5, bias=bias.to(dev), mode=mode)
    C2 = torch.zeros(M, N, device=dev)
    T.gemm_ex(Ad, a_str, Bd, b_str, C2, M=M, N_=N, K=K, ldc=N, alpha=0.5, beta=1.0, bias=bias.to(dev), ksplit=4,
              mode=mode)
    torch.cuda.synchronize()
    # f32: fp32 rounding; bf16x3: ~2^-16 of each product (|a b| ~ 1 here, a random walk over K)
    tol = 1e-5 * math.sqrt(K) * 4 if mode == "f32" else 2 ** -15 * math.sqrt(K) * 4
    assert (C.cpu().double() - ref).abs().max().item() < tol
    assert (C2.cpu().double() - ref).abs().max().item() < tol
    if mode == "bf16x3":
        # a_rowsum (ABI 17): the fp32 row sums of A accumulated by the first column tile, split-K too
        rs = torch.zeros(M, device=dev)
        C4 = torch.zeros(M, N, device=dev)
        T.gemm_ex(Ad, a_str, Bd, b_str, C4, M=M, N_=N, K=K, ldc=N, beta=1.0, ksplit=4, mode=mode, a_rowsum=rs)
        torch.cuda.synchronize()
        want = (A.double().t() if ta else A.double()).sum(1)
        assert (rs.cpu().double() - want).abs().max().item() < 1e-5 * math.sqrt(K) * 4
        tiny = 2.0 ** -30
        C3 = torch.empty(M, N, device=dev)
        T.gemm_ex(Ad * tiny, a_str, Bd * tiny, b_str, C3, M=M, N_=N, K=K, ldc=N, alpha=0.5, mode=mode)
        torch.cuda.synchronize()
        ref3 = (ref - bias.double()) * tiny * tiny
        assert (C3.cpu().double() - ref3).abs().max().item() < tol * tiny * tiny


@pytest.mark.parametrize("M,K,N,ks,case", [
    (384, 256, 256, 1, "dX and dW on the k-wave kernel (< 256 tiles, >= 4 k-steps, unsplit)"),
    (8192, 256, 1024, 8, "dW on 128 x 128 tiles, the split re-chosen 8 -> 32 after the zero fill"),
    (4096, 256, 64, 8, "dX on the plain 64 x 64 tile (2-step reduction), dW split on 64 x 64"),
    (30, 96, 48, 2, "split 2 rounded back to 1 by the k chunk while beta is 1 (zero-filled dW)")])
@pytest.mark.parametrize("need", [(True, True, True), (True, True, False), (True, False, True), (False, True, True)])
def test_linear_bwd_bf16x3_direct(dev, M, K, N, ks, case, need):
    """cmt_linear_bwd_bf16x3 (ABI 23, one call: dX = dY W, dW = dY^T X with the bias gradient
    as the A row sums of the weight-gradient GEMM) against float64, with the split chosen
    by the caller -- each shape selects another kernel path (``case``) -- and every
    need_dx / need_dw / need_db combination (need_db without need_dw: the column sum)."""
    from projects.mmdet3d_plugin import native as N_
    T = _T()
    need_dx, need_dw, need_db = need
    g = torch.Generator().manual_seed(M + K + N)
    dY, X, W = torch.randn(M, N, generator=g), torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    dYd, Xd, Wd = dY.to(dev), X.to(dev), W.to(dev)
    if need_dw:       # the raw entry point, with this case's split (the wrapper picks its own)
        dX = torch.full((M, K), float("nan"), device=dev) if need_dx else None
        dW = torch.full((N, K), float("nan"), device=dev)
        dB = torch.full((N,), float("nan"), device=dev) if need_db else None
        p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        N_._check(N_.lib().cmt_linear_bwd_bf16x3(dYd.data_ptr(), Xd.data_ptr(), Wd.data_ptr(), p(dX), p(dW), p(dB),
                                                 M, K, N, K, ks, N_._stream()), "cmt_linear_bwd_bf16x3")
    else:
        prev = T._gemm_mode
        T.set_train_gemm("bf16x3")
        try:
            dX, dW, dB = T.linear_bwd(dYd, Xd, Wd, need_dx=need_dx, need_dw=False, need_db=need_db)
        finally:
            T.set_train_gemm(prev)
    torch.cuda.synchronize()
    want = {"dX": dY.double() @ W.double(), "dW": dY.double().t() @ X.double(), "dB": dY.double().sum(0)}
    got = {"dX": dX, "dW": dW, "dB": dB}
    for name, on in (("dX", need_dx), ("dW", need_dw), ("dB", need_db)):
        if not on:
            assert got[name] is None, (case, name)
            continue
        red = {"dX": N, "dW": M, "dB": M}[name]
        # bf16x3: ~2^-16 of each product, a random walk over the reduction; dB is an fp32 sum
        tol = (2 ** -15 if name != "dB" else 1e-6) * math.sqrt(red) * 4
        err = (got[name].cpu().double() - want[name]).abs().max().item()
        assert err < tol, (case, name, err, tol)



@pytest.mark.parametrize("L,M,K,N", [(6, 1100, 192, 64), (3, 70, 33, 10)])
def test_linear_batched_fwd_bwd(dev, L, M, K, N):
    """train_ops.linear_batched (one batched launch per product, per-entry bias through the
    ABI-16 bias batch stride) against float64 autograd of L separate Linears."""
    from projects.mmdet3d_plugin.models.utils import train_ops as ops
    g = torch.Generator().manual_seed(L * M + K)
    x, w, b = torch.randn(L, M, K, generator=g), torch.randn(L, N, K, generator=g) * 0.1, torch.randn(L, N, generator=g)
    dy = torch.randn(L, M, N, generator=g)
    xd, wd, bd = (t.double().requires_grad_() for t in (x, w, b))
    yd = torch.einsum("lmk,lnk->lmn", xd, wd) + bd[:, None]
    yd.backward(dy.double())
    xg, wg, bg = (t.to(dev).requires_grad_() for t in (x, w, b))
    y = ops.linear_batched(xg, wg, bg)
    y.backward(dy.to(dev))
    torch.cuda.synchronize()
    tol = 2 ** -15 * math.sqrt(max(K, M)) * 8
    for got, want in ((y, yd), (xg.grad, xd.grad), (wg.grad, wd.grad), (bg.grad, bd.grad)):
        err = (got.detach().cpu().double() - want.detach()).abs().max().item()
        assert err < tol * max(1.0, want.abs().max().item() / 10), err


def _mix32(x):
    x = x.astype(np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7feb352d) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846ca68b) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def keep_mask(seed, B, H, Nq, Nk, p):
    """Host restatement of attn_train.hip keep(): keep iff hash >= p * 2^32."""
    bh = np.arange(B * H, dtype=np.uint64)[:, None, None]
    q = np.arange(Nq, dtype=np.uint64)[None, :, None]
    k = np.arange(Nk, dtype=np.uint64)[None, None, :]
    h = _mix32(np.uint64(seed) ^ _mix32((bh * 0x9e3779b9 + q) & 0xFFFFFFFF))
    h = _mix32(h ^ ((k * 0x85ebca6b) & 0xFFFFFFFF))
    thr = min(int(p * 4294967296.0), 0xFFFFFFFF)
    return torch.from_numpy(h >= thr).view(B, H, Nq, Nk)


def dn_mask(Nq, Nk, pad, grp):
    q = torch.arange(Nq)[:, None]
    k = torch.arange(Nk)[None, :]
    return (k < pad) & ((q >= pad) | (k // grp != q // grp))


@pytest.mark.parametrize("B,Nq,Nk,pad,grp,fp16,p", [(1, 100, 1000, 0, 0, False, 0.0), (2, 70, 70, 30, 10, False, 0.0),
                                                    (1, 140, 140, 40, 8, False, 0.25), (1, 96, 3000, 0, 0, True, 0.0),
                                                    (2, 150, 1100, 50, 10, True, 0.25), (1, 200, 2049, 0, 0, True, 0.1),
                                                    (1, 77, 300, 40, 8, True, 0.0),
                                                    # the long-key fp16 path (cross-attention of the training step:
                                                    # attention core with the row statistic, LDS-resident dK/dV,
                                                    # K/V-streaming dQ): ragged key tiles, two batch elements, the
                                                    # LDS bound of 1 152 queries; 1 200 queries take the general kernels
                                                    (1, 900, 8192, 0, 0, True, 0.0), (2, 1100, 4100, 0, 0, True, 0.0),
                                                    (1, 1152, 5000, 0, 0, True, 0.0), (1, 1200, 4096, 0, 0, True, 0.0)])
def test_attention_train_fwd_bwd(dev, B, Nq, Nk, pad, grp, fp16, p):
    T = _T()
    H, C = 8, 256
    g = torch.Generator().manual_seed(Nq * 7 + Nk)
    q = torch.randn(B, Nq, C, generator=g)
    k = torch.randn(B, Nk, C, generator=g)
    v = torch.randn(B, Nk, C, generator=g)
    do = torch.randn(B, Nq, C, generator=g)
    seed = 1234

    def ref_fn(q, k, v):
        def r(t):
            return t.half().double() if fp16 else t
        qh = r(q).view(B, Nq, H, 32).transpose(1, 2)
        kh = r(k).view(B, Nk, H, 32).transpose(1, 2)
        vh = r(v).view(B, Nk, H, 32).transpose(1, 2)
        s = qh @ kh.transpose(-1, -2) / math.sqrt(32)
        if pad:
            s = s.masked_fill(dn_mask(Nq, Nk, pad, grp), float("-inf"))
        pr = torch.softmax(s, -1)
        if p > 0:
            pr = pr * keep_mask(seed, B, H, Nq, Nk, p).double() / (1 - p)
        return (pr @ vh).transpose(1, 2).reshape(B, Nq, C)
    qd, kd, vd = (t.double().requires_grad_() for t in (q, k, v))
    ref = ref_fn(qd, kd, vd)
    ref.backward(do.double())
    qg, kg, vg = (t.to(dev).requires_grad_() for t in (q, k, v))
    from projects.mmdet3d_plugin.models.utils import train_ops as O
    out = O.attention(qg, kg, vg, H, dn_pad=pad, dn_group=grp, fp16=fp16, dropout_p=p, seed=seed)
    out.backward(do.to(dev))
    torch.cuda.synchronize()
    tol = 2e-3 if fp16 else 2e-5
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() < tol
    for got, want, name in ((qg.grad, qd.grad, "dq"), (kg.grad, kd.grad, "dk"), (vg.grad, vd.grad, "dv")):
        err = (got.cpu().double() - want).abs().max().item() / max(want.abs().max().item(), 1e-6)
        assert err < (5e-3 if fp16 else 2e-5), (name, err)


def test_attention_train_bwd_reuses_forward_copies(dev):
    """ABI 25 ws_reuse: the long-key backward handed the forward's workspace reuses its f16 copies
    of Q / K / V (only dO is converted) and returns the same gradients as a backward that converts
    all four into a fresh workspace (dK / dV bit for bit, dQ up to the order of its split sums) --
    on strided K / V views (the all-layer K / V arena of the training step), two batch elements."""
    T = _T()
    B, Nq, Nk, H, C = 2, 900, 4500, 8, 256
    g = torch.Generator().manual_seed(5)
    q = torch.randn(B, Nq, C, generator=g).to(dev)
    kv = torch.randn(B, Nk, 3 * C, generator=g).to(dev)     # layer 1 of a 3-layer arena
    k, v = kv[..., C:2 * C], (kv * 0.5)[..., 2 * C:]
    do = torch.randn(B, Nq, C, generator=g).to(dev)
    o = torch.empty_like(q)
    lse = torch.empty(B * H * Nq, dtype=torch.float32, device=dev)
    kw = dict(B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(Nq * C, 32, C), k_strides=(k.stride(0), 32, k.stride(1)),
              v_strides=(v.stride(0), 32, v.stride(1)), o_strides=(Nq * C, 32, C), scale=1 / math.sqrt(32),
              fp16_inputs=True)
    ws = T.attn_train_fwd(q, k, v, o, lse, **kw)
    assert ws is not None
    outs = []
    for reuse in (False, True):
        # dK / dV take the strides of K / V: slices of arenas shaped like kv
        dkv = torch.empty(2, B, Nk, 3 * C, device=dev)
        dq, dk, dv = torch.empty_like(q), dkv[0][..., C:2 * C], dkv[1][..., 2 * C:]
        T.attn_train_bwd(q, k, v, o, lse, do, dq, dk, dv, ws=ws if reuse else None, **kw)
        outs.append((dq, dk, dv))
    torch.cuda.synchronize()
    (dq0, dk0, dv0), (dq1, dk1, dv1) = outs
    assert torch.equal(dk0, dk1) and torch.equal(dv0, dv1)
    # dQ sums its key splits with f32 atomics: equal up to their order
    assert (dq0 - dq1).abs().max().item() <= 1e-5 * dq0.abs().max().item()
    assert dq0.abs().max().item() > 0


@pytest.mark.parametrize("rows,C,G,eps", [(333, 256, 1, 1e-5), (1100, 256, 1, 1e-5), (6 * 70, 64, 6, 1e-6)])
def test_layernorm_train(dev, rows, C, G, eps):
    from projects.mmdet3d_plugin.models.utils import train_ops as O
    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, C, generator=g) * 2 + 0.5
    w = torch.randn(G * C, generator=g)
    b = torch.randn(G * C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    xd, wd, bd = (t.double().requires_grad_() for t in (x, w, b))
    R = rows // G
    ref = torch.cat([torch.nn.functional.layer_norm(xd[i * R:(i + 1) * R], (C,), wd[i * C:(i + 1) * C],
                                                    bd[i * C:(i + 1) * C], eps) for i in range(G)])
    ref.backward(dy.double())
    xg, wg, bg = (t.to(dev).requires_grad_() for t in (x, w, b))
    out = O.layer_norm(xg, wg, bg, eps) if G == 1 else O.group_layer_norm(xg.view(G, R, C), wg, bg, eps).view(rows, C)
    out.backward(dy.to(dev))
    torch.cuda.synchronize()
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() < 1e-5
    for got, want in ((xg.grad, xd.grad), (wg.grad, wd.grad), (bg.grad, bd.grad)):
        assert (got.cpu().double() - want).abs().max().item() < 1e-4 * max(1.0, want.abs().max().item())


def test_bn_relu_and_conv_weight_grad(dev):
    from projects.mmdet3d_plugin.models.utils import train_ops as O
    g = torch.Generator().manual_seed(5)
    B, H, W, Cin, Cout = 2, 9, 11, 32, 64
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.2
    bn = torch.nn.BatchNorm2d(Cout).double()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    bn.train()
    wd = w.double().requires_grad_()
    ref = torch.relu(bn(torch.nn.functional.conv2d(x.double(), wd, padding=1)))
    dy = torch.randn(ref.shape, generator=g).double()
    ref.backward(dy)
    bng = torch.nn.BatchNorm2d(Cout).to(dev)
    with torch.no_grad():
        bng.weight.copy_(bn.weight.float())
        bng.bias.copy_(bn.bias.float())
    xr = x.permute(0, 2, 3, 1).reshape(-1, Cin).contiguous().to(dev)
    wt = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).contiguous().to(dev).requires_grad_()
    y = O.bn_relu(O.conv3x3(xr, wt, (B, H, W, Cin)), bng)
    y.backward(dy.float().permute(0, 2, 3, 1).reshape(-1, Cout).to(dev))
    torch.cuda.synchronize()
    got = y.detach().cpu().view(B, H, W, Cout).permute(0, 3, 1, 2).double()
    assert (got - ref.detach()).abs().max().item() < 1e-4
    gw = wt.grad.cpu().view(Cout, 3, 3, Cin).permute(0, 3, 1, 2).double()
    assert (gw - wd.grad).abs().max().item() < 1e-3 * max(1.0, wd.grad.abs().max().item())
    assert (bng.weight.grad.cpu().double() - bn.weight.grad).abs().max().item() < 1e-3
    assert (bng.bias.grad.cpu().double() - bn.bias.grad).abs().max().item() < 1e-3
    assert (bng.running_mean.cpu().double() - bn.running_mean).abs().max().item() < 1e-5
    assert (bng.running_var.cpu().double() - bn.running_var).abs().max().item() < 1e-4


@pytest.mark.parametrize("nimg,H,W,Cin,Cout,ks", [(2, 9, 11, 36, 20, 1), (1, 40, 37, 64, 128, 3), (1, 180, 180, 8, 4, 7),
                                                   (1, 180, 180, 64, 128, 2)])   # 128 x 128 tiles, split re-chosen
def test_conv3x3_wgrad_implicit(dev, nimg, H, W, Cin, Cout, ks):
    """cmt_conv3x3_wgrad_bf16x3 (ABI 21: the im2col operand gathered inside the bf16x3 GEMM) against
    float64 conv2d's weight gradient and bitwise against the im2col matrix + cmt_gemm_bf16x3_ex at
    ksplit 1 (the same products in the same order): ragged tiles (9 Cin = 324, Cout = 20), split-K,
    a 32 400-row reduction."""
    T = _T()
    g = torch.Generator().manual_seed(H * W + Cin)
    x = torch.randn(nimg, Cin, H, W, generator=g)
    dy = torch.randn(nimg, Cout, H, W, generator=g)
    wd = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    torch.nn.functional.conv2d(x.double(), wd, padding=1).backward(dy.double())
    want = wd.grad.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)           # tap-major
    xr = x.permute(0, 2, 3, 1).reshape(-1, Cin).contiguous().to(dev)
    dyr = dy.permute(0, 2, 3, 1).reshape(-1, Cout).contiguous().to(dev)
    got = T.conv3x3_wgrad(xr, dyr, nimg, H, W, Cin, ks)
    torch.cuda.synchronize()
    rows = nimg * H * W
    err = (got.cpu().double() - want).abs().max().item()
    assert err < 2 ** -15 * math.sqrt(rows) * 4, err
    if ks == 1:
        col = T.im2col3x3(xr, nimg, H, W, Cin)
        ref = torch.empty(Cout, 9 * Cin, device=dev)
        T.gemm_ex(dyr, (1, Cout), col, (1, 9 * Cin), ref, M=Cout, N_=9 * Cin, K=rows, ldc=9 * Cin, mode="bf16x3")
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), ref.cpu())


@pytest.mark.parametrize("rows", [1000, 32400])
def test_bn_relu_train_deterministic(dev, rows):
    """BatchNorm batch statistics and parameter gradients do not depend on the arrival order of
    the row blocks: two forward + backward passes are bitwise equal at 1 000 and 32 400 rows
    (4 and 507 row blocks), and the statistics match a float64 restatement."""
    from projects.mmdet3d_plugin import native_train as NT
    g = torch.Generator().manual_seed(11)
    C = 256
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(dev)
    w = (torch.rand(C, generator=g) + 0.5).to(dev)
    b = (torch.rand(C, generator=g) - 0.5).to(dev)
    dy = torch.randn(rows, C, generator=g).to(dev)
    outs = []
    for _ in range(2):
        y, mean, rstd = NT.bn_relu_train_fwd(x, w, b)
        dx, dw, db = NT.bn_relu_train_bwd(dy, x, y, w, mean, rstd)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (y, mean, rstd, dx, dw, db)])
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    xd = x.cpu().double()
    assert (outs[0][1].double() - xd.mean(0)).abs().max().item() < 1e-5
    var = xd.var(0, unbiased=False)
    assert ((outs[0][2].double() - (var + 1e-5).rsqrt()).abs() / (var + 1e-5).rsqrt()).max().item() < 1e-5


def test_det_loss_and_match_cost(dev):
    from oracle import cmt_train_oracle as TO
    T = _T()
    g = torch.Generator().manual_seed(9)
    R, ncls, Rb = 300, 10, 40
    logits = torch.randn(R, ncls, generator=g) * 2
    labels = torch.randint(0, ncls + 1, (R,), generator=g)
    lw = torch.rand(R, generator=g)
    boxes = torch.randn(Rb, 10, generator=g)
    tg = torch.randn(Rb, 10, generator=g)
    bw = torch.rand(Rb, 10, generator=g)
    cfg = dict(gamma=2.0, alpha=0.25, cls_weight=2.0, box_weight=0.25, cls_avg=37.5, box_avg=12.0)
    ld, bd = logits.double().requires_grad_(), boxes.double().requires_grad_()
    lc = TO.focal_loss(ld, labels, lw.double(), 2.0, 0.25, 2.0, 37.5)
    lb = TO.l1_loss(bd, tg.double(), bw.double(), 0.25, 12.0)
    (lc + lb).backward()
    out, dl, db = T.det_loss(logits.to(dev), labels.int().to(dev), lw.to(dev), boxes.to(dev), tg.to(dev), bw.to(dev),
                             **cfg)
    torch.cuda.synchronize()
    assert abs(out[0].item() - lc.item()) < 1e-4 * max(1, abs(lc.item()))
    assert abs(out[1].item() - lb.item()) < 1e-4 * max(1, abs(lb.item()))
    assert (dl.cpu().double() - ld.grad).abs().max().item() < 1e-5
    assert (db.cpu().double() - bd.grad).abs().max().item() < 1e-6
    gt = torch.randn(7, 10, generator=g)
    gl = torch.randint(0, ncls, (7,), generator=g)
    cw = torch.tensor([2.0, 2.0, 1, 1, 1, 1, 1, 1, 0.2, 0.2])
    ref = TO.match_cost(logits.double(), boxes[:1].repeat(R, 1).double(), gt.double(), gl, cw.double(), 2.0, 0.25)
    got = T.match_cost(logits.to(dev), boxes[:1].repeat(R, 1).to(dev), gt.to(dev), gl.int().to(dev), cw.to(dev),
                       gamma=2.0, alpha=0.25, cls_weight=2.0, reg_weight=0.25)
    torch.cuda.synchronize()
    assert (got.cpu().double() - ref).abs().max().item() < 1e-4


def test_adamw_with_clip(dev):
    T = _T()
    g = torch.Generator().manual_seed(3)
    n = 10000
    p0 = torch.randn(n, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=0.01)
    pd = p0.to(dev)
    m, v = torch.zeros_like(pd), torch.zeros_like(pd)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g) * 3
        ref.grad = grad.clone()
        torch.nn.utils.clip_grad_norm_([ref], 35.0)
        opt.step()
        ss = torch.zeros(1, device=dev)
        gd = grad.to(dev)
        T.sumsq(gd, ss)
        T.adamw_step(pd, gd, m, v, step=step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01,
                     max_norm=35.0, sumsq_buf=ss)
    torch.cuda.synchronize()
    assert (pd.cpu() - ref.detach()).abs().max().item() < 1e-5
