"""Split-f16 ('ref' policy) kernels against float64 PyTorch references.

The reference computes every projection / MLP / conv of the head in fp32; the
'ref' policy carries each fp32 operand as an f16 pair x = hi + lo (cmt_hip.h
CMT_F16P) and multiplies in three f16 MFMA passes.  These tests hold the
split GEMM (row, implicit 3x3 conv, implicit k=3 conv1d modes; fp32, f16
head-split and pair outputs; pair residual), every producer of pair operands
and the f16 long-key cross-attention (flash-attn 0.2.2 numerics) to bounds
that an fp32 GEMM meets and a bf16 one misses by three orders of magnitude.
Every call goes through the C ABI."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
SPLIT = torch.uint16


@pytest.fixture(scope="module")
def N():
    from projects.mmdet3d_plugin import native
    native.lib()
    return native


def _pair(x):
    """fp32 [..., C] -> [..., 2, C] uint16 (the host restatement of the f16 split)."""
    hi = x.float().half()
    lo = (x.float() - hi.float()).half()
    return torch.stack([hi, lo], -2).contiguous().view(SPLIT)


def _same(a, b):
    """Bit equality of two pair tensors (16-bit words compared as int16)."""
    return torch.equal(a.cpu().view(torch.int16), b.cpu().view(torch.int16))


def _unpair(p):
    b = p.view(torch.float16).double()
    return b[..., 0, :] + b[..., 1, :]


def _tol(ref, K):
    # three f16 passes: <= ~2^-21 relative per product (2^-25 absolute below f16's normal range)
    return 3e-6 * ref.abs().max().item() + 1e-6


@pytest.mark.parametrize("M,N_,K", [(900, 256, 256), (130, 768, 512), (2000, 3072, 256), (64, 1024, 192),
                                    (24000, 256, 1024)])
def test_gemm_split_rows(N, dev, M, N_, K):
    g = torch.Generator().manual_seed(M + N_ + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N_, K, generator=g) / math.sqrt(K)
    b = torch.randn(N_, generator=g)
    R = torch.randn(M, N_, generator=g)
    ref = A.double() @ W.double().t() + b.double()
    out = torch.empty(M, N_, device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), out, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_, bias=b.to(dev))
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= _tol(ref, K), err
    # relu + fp32 residual, pair output (the next GEMM's operand) and pair residual
    ref2 = torch.relu(ref) + R.double()
    outp = torch.empty(M, 2, N_, dtype=SPLIT, device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), outp, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_, bias=b.to(dev),
           relu=True, R=_pair(R).to(dev), ldr=N_)
    err2 = (_unpair(outp.cpu()) - ref2).abs().max().item()
    # the pair output itself keeps 22 significant bits
    assert err2 <= _tol(ref2, K) + 2 ** -21 * ref2.abs().max().item(), err2
    bf = (A.bfloat16().double() @ W.bfloat16().double().t() + b.double() - ref).abs().max().item()
    print(f"split GEMM {M}x{N_}x{K}: max abs err {err:.2e} (bf16 operands: {bf:.2e})")
    assert err * 300 < bf


@pytest.mark.parametrize("wscale", [0.05, 0.005])
def test_gemm_split_small_weights(N, dev, wscale):
    """Xavier-range weights (|w| <= 0.05 for a 256-wide layer; 0.005 as a harder
    case): their f16-pair lo half is subnormal, so each weight carries the
    absolute 2^-25 of CMT_F16P (include/cmt_hip.h), not 2^-22 relative.  The
    kernel is held, element by element, to the bound that representation allows:
    sum_k |a_k| e(w_k) + e(a_k) |w_k| (+ the dropped lo*lo term and fp32
    accumulation), with e(x) = max(2^-22 |x|, 2^-25)."""
    g = torch.Generator().manual_seed(7)
    M, N_, K = 900, 256, 256
    A = torch.randn(M, K, generator=g)
    A[:, :32] *= 1e-3                       # small activations too (subnormal lo on that side)
    W = (torch.rand(N_, K, generator=g) * 2 - 1) * wscale
    ref = A.double() @ W.double().t()
    out = torch.empty(M, N_, device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), out, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_)
    err = (out.cpu().double() - ref).abs()

    def e(x):
        return torch.maximum(x.abs().double() * 2 ** -22, torch.full_like(x.double(), 2 ** -25))
    a, w = A.abs().double(), W.abs().double()
    bound = a @ e(W).t() + e(A) @ w.t() + (a @ w.t()) * (K * 2 ** -24 + 2 ** -21)
    worst = (err / bound).max().item()
    rel = (err.max() / ref.abs().max()).item()
    print(f"split GEMM, |w| <= {wscale}: max err {err.max().item():.2e} ({rel:.2e} of scale, ~2^{math.log2(rel):.1f}),"
          f" max err / representation bound {worst:.3f}")
    assert worst <= 1.0, worst


@pytest.mark.parametrize("K,ks", [(256, 4), (1024, 4), (512, 2)])
def test_gemm_split_k_into_layernorm(N, dev, K, ks):
    """Split-K pair GEMM (the decoder's out-projections / fc2 at 900 rows): ks fp32
    partial blocks, bias + residual in the first, summed by layernorm_ex(nparts)."""
    g = torch.Generator().manual_seed(K + ks)
    M, C = 900, 256
    A = torch.randn(M, K, generator=g)
    W = torch.randn(C, K, generator=g) / math.sqrt(K)
    b = torch.randn(C, generator=g)
    R = torch.randn(M, C, generator=g)
    lw, lb = torch.randn(C, generator=g), torch.randn(C, generator=g)
    t = A.double() @ W.double().t() + b.double() + R.double()
    part = torch.full((ks, M, C), float("nan"), device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), part, M=M, N=C, K=K, lda=K, ldw=K, ldc=C, bias=b.to(dev),
           R=R.to(dev), ldr=C, k_splits=ks)
    got = part.cpu().double().sum(0)
    assert (got - t).abs().max().item() <= _tol(t, K), (got - t).abs().max().item()
    # part 0 carries bias + R, the others only their K slice
    kk = K // ks
    p1 = A[:, kk:2 * kk].double() @ W[:, kk:2 * kk].double().t()
    assert (part[1].cpu().double() - p1).abs().max().item() <= _tol(p1, kk)
    y = torch.empty(M, C, device=dev)
    yl = torch.empty(M, 2, C, dtype=SPLIT, device=dev)
    N.layernorm_ex(part, lw.to(dev), lb.to(dev), rows=M, C=C, ldx=C, eps=1e-5, Y=y, ldy=C, Yl=yl, nparts=ks)
    ref = torch.nn.functional.layer_norm(t, (C,), lw.double(), lb.double(), 1e-5)
    assert (y.cpu().double() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
    assert _same(yl, _pair(y.cpu()))
    with pytest.raises(RuntimeError):   # relu does not distribute over the parts
        N.gemm(_pair(A).to(dev), _pair(W).to(dev), part, M=M, N=C, K=K, lda=K, ldw=K, ldc=C, relu=True,
               k_splits=ks)


@pytest.mark.parametrize("M,with_r", [(900, True), (900, False), (77, True)])
def test_gemm_ln_split(N, dev, M, with_r):
    """cmt_gemm_ln on f16 pairs (the split out-projection + norms[0] / norms[1]):
    LN(A W^T + b + R) to fp32 accuracy, pair Yl = pair(y) and Yp = pair(y + P)
    bit-exact against the split of the fp32 output."""
    g = torch.Generator().manual_seed(M + with_r)
    C = 256
    A = torch.randn(M, C, generator=g)
    W = torch.randn(C, C, generator=g) / 16
    b = torch.randn(C, generator=g)
    R = torch.randn(M, C, generator=g)
    P = torch.randn(M, C, generator=g)
    lw, lb = torch.randn(C, generator=g), torch.randn(C, generator=g)
    t = A.double() @ W.double().t() + b.double() + (R.double() if with_r else 0)
    ref = torch.nn.functional.layer_norm(t, (C,), lw.double(), lb.double(), 1e-5)
    y = torch.empty(M, C, device=dev)
    yl = torch.empty(M, 2, C, dtype=SPLIT, device=dev)
    yp = torch.empty(M, 2, C, dtype=SPLIT, device=dev)
    N.gemm_ln(_pair(A).to(dev), _pair(W).to(dev), M=M, K=C, lda=C, ldw=C, bias=b.to(dev),
              R=R.to(dev) if with_r else None, ldr=C if with_r else 0, ln_w=lw.to(dev), ln_b=lb.to(dev), eps=1e-5,
              Y=y, Yl=yl, Yp=yp, P=P.to(dev))
    err = (y.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * ref.abs().max().item(), err
    assert _same(yl, _pair(y.cpu()))
    assert _same(yp, _pair(y.cpu() + P))
    # the same as the split-K GEMM + layernorm_ex it replaces, to fp32 rounding
    part = torch.empty(4, M, C, device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), part, M=M, N=C, K=C, lda=C, ldw=C, ldc=C, bias=b.to(dev),
           R=R.to(dev) if with_r else None, ldr=C if with_r else 0, k_splits=4)
    y2 = torch.empty(M, C, device=dev)
    N.layernorm_ex(part, lw.to(dev), lb.to(dev), rows=M, C=C, ldx=C, eps=1e-5, Y=y2, ldy=C, nparts=4)
    assert (y.cpu() - y2.cpu()).abs().max().item() <= 1e-5 * ref.abs().max().item()


def _pair_heads(x, B, S, H):
    """fp32 [B*S, H*32] rows -> head-split f16 pairs [B][H][S][64] (hi 32 | lo 32) as uint16."""
    hi = x.float().half()
    lo = (x.float() - hi.float()).half()
    t = torch.cat([hi.view(B, S, H, 32), lo.view(B, S, H, 32)], -1)       # [B, S, H, 64]
    return t.permute(0, 2, 1, 3).contiguous().view(SPLIT)


def test_gemm_split_headsplit_pair_output(N, dev):
    """Pair C in head-split mode (the split self-attention's Q|K|V): 64 16-bit
    elements per (head, row), hi 32 then lo 32; Q|K columns from A2 (select)."""
    g = torch.Generator().manual_seed(17)
    B, S, C = 2, 450, 256
    M, N_ = B * S, 3 * C
    A = torch.randn(M, C, generator=g)
    A2 = torch.randn(M, C, generator=g)
    W = torch.randn(N_, C, generator=g) / 16
    b = torch.randn(N_, generator=g)
    ref = torch.cat([A2.double() @ W[:2 * C].double().t(), A.double() @ W[2 * C:].double().t()], 1) + b.double()
    out = torch.empty(B * N_ * S * 2, dtype=SPLIT, device=dev)
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), out, M=M, N=N_, K=C, lda=C, ldw=C, ldc=0, bias=b.to(dev),
           A2=_pair(A2).to(dev), lda2=C, a2_cols=2 * C, headsplit_rows=S)
    h = out.cpu().view(torch.float16).double().view(B, N_ // 32, S, 64)
    got = (h[..., :32] + h[..., 32:]).permute(0, 2, 1, 3).reshape(M, N_)
    assert (got - ref).abs().max().item() <= _tol(ref, C) + 2 ** -21 * ref.abs().max().item()


@pytest.mark.parametrize("B,Nq,Nk,scale", [(1, 900, 900, 1.0), (2, 77, 301, 3.0), (1, 33, 5, 1.0)])
def test_attention_pair_self(N, dev, B, Nq, Nk, scale):
    """Split-f16 attention core (CMT_F16P Q/K/V, head-split pair rows): the
    reference-numerics self-attention -- fp32 softmax(QK^T / sqrt(32)) V to
    ~2^-20 relative, f32 and pair outputs; ragged key tiles."""
    g = torch.Generator().manual_seed(Nq + Nk)
    H, C = 8, 256
    q = torch.randn(B * Nq, C, generator=g) * scale
    k = torch.randn(B * Nk, C, generator=g) * scale
    v = torch.randn(B * Nk, C, generator=g)
    qp, kp, vp = _pair_heads(q, B, Nq, H).to(dev), _pair_heads(k, B, Nk, H).to(dev), _pair_heads(v, B, Nk, H).to(dev)
    qd = q.double().view(B, Nq, H, 32).transpose(1, 2)
    kd = k.double().view(B, Nk, H, 32).transpose(1, 2)
    vd = v.double().view(B, Nk, H, 32).transpose(1, 2)
    att = torch.softmax(qd @ kd.transpose(-1, -2) / math.sqrt(32), -1)
    ref = (att @ vd).transpose(1, 2).reshape(B * Nq, C)
    qs, ks = (H * Nq * 64, Nq * 64, 64), (H * Nk * 64, Nk * 64, 64)
    o32 = torch.empty(B * Nq, C, device=dev)
    N.attention(qp, kp, vp, o32, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=qs, k_strides=ks, v_strides=ks,
                o_strides=(Nq * C, C), scale=1.0 / math.sqrt(32))
    err = (o32.cpu().double() - ref).abs().max().item()
    tol = 4e-6 * ref.abs().max().item() + 1e-6
    assert err <= tol, (err, tol)
    op = torch.empty(B * Nq, 2, C, dtype=SPLIT, device=dev)
    N.attention(qp, kp, vp, op, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=qs, k_strides=ks, v_strides=ks,
                o_strides=(Nq * C, C), scale=1.0 / math.sqrt(32))
    assert _same(op, _pair(o32.cpu()))
    b16 = torch.softmax((qd.half().double() @ kd.half().double().transpose(-1, -2)) / math.sqrt(32), -1)
    e16 = ((b16 @ vd.half().double()).transpose(1, 2).reshape(B * Nq, C) - ref).abs().max().item()
    print(f"pair self-attention B{B} {Nq}x{Nk}: max abs err {err:.2e} (f16 operands: {e16:.2e})")
    assert err * 100 < e16


def test_gemm_split_headsplit_select(N, dev):
    """Q|K columns from A2 (select), V columns from A, head-split f16 / f32 output
    with the key-norm partials (the K/V projection contract)."""
    g = torch.Generator().manual_seed(3)
    B, S, C = 2, 300, 256
    M, N_ = B * S, 4 * C
    A = torch.randn(M, C, generator=g)
    A2 = torch.randn(M, C, generator=g)
    W = torch.randn(N_, C, generator=g) / 16
    b = torch.randn(N_, generator=g)
    sel = torch.cat([A2.double() @ W[:2 * C].double().t(), A.double() @ W[2 * C:].double().t()], 1) + b.double()
    for odt in (torch.float16, torch.float32):
        out = torch.empty(B * N_ * S, dtype=odt, device=dev)
        pm = torch.empty(-(-M // 64) * (2 * C // 32), device=dev) if odt == torch.float16 else None
        N.gemm(_pair(A).to(dev), _pair(W).to(dev), out, M=M, N=N_, K=C, lda=C, ldw=C, ldc=0, bias=b.to(dev),
               A2=_pair(A2).to(dev), lda2=C, a2_cols=2 * C, headsplit_rows=S, plane_max2=pm,
               plane_max_cols=2 * C if pm is not None else 0)
        got = out.cpu().double().view(B, N_ // 32, S, 32).permute(0, 2, 1, 3).reshape(M, N_)
        if odt == torch.float16:
            # one f16 rounding of the fp32-accurate result
            assert torch.equal(got.half(), sel.half().double()) or \
                (got - sel).abs().max().item() <= 2 ** -10 * sel.abs().max().item()
            ss = (got[:, :2 * C].view(M, 2 * C // 32, 32) ** 2).sum(-1)
            nb = -(-M // 64)
            pref = torch.cat([ss, torch.zeros(nb * 64 - M, ss.shape[1], dtype=ss.dtype)], 0).view(nb, 64, -1).amax(1)
            assert torch.allclose(pm.cpu().double().view(nb, -1), pref, rtol=1e-5, atol=1e-6)
        else:
            assert (got - sel).abs().max().item() <= _tol(sel, C)


@pytest.mark.parametrize("B,Cin,H,W", [(2, 128, 29, 33), (1, 64, 150, 140), (1, 64, 120, 130), (2, 64, 131, 127)])
def test_gemm_split_conv3x3(N, dev, B, Cin, H, W):
    """Implicit 3x3 conv (shared_conv) on split operands: NCHW fp32 -> pair rows
    (cmt_nchw_to_rows) -> conv + BN-folded bias + ReLU into pair memory rows.
    Maps whose 256-row grid covers most CUs run on gemm_x3_kernel (1 or 2
    images), the others on the 128 x 128 DMA tile."""
    g = torch.Generator().manual_seed(13 + H)
    Cout = 256
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / 34
    b = torch.randn(Cout, generator=g)
    xin = torch.empty(B * H * W, 2, Cin, dtype=SPLIT, device=dev)
    N.nchw_to_rows(x.to(dev), xin, nb=B, nv=1, C=Cin, HW=H * W, ldy=Cin, rows_per_batch=H * W)
    assert _same(xin, _pair(x.permute(0, 2, 3, 1).reshape(-1, Cin)))
    wp = _pair(w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)).to(dev)
    Nk = H * W + 5
    out = torch.empty(B * Nk, 2, Cout, dtype=SPLIT, device=dev)
    N.gemm(xin, wp, out, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout, bias=b.to(dev), relu=True,
           a_mode=N.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin, c_bstride=Nk * Cout)
    ref = torch.relu(torch.nn.functional.conv2d(x.double(), w.double(), b.double(), padding=1))
    ref = ref.flatten(2).permute(0, 2, 1)
    got = _unpair(out.cpu()).view(B, Nk, Cout)[:, :H * W]
    err = (got - ref).abs().max().item()
    assert err <= _tol(ref, 9 * Cin) + 2 ** -21 * ref.abs().max().item(), err


@pytest.mark.parametrize("B,Cin,H,W,Cout,cdt", [(1, 512, 180, 180, 256, "pair"),    # configs[2] shared_conv
                                                (2, 48, 37, 41, 128, "pair"),
                                                (1, 16, 16, 16, 256, "f32"),        # one chunk, one tile
                                                (1, 32, 9, 180, 384, "pair"),       # widest row
                                                (3, 64, 1, 70, 128, "f32"),         # one image row
                                                (1, 32, 300, 1, 128, "pair")])      # one image column
def test_gemm_split_conv3x3_nchw(N, dev, B, Cin, H, W, Cout, cdt):
    """shared_conv at the reference's numerics straight from the NCHW fp32 map
    (CMT_A_CONV3X3_NCHW: per-workgroup pixel halo split once, nine taps from
    LDS, image-edge zeroing) + BN-folded bias + ReLU, into batch-strided pair
    memory rows or fp32 rows, and the second output out + P (lowp(memory + pos)),
    against float64 conv2d."""
    g = torch.Generator().manual_seed(7 + H + W)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    b = torch.randn(Cout, generator=g)
    wp = _pair(w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)).to(dev)
    Nk = H * W + 37
    out = (torch.full((B * Nk, 2, Cout), 0x7e00, dtype=torch.int16, device=dev).view(SPLIT) if cdt == "pair"
           else torch.full((B * Nk, Cout), float("nan"), device=dev))
    # second output out + P (the kept BEV position rows, the same for every image): lowp(memory + pos)
    P = torch.randn(H * W, Cout, generator=g)
    out2 = torch.full_like(out, float("nan")) if cdt != "pair" else torch.full_like(out.view(torch.int16), 0x7e00).view(SPLIT)
    N.gemm(x.to(dev), wp, out, M=H * W, N=Cout, K=9 * Cin, lda=H * W, ldw=9 * Cin, ldc=Cout, bias=b.to(dev),
           relu=True, a_mode=N.A_CONV3X3_NCHW, conv=(H, W, Cin), batch=B, a_bstride=Cin * H * W,
           c_bstride=Nk * Cout, A2=P.to(dev), lda2=Cout, c2=out2)
    ref = torch.relu(torch.nn.functional.conv2d(x.double(), w.double(), b.double(), padding=1))
    ref = ref.flatten(2).permute(0, 2, 1)
    un = (lambda t: _unpair(t.cpu())) if cdt == "pair" else (lambda t: t.cpu().double())
    o, o2 = un(out), un(out2)
    got = o.view(B, Nk, Cout)[:, :H * W]
    err = (got - ref).abs().max().item()
    tol = _tol(ref, 9 * Cin) + (2 ** -21 * ref.abs().max().item() if cdt == "pair" else 0)
    print(f"NCHW split conv B{B} {Cin}->{Cout} {H}x{W}: max abs err {err:.2e} (bound {tol:.2e})")
    assert err <= tol, err
    ref2 = ref + P.double()
    err2 = (o2.view(B, Nk, Cout)[:, :H * W] - ref2).abs().max().item()
    assert err2 <= tol + 2 ** -21 * ref2.abs().max().item(), err2
    # rows past each image's map are untouched
    assert torch.isnan(o.view(B, Nk, Cout)[:, H * W:]).all() and torch.isnan(o2.view(B, Nk, Cout)[:, H * W:]).all()


@pytest.mark.parametrize("B,Cin,H,W,Cout,dt,out", [(1, 512, 180, 180, 256, torch.float16, "lowp"),   # configs[4]
                                                   (1, 512, 180, 180, 256, torch.bfloat16, "lowp"),
                                                   (2, 48, 37, 41, 128, torch.float16, "f32"),
                                                   (1, 32, 9, 180, 384, torch.bfloat16, "lowp"),
                                                   (1, 32, 300, 1, 128, torch.float16, "lowp")])
def test_gemm_conv3x3_nchw_one_pass(N, dev, B, Cin, H, W, Cout, dt, out):
    """The 'fp16' / 'bf16' policies' shared_conv from the NCHW fp32 map (round 6): the same halo
    kernel in ONE MFMA pass on f16 / bf16 pixels and weights (fp32 accumulate), W-dtype or fp32 row
    C, the second output out + P -- against float64 conv2d of the same rounded operands."""
    g = torch.Generator().manual_seed(11 + H + W)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    b = torch.randn(Cout, generator=g)
    wl = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).to(dt).contiguous().to(dev)
    Nk = H * W + 37
    cdt = dt if out == "lowp" else torch.float32
    o = torch.full((B * Nk, Cout), float("nan"), dtype=cdt, device=dev)
    P = torch.randn(H * W, Cout, generator=g)
    o2 = torch.full_like(o, float("nan"))
    N.gemm(x.to(dev), wl, o, M=H * W, N=Cout, K=9 * Cin, lda=H * W, ldw=9 * Cin, ldc=Cout, bias=b.to(dev),
           relu=True, a_mode=N.A_CONV3X3_NCHW, conv=(H, W, Cin), batch=B, a_bstride=Cin * H * W,
           c_bstride=Nk * Cout, A2=P.to(dev), lda2=Cout, c2=o2)
    xr, wr = x.to(dt).double(), w.to(dt).double()
    ref = torch.relu(torch.nn.functional.conv2d(xr, wr, b.double(), padding=1)).flatten(2).permute(0, 2, 1)
    got = o.cpu().double().view(B, Nk, Cout)[:, :H * W]
    eps = 2 ** -8 if dt == torch.bfloat16 else 2 ** -11
    scale = ref.abs().max().item()
    # fp32 accumulation order (~K 2^-24 relative) plus the output's rounding to the W dtype
    tol = (eps if out == "lowp" else 0) * scale + 9 * Cin * 2 ** -22 * scale
    err = (got - ref).abs().max().item()
    assert err <= tol, (err, tol)
    ref2 = ref + P.double()
    err2 = (o2.cpu().double().view(B, Nk, Cout)[:, :H * W] - ref2).abs().max().item()
    assert err2 <= tol + (eps if out == "lowp" else 0) * ref2.abs().max().item(), err2
    assert torch.isnan(o.cpu().float().view(B, Nk, Cout)[:, H * W:]).all()


def test_gemm_split_conv3x3_nchw_rejects(N, dev):
    x = torch.zeros(1, 16, 4, 181, device=dev)
    wp = torch.zeros(128, 2, 144, dtype=SPLIT, device=dev)
    out = torch.zeros(4 * 181, 2, 128, dtype=SPLIT, device=dev)
    with pytest.raises(RuntimeError, match="width"):
        N.gemm(x, wp, out, M=4 * 181, N=128, K=144, lda=4 * 181, ldw=144, ldc=128,
               a_mode=N.A_CONV3X3_NCHW, conv=(4, 181, 16), a_bstride=16 * 4 * 181)


@pytest.mark.parametrize("M,N_,K,batch,rdt,cdt,relu", [(30000, 256, 512, 1, "pair", "pair", False),
                                                      (12000, 256, 1024, 2, "pair", "pair", False),
                                                      (24000, 1024, 192, 1, None, "pair", True),
                                                      (20500, 384, 256, 1, "f32", "f32", True)])
def test_gemm_split_x3_epilogues(N, dev, M, N_, K, batch, rdt, cdt, relu):
    """gemm_x3_kernel (the large split GEMMs: BEV / RV position MLPs) with batch
    strides, pair or fp32 residual, ReLU, pair or fp32 output and ragged row tiles,
    against float64."""
    g = torch.Generator().manual_seed(M + K)
    A = torch.randn(batch, M, K, generator=g)
    W = torch.randn(N_, K, generator=g) / math.sqrt(K)
    b = torch.randn(N_, generator=g)
    R = torch.randn(batch, M, N_, generator=g) if rdt else None
    ref = A.double() @ W.double().t() + b.double()
    if relu:
        ref = torch.relu(ref)
    if R is not None:
        ref = ref + R.double()
    Rd = None if R is None else (_pair(R).to(dev) if rdt == "pair" else R.to(dev))
    out = (torch.empty(batch, M, 2, N_, dtype=SPLIT, device=dev) if cdt == "pair"
           else torch.empty(batch, M, N_, device=dev))
    N.gemm(_pair(A).to(dev), _pair(W).to(dev), out, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_, bias=b.to(dev),
           relu=relu, R=Rd, ldr=N_ if R is not None else 0, batch=batch, a_bstride=M * K, c_bstride=M * N_,
           r_bstride=M * N_ if R is not None else 0)
    got = _unpair(out.cpu()) if cdt == "pair" else out.cpu().double()
    err = (got - ref).abs().max().item()
    bound = _tol(ref, K) + (2 ** -21 * ref.abs().max().item() if cdt == "pair" else 0.0)
    assert err <= bound, (err, bound)


def test_gemm_split_conv1d3_grouped(N, dev):
    """The task heads' grouped k = 3 Conv1d (batched over layers) on split operands."""
    g = torch.Generator().manual_seed(12)
    L, B, Nq, C, O = 3, 2, 37, 256, 128
    x = torch.randn(L, B * Nq, C, generator=g)
    w = torch.randn(L * O, C, 3, generator=g) / 30
    wp = w.view(L, O, C, 3).permute(0, 1, 3, 2).reshape(L, O, 3 * C)
    out = torch.empty(L, B * Nq, O, device=dev)
    N.gemm(_pair(x).to(dev), _pair(wp).to(dev), out, M=B * Nq, N=O, K=3 * C, lda=C, ldw=3 * C, ldc=O, batch=L,
           a_bstride=B * Nq * C, w_bstride=O * 3 * C, c_bstride=B * Nq * O, a_mode=N.A_CONV1D3, seg_len=Nq)
    xin = x.view(L, B, Nq, C).permute(1, 0, 3, 2).reshape(B, L * C, Nq).double()
    ref = torch.nn.functional.conv1d(xin, w.double(), padding=1, groups=L)
    ref = ref.view(B, L, O, Nq).permute(1, 0, 3, 2).reshape(L, B * Nq, O)
    assert (out.cpu().double() - ref).abs().max().item() <= _tol(ref, 3 * C)


def test_split_producers(N, dev):
    """Every kernel that writes a pair operand writes exactly the host split of
    the fp32 value it writes in the fp32 policy."""
    g = torch.Generator().manual_seed(9)
    rows, C = 301, 256
    x = torch.randn(rows, C, generator=g) * 2
    w, b = torch.randn(C, generator=g), torch.randn(C, generator=g)
    P = torch.randn(rows, C, generator=g)
    xd, Pd = x.to(dev), P.to(dev)
    Y = torch.empty(rows, C, device=dev)
    Yl = torch.empty(rows, 2, C, dtype=SPLIT, device=dev)
    Yp = torch.empty_like(Yl)
    N.layernorm_ex(xd, w.to(dev), b.to(dev), rows=rows, C=C, ldx=C, Y=Y, ldy=C, Yl=Yl, Yp=Yp, P=Pd)
    y = Y.cpu()
    assert _same(Yl, _pair(y))
    assert _same(Yp, _pair(y + P))
    Zl, Zp = torch.empty_like(Yl), torch.empty_like(Yp)
    N.add_cast(Y, rows=rows, C=C, Yl=Zl, Yp=Zp, P=Pd)
    assert _same(Zl, Yl) and _same(Zp, Yp)
    assert _same(N.split_rows(xd), _pair(x))
    # pos2embed (BEV grid and reference points)
    pos = torch.rand(1000, 3, device=dev)
    o32 = torch.empty(1000, 512, device=dev)
    op = torch.empty(1000, 2, 512, dtype=SPLIT, device=dev)
    for o in (o32, op):
        N.pos2embed(pos, o, n=1000, F=256, mode=1, pos_stride=3)
    assert _same(op, _pair(o32.cpu()))
    # rv_pe coordinates
    i2l = torch.randn(3, 4, 4, device=dev)
    r32 = torch.empty(3 * 8 * 10, 192, device=dev)
    rp = torch.empty(3 * 8 * 10, 2, 192, dtype=SPLIT, device=dev)
    for o in (r32, rp):
        N.rv_pe_coords(i2l, o, BV=3, h=8, w=10, D=64, pad_h=128.0, pad_w=320.0, depth_max=61.2,
                       pc_range=[-61.2, -61.2, -10.0, 61.2, 61.2, 10.0])
    assert _same(rp, _pair(r32.cpu()))
    # rv query coordinates + masked view sum (with the decoder's first operands)
    B, V, Nq, D = 1, 2, 50, 64
    ref = torch.rand(B, Nq, 3, device=dev)
    l2i = torch.randn(B, V, 4, 4, device=dev) * 100
    i2lq = torch.randn(B, V, 4, 4, device=dev)
    q32 = torch.empty(B * V * Nq, 3 * D, device=dev)
    qp = torch.empty(B * V * Nq, 2, 3 * D, dtype=SPLIT, device=dev)
    m32 = torch.empty(B * V * Nq, device=dev)
    mp = torch.empty_like(m32)
    N.rv_query_coords(ref, l2i, i2lq, q32, m32, B=B, V=V, Nq=Nq, D=D, pad_h=640.0, pad_w=1600.0,
                      pc_range=[-54.0, -54.0, -5.0, 54.0, 54.0, 3.0])
    N.rv_query_coords_lowp(ref, l2i, i2lq, qp, mp, B=B, V=V, Nq=Nq, D=D, pad_h=640.0, pad_w=1600.0,
                           pc_range=[-54.0, -54.0, -5.0, 54.0, 54.0, 3.0])
    assert _same(qp, _pair(q32.cpu())) and torch.equal(mp, m32)
    X = torch.randn(B * V * Nq, C, device=dev)
    base = torch.randn(Nq, C, device=dev)
    Yq = torch.empty(B * Nq, C, device=dev)
    Ql, Qp = torch.empty(B * Nq, 2, C, dtype=SPLIT, device=dev), torch.empty(B * Nq, 2, C, dtype=SPLIT, device=dev)
    N.masked_view_sum(X, m32, Yq, B=B, V=V, Nq=Nq, C=C, base=base, Yl=Ql, Yp=Qp)
    assert _same(Qp, _pair(Yq.cpu()))
    assert (_unpair(Ql.cpu()) == 0).all()


def _attn_ref16(q, k, v, scale):
    """flash-attn 0.2.2's f16 core (oracle.flash_core_fp16): f16 q/k/v, f32
    scores and row statistics, P rounded to f16, f16 output -- in float64."""
    s = (q.double() @ k.double().transpose(-1, -2)) * scale
    p = torch.exp(s - s.amax(-1, keepdim=True))
    return ((p.half().double() @ v.double()) / p.sum(-1, keepdim=True)).half().double()


def _kmax2(k, B, Nk, H):
    ss = (k.double().permute(0, 2, 1, 3).reshape(B * Nk, H, 32) ** 2).sum(-1)
    nb = -(-B * Nk // 64)
    return torch.cat([ss, torch.zeros(nb * 64 - B * Nk, H, dtype=ss.dtype)], 0).view(nb, 64, H).amax(1).float()


@pytest.mark.parametrize("B,Nq,Nk,splits,mode", [(1, 900, 56400, 0, "rand"), (2, 300, 4097, 3, "rand"),
                                                 (1, 257, 8192, 1, "rand"), (1, 900, 32400, 0, "loose"),
                                                 (1, 300, 8192, 1, "loose"), (1, 900, 4160, 5, "scaled")])
def test_attention_f16_long(N, dev, B, Nq, Nk, splits, mode):
    """f16 long-key kernel (the 'ref' policy's cross-attention): bounded offsets
    from the K norm partials, the loose-bound redo (one key of huge norm
    orthogonal to every query: its bound puts every P of the split below
    f16's normal range, so the workgroup reruns that split on the online max),
    the online max alone (no partials), q * scale kept as hi + lo (QS) or q
    unscaled with the scale applied to the fp32 scores (US,
    CMT_ATTN_UNSCALED_Q), and the scale fold.  Held to the f16 core's own
    output rounding."""
    H = 8
    g = torch.Generator().manual_seed(Nk + Nq)
    sq = 3.0 if mode == "scaled" else 1.0
    q = (torch.randn(B, H, Nq, 32, generator=g) * sq).half()
    k = torch.randn(B, H, Nk, 32, generator=g).half()
    v = torch.randn(B, H, Nk, 32, generator=g).half()
    if mode == "loose":
        q[..., 0] = 0
        k[:, :, Nk // 2] = 0
        k[:, :, Nk // 2, 0] = 500.0
    ref = _attn_ref16(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
    km = _kmax2(k, B, Nk, H).to(dev)
    qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
    outs = {}
    for name, kmax2, fold, fl in (("bounded", km, False, 0), ("online", None, False, 0), ("fold", km, True, 0),
                                  ("bounded_us", km, False, 1024), ("online_us", None, False, 1024)):
        O = torch.full((B, Nq, H * 32), float("nan"), device=dev)
        N.attention(qd, kd, vd, O, B=B, H=H, Nq=Nq, Nk=Nk,
                    q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                    v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32),
                    kv_splits=splits, round_output=True, fold_scale=fold, kmax2=kmax2, kmax_ld=H if kmax2 is not None
                    else 0, kmax_plane0=0, _diag_flags=fl)
        torch.cuda.synchronize()
        got = O.cpu().double()
        assert torch.isfinite(got).all(), name
        outs[name] = got
    # an f16 output ulp either way (P rounded at another offset moves O across a rounding boundary;
    # 2^-9 |x| covers one ulp of the larger neighbour at a binade boundary), plus the f16 rounding of
    # the dominant P itself when a few keys carry the row (scaled q): 2^-11 of the largest |v|
    tol = 2 ** -9 * ref.abs().clamp(min=2 ** -4) + 2 ** -11 * v.double().abs().max().item()
    for name in ("bounded", "online", "bounded_us", "online_us"):
        d = (outs[name] - ref).abs()
        assert (d <= tol).all(), (name, d.max().item())
    # the fold permission rounds q*c once to f16: a slightly larger deviation, still small
    assert (outs["fold"] - ref).abs().max().item() < 2e-2


def test_attention_pair_output(N, dev):
    """Attention output written as the split f16 operand of the out-projection:
    exactly the split of the f32 output (f16-rounded values are exact as hi + lo)."""
    g = torch.Generator().manual_seed(21)
    B, H, Nq, Nk = 1, 8, 300, 5000
    q, k, v = (torch.randn(B, H, n, 32, generator=g).half().to(dev) for n in (Nq, Nk, Nk))
    O32 = torch.empty(B, Nq, H * 32, device=dev)
    Op = torch.empty(B * Nq, 2, H * 32, dtype=SPLIT, device=dev)
    for O in (O32, Op):
        N.attention(q, k, v, O, B=B, H=H, Nq=Nq, Nk=Nk,
                    q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                    v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=32 ** -0.5,
                    round_output=True)
    assert _same(Op, _pair(O32.cpu().view(B * Nq, H * 32)))
    assert torch.equal(_unpair(Op.cpu()), O32.cpu().double().view(B * Nq, H * 32))


@pytest.mark.parametrize("B,S", [(1, 32400), (2, 4100), (1, 100), (1, 56400)])
def test_kvproj_split(N, dev, B, S):
    """cmt_kv_proj's split f16 form (K columns from lowp(mem + pos), V columns
    from lowp(mem); all layers in one launch) against float64, with the key-norm
    partials of the K planes; ragged last row tile.  56 400 tokens (the fusion
    frame: 441 token tiles) takes the doubled column parts (4 per tile)."""
    g = torch.Generator().manual_seed(B * S)
    C, L = 256, 2
    M, N_ = B * S, 2 * L * C
    A = torch.randn(M, C, generator=g)
    A2 = torch.randn(M, C, generator=g)
    W = torch.randn(N_, C, generator=g) / 16
    b = torch.randn(N_, generator=g)
    ref = torch.cat([A2.double() @ W[:N_ // 2].double().t(), A.double() @ W[N_ // 2:].double().t()], 1) + b.double()
    Wp = _pair(W)
    wb = Wp.view(torch.float16)
    packed = torch.cat([N.kv_pack(wb[:, 0].contiguous()), N.kv_pack(wb[:, 1].contiguous())]).view(SPLIT).to(dev)
    out = torch.empty(B * N_ * S, dtype=torch.float16, device=dev)
    pm = torch.empty(-(-M // 64) * (N_ // 2 // 32), device=dev)
    N.kv_proj(_pair(A).to(dev), packed, out, M=M, N=N_, bias=b.to(dev), A2=_pair(A2).to(dev), headsplit_rows=S,
              plane_max2=pm, plane_max_cols=N_ // 2)
    got = out.cpu().double().view(B, N_ // 32, S, 32).permute(0, 2, 1, 3).reshape(M, N_)
    # one f16 rounding of the fp32-accurate product
    assert ((got - ref).abs() <= 2 ** -11 * ref.abs() + 1e-4).all(), (got - ref).abs().max().item()
    ss = (got[:, :N_ // 2].view(M, N_ // 64, 32) ** 2).sum(-1)
    nb = -(-M // 64)
    pref = torch.cat([ss, torch.zeros(nb * 64 - M, ss.shape[1], dtype=ss.dtype)], 0).view(nb, 64, -1).amax(1)
    assert torch.allclose(pm.cpu().double().view(nb, -1), pref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("form", ["split", "bf16"])
@pytest.mark.parametrize("B,S", [(2, 4100), (1, 1000)])
def test_kvproj_per_layer_equals_all_layers(N, dev, form, B, S):
    """One cmt_kv_proj launch per layer (c_offset at the layer's K plane,
    c_bstride = the whole [L][K|V][H] buffer per batch element, the decoder's
    K/V-stream schedule) writes the same K/V values and key-norm maxima bit for
    bit as the all-layer launch, into the per-layer layout [B][L][K|V][H][S][32]."""
    g = torch.Generator().manual_seed(7 * B + S)
    C, L, H = 256, 3, 8
    M = B * S
    A = torch.randn(M, C, generator=g)
    A2 = torch.randn(M, C, generator=g)
    Wk = [torch.randn(C, C, generator=g) / 16 for _ in range(L)]
    Wv = [torch.randn(C, C, generator=g) / 16 for _ in range(L)]
    bk = [torch.randn(C, generator=g) for _ in range(L)]
    bv = [torch.randn(C, generator=g) for _ in range(L)]
    if form == "split":
        op = lambda x: _pair(x).to(dev)   # noqa: E731

        def pack(w):
            wb = _pair(w).view(torch.float16)
            return torch.cat([N.kv_pack(wb[:, 0].contiguous()), N.kv_pack(wb[:, 1].contiguous())]).view(SPLIT).to(dev)
        cdt = torch.float16
    else:
        op = lambda x: x.to(torch.bfloat16).to(dev)   # noqa: E731
        pack = lambda w: N.kv_pack(w.to(torch.bfloat16)).to(dev)   # noqa: E731
        cdt = torch.bfloat16
    a, a2 = op(A), op(A2)
    E = -(-M // 64)
    full = torch.empty(B * 2 * L * C * S, dtype=cdt, device=dev)
    pm_full = torch.empty(E, L * H, device=dev)
    N.kv_proj(a, pack(torch.cat(Wk + Wv)), full, M=M, N=2 * L * C, bias=torch.cat(bk + bv).to(dev), A2=a2,
              headsplit_rows=S, plane_max2=pm_full, plane_max_cols=L * C)
    per = torch.full((B * 2 * L * C * S,), float("nan"), dtype=cdt, device=dev)
    pm_per = torch.empty(L, E, H, device=dev)
    for l in range(L):
        N.kv_proj(a, pack(torch.cat([Wk[l], Wv[l]])), per, M=M, N=2 * C, bias=torch.cat([bk[l], bv[l]]).to(dev),
                  A2=a2, headsplit_rows=S, plane_max2=pm_per[l], plane_max_cols=C, c_offset=2 * l * C * S,
                  c_bstride=2 * L * C * S)
    torch.cuda.synchronize()
    f = full.cpu().view(torch.int16).view(B, 2, L, H, S, 32)        # [b][K|V][layer][head]
    p = per.cpu().view(torch.int16).view(B, L, 2, H, S, 32)         # [b][layer][K|V][head]
    assert torch.equal(f.permute(0, 2, 1, 3, 4, 5), p)
    assert torch.equal(pm_full.cpu().view(E, L, H).permute(1, 0, 2), pm_per.cpu())
