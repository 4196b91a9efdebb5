"""Kernel-level numerics of libcmt_hip.so against plain PyTorch (CPU, fp64 /
fp32) references of the same op, on seeded inputs including ragged edges.
Every call goes through the C ABI (ctypes) -- no torch compute on the device."""
import ctypes
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from projects.mmdet3d_plugin import native
    native.lib()
    return native


def _rt(x, dt):
    return x.to(dt).to(torch.float64)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N_,K", [(900, 256, 256), (130, 768, 512), (2000, 3072, 256), (64, 1024, 192)])
def test_gemm_plain(N, dev, dt, M, N_, K):
    g = torch.Generator().manual_seed(M + N_ + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N_, K, generator=g) / math.sqrt(K)
    b = torch.randn(N_, generator=g)
    R = torch.randn(M, N_, generator=g)
    C = torch.empty(M, N_, device=dev)
    N.gemm(A.to(dev), W.to(dt).to(dev), C, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_, bias=b.to(dev), relu=True,
           R=R.to(dev), ldr=N_)
    ref = torch.relu(_rt(A, dt) @ _rt(W, dt).T + b.double()) + R.double()
    err = (C.cpu().double() - ref).abs().max().item()
    tol = 1e-4 if dt == torch.float32 else 5e-3
    assert err < tol, err


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_pos_add_headsplit(N, dev, dt):
    g = torch.Generator().manual_seed(3)
    B, S, C, K = 2, 300, 768, 256
    A = torch.randn(B * S, K, generator=g)
    A2 = torch.randn(B * S, K, generator=g)
    W = torch.randn(C, K, generator=g) / 16
    bias = torch.randn(C, generator=g)
    out_dt = torch.float16 if dt == torch.float32 else torch.bfloat16
    Y = torch.empty(B * 3 * 256 * S, dtype=out_dt, device=dev)
    N.gemm(A.to(dev), W.to(dt).to(dev), Y, M=B * S, N=C, K=K, lda=K, ldw=K, ldc=0, bias=bias.to(dev),
           A2=A2.to(dev), lda2=K, a2_cols=512, headsplit_rows=S)
    Aeff = torch.cat([A + A2, A], 0)
    full = (_rt(Aeff.float(), dt) @ _rt(W, dt).T + bias.double())
    ref_qk = full[:B * S, :512]
    ref_v = full[B * S:, 512:]
    ref = torch.cat([ref_qk, ref_v], 1).view(B, S, 24, 32).permute(0, 2, 1, 3).reshape(-1)
    got = Y.cpu().double()
    rel = (got - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_conv3x3(N, dev, dt):
    g = torch.Generator().manual_seed(5)
    B, Cin, H, W, Cout = 2, 64, 13, 17, 128
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / 24
    b = torch.randn(Cout, generator=g)
    xin = torch.empty(B * H * W, Cin, dtype=dt if dt != torch.float32 else torch.float32, device=dev)
    N.nchw_to_rows(x.to(dev), xin, nb=B, nv=1, C=Cin, HW=H * W, ldy=Cin, rows_per_batch=H * W)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).to(dt).to(dev).contiguous()
    Nk = H * W + 5   # rows per batch in the destination (leaves a gap, as in the fusion memory)
    out = torch.full((B * Nk, Cout), float("nan"), device=dev)
    N.gemm(xin, wp, out, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout, bias=b.to(dev), relu=True,
           a_mode=N.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin, c_bstride=Nk * Cout)
    ref = torch.relu(torch.nn.functional.conv2d(_rt(x, dt), _rt(w, dt), b.double(), padding=1))
    ref = ref.flatten(2).permute(0, 2, 1)
    got = out.view(B, Nk, Cout)[:, :H * W].cpu().double()
    tol = 1e-4 if dt == torch.float32 else 5e-3
    assert (got - ref).abs().max().item() < tol
    assert torch.isnan(out.view(B, Nk, Cout)[:, H * W:]).all(), "conv wrote outside its rows"


def test_gemm_conv1d3_grouped(N, dev):
    g = torch.Generator().manual_seed(6)
    L, B, Nq, C, O = 3, 2, 37, 256, 128
    x = torch.randn(L, B * Nq, C, generator=g)
    w = torch.randn(L * O, C, 3, generator=g) / 30
    wp = w.view(L, O, C, 3).permute(0, 1, 3, 2).reshape(L, O, 3 * C).contiguous()
    out = torch.empty(L, B * Nq, O, device=dev)
    N.gemm(x.to(dev), wp.to(dev), out, M=B * Nq, N=O, K=3 * C, lda=C, ldw=3 * C, ldc=O, batch=L,
           a_bstride=B * Nq * C, w_bstride=O * 3 * C, c_bstride=B * Nq * O, a_mode=N.A_CONV1D3, seg_len=Nq)
    xin = x.view(L, B, Nq, C).permute(1, 0, 3, 2).reshape(B, L * C, Nq).double()
    ref = torch.nn.functional.conv1d(xin, w.double(), padding=1, groups=L)        # [B, L*O, Nq]
    ref = ref.view(B, L, O, Nq).permute(1, 0, 3, 2).reshape(L, B * Nq, O)
    assert (out.cpu().double() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N_,K,r_lowp,out_lowp", [(900, 256, 256, False, False), (130, 768, 512, True, True),
                                                    (8200, 1024, 256, True, False), (64, 1024, 192, False, True),
                                                    (900, 256, 1024, False, False)])
def test_gemm_dma_lowp_a(N, dev, dt, M, N_, K, r_lowp, out_lowp):
    """A already in the compute dtype: the LDS-DMA kernel (both tile shapes,
    ragged M, bf16/fp32 residual and output)."""
    g = torch.Generator().manual_seed(M * 7 + N_ + K)
    A = torch.randn(M, K, generator=g).to(dt)
    W = (torch.randn(N_, K, generator=g) / math.sqrt(K)).to(dt)
    b = torch.randn(N_, generator=g)
    R = torch.randn(M, N_, generator=g)
    if r_lowp:
        R = R.to(dt)
    C = torch.empty(M, N_, device=dev, dtype=dt if out_lowp else torch.float32)
    N.gemm(A.to(dev), W.to(dev), C, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_, bias=b.to(dev), relu=True,
           R=R.to(dev), ldr=N_)
    ref = torch.relu(A.double() @ W.double().T + b.double()) + R.double()
    err = (C.cpu().double() - ref).abs().max().item()
    tol = 5e-3 + (ref.abs().max().item() * (2 ** -7 if out_lowp else 0))
    assert err < tol, err


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_gemm_dma_select_headsplit(N, dev, dt):
    """A2 select mode: columns < a2_cols read A2 (e.g. LN(x)+pos written by the
    LN kernel), the rest read A; head-split [B][N/32][S][32] output."""
    g = torch.Generator().manual_seed(11)
    B, S, C, K = 2, 300, 768, 256
    A = torch.randn(B * S, K, generator=g).to(dt)
    A2 = torch.randn(B * S, K, generator=g).to(dt)
    W = (torch.randn(C, K, generator=g) / 16).to(dt)
    bias = torch.randn(C, generator=g)
    Y = torch.empty(B * C * S, dtype=dt, device=dev)
    N.gemm(A.to(dev), W.to(dev), Y, M=B * S, N=C, K=K, lda=K, ldw=K, ldc=0, bias=bias.to(dev),
           A2=A2.to(dev), lda2=K, a2_cols=512, headsplit_rows=S)
    qk = A2.double() @ W.double()[:512].T + bias.double()[:512]
    v = A.double() @ W.double()[512:].T + bias.double()[512:]
    ref = torch.cat([qk, v], 1).view(B, S, 24, 32).permute(0, 2, 1, 3).reshape(-1)
    got = Y.cpu().double()
    rel = (got - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,S,big", [(2, 300, False), (1, 32400, True), (2, 4100, True)])
def test_gemm_plane_max2(N, dev, dt, B, S, big):
    """Head-split GEMM epilogue by-product: per 64-row block and head plane the
    max squared row norm of the stored (rounded) values, planes < plane_max_cols
    (the K half of a K|V projection); 64x64 and 128x128 tiles, ragged M,
    blocks straddling the batch boundary."""
    g = torch.Generator().manual_seed(S + B)
    K, Nc = 256, (3072 if big else 512)
    M = B * S
    A = torch.randn(M, K, generator=g).to(dt)
    W = (torch.randn(Nc, K, generator=g) / 16).to(dt)
    Y = torch.empty(M * Nc, dtype=dt, device=dev)
    cols = Nc // 2
    nb = -(-M // 64)
    pm = torch.full((nb, cols // 32), -1.0, device=dev)
    N.gemm(A.to(dev), W.to(dev), Y, M=M, N=Nc, K=K, lda=K, ldw=K, ldc=0, headsplit_rows=S, plane_max2=pm,
           plane_max_cols=cols)
    y = Y.cpu().view(B, Nc // 32, S, 32).permute(0, 2, 1, 3).reshape(M, Nc // 32, 32).double()
    ss = (y[:, :cols // 32] ** 2).sum(-1)                       # [M, planes]
    pad = nb * 64 - M
    ref = torch.cat([ss, torch.zeros(pad, cols // 32, dtype=ss.dtype)], 0).view(nb, 64, -1).amax(1)
    assert torch.allclose(pm.cpu().double(), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("with_a2", [True, False])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,S", [(1, 32400), (2, 4100), (1, 100)])
def test_kvproj_select_plane_max(N, dev, dt, B, S, with_a2):
    """All-layer K/V projection shape (N = 3072, K = 256, A2 select on the K half,
    head-split output, K-half key-norm maxima) through cmt_kv_proj, the
    A-stationary kernel on fragment-packed W (kvproj.hip); ragged M, row tiles
    straddling the batch boundary, a grid smaller than one 128-row tile pair;
    without A2 a single column part (N = 1536) reads A only."""
    g = torch.Generator().manual_seed(S * 7 + B)
    K, Nc = 256, 3072 if with_a2 else 1536
    M, cols = B * S, Nc // 2 if with_a2 else Nc
    A = torch.randn(M, K, generator=g).to(dt)
    A2 = torch.randn(M, K, generator=g).to(dt) if with_a2 else A
    W = (torch.randn(Nc, K, generator=g) / 16).to(dt)
    bias = torch.randn(Nc, generator=g) * 0.1
    Y = torch.empty(M * Nc, dtype=dt, device=dev)
    nb = -(-M // 64)
    pm = torch.full((nb, cols // 32), -1.0, device=dev)
    N.kv_proj(A.to(dev), N.kv_pack(W.to(dev)), Y, M=M, N=Nc, bias=bias.to(dev),
              A2=A2.to(dev) if with_a2 else None, headsplit_rows=S, plane_max2=pm, plane_max_cols=cols)
    d = lambda t: t.double()
    ref = torch.cat([d(A2) @ d(W[:Nc // 2]).T, d(A) @ d(W[Nc // 2:]).T], 1) + d(bias)
    y = Y.cpu().view(B, Nc // 32, S, 32).permute(0, 2, 1, 3).reshape(M, Nc).double()
    rel = (y - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 1e-2, rel
    ss = (y[:, :cols].view(M, cols // 32, 32) ** 2).sum(-1)
    pad = nb * 64 - M
    pref = torch.cat([ss, torch.zeros(pad, cols // 32, dtype=ss.dtype)], 0).view(nb, 64, -1).amax(1)
    assert torch.allclose(pm.cpu().double(), pref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("scale_q", [1.0, 40.0])
@pytest.mark.parametrize("B,Nq,Nk,splits", [(1, 900, 32400, 0), (2, 300, 4097, 3), (1, 257, 8192, 1)])
def test_attention_bounded_max(N, dev, B, Nq, Nk, splits, scale_q):
    """bf16 long-key kernel with the K max-norm partials: every query's softmax
    offset is the Cauchy-Schwarz bound (scale_q = 1); with large |q| (40) the
    bound exceeds 60 exp2 units and the waves fall back to the running max
    (there without the scale fold: rounding q*scale*log2e to bf16 moves scores
    of ~100 exp2 units by ~0.2, beyond any tolerance of this check)."""
    H = 8
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(Nk + B)
    q = (torch.randn(B, H, Nq, 32, generator=g) * scale_q).to(dt)
    k = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    k[:, :, Nk // 3] *= 3                                       # one long key per plane
    v = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    kr = k.double().permute(0, 2, 1, 3).reshape(B * Nk, H, 32)
    ss = (kr ** 2).sum(-1)
    nb = -(-B * Nk // 64)
    km = torch.cat([ss, torch.zeros(nb * 64 - B * Nk, H, dtype=ss.dtype)], 0).view(nb, 64, H).amax(1)
    kmax2 = torch.cat([torch.zeros(nb, 3), km.float(), torch.zeros(nb, 5)], 1).contiguous()   # planes 3..10
    for fold in ((False, True) if scale_q == 1.0 else (False,)):
        O = torch.empty(B, Nq, H * 32, device=dev)
        N.attention(q.to(dev), k.to(dev), v.to(dev), O, B=B, H=H, Nq=Nq, Nk=Nk,
                    q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                    v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32),
                    kv_splits=splits, fold_scale=fold, kmax2=kmax2.to(dev), kmax_ld=16, kmax_plane0=3)
        ref = _attn_ref(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
        got = O.cpu().double()
        assert torch.isfinite(got).all()
        err = (got - ref).abs().max().item()
        assert err < 2e-2, (fold, err)


@pytest.mark.parametrize("B,Nq,Nk,splits,scale_q", [(1, 900, 56400, 0, 1.0), (2, 300, 4097, 3, 1.0),
                                                    (1, 257, 8192, 1, 1.0), (1, 900, 4160, 5, 1.0),
                                                    (1, 900, 32400, 0, 12.0)])
def test_attention_pb2_bounded_matches_online(N, dev, B, Nq, Nk, splits, scale_q):
    """bf16 long-key kernel (128 keys per ping-pong window): the offset-free
    bounded path (K norm partials) against the online-max path (no partials)
    on the same inputs, odd full-tile counts per split, a ragged last tile and
    1-5 splits; with large |q| every wave of the bounded launch falls back to
    the online max (bound > 60 exp2 units) and the two launches agree exactly."""
    H = 8
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(Nk + Nq)
    q = (torch.randn(B, H, Nq, 32, generator=g) * scale_q).to(dt).to(dev)
    k = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    v = torch.randn(B, H, Nk, 32, generator=g).to(dt).to(dev)
    ss = (k.double().permute(0, 2, 1, 3).reshape(B * Nk, H, 32) ** 2).sum(-1)
    nb = -(-B * Nk // 64)
    km = torch.cat([ss, torch.zeros(nb * 64 - B * Nk, H, dtype=ss.dtype)], 0).view(nb, 64, H).amax(1)
    kmax2 = km.float().contiguous().to(dev)
    k = k.to(dev)
    outs = []
    for km2 in (kmax2, None):
        O = torch.empty(B, Nq, H * 32, device=dev)
        N.attention(q, k, v, O, B=B, H=H, Nq=Nq, Nk=Nk,
                    q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                    v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32),
                    kv_splits=splits, fold_scale=True, kmax2=km2, kmax_ld=H if km2 is not None else 0,
                    kmax_plane0=0)
        torch.cuda.synchronize()
        outs.append(O.cpu())
    assert torch.isfinite(outs[0]).all() and torch.isfinite(outs[1]).all()
    if scale_q == 1.0:
        # P at another offset: bf16 rounding of P differs, O agrees to bf16 precision
        assert (outs[0] - outs[1]).abs().max().item() < 2e-2
    else:
        assert torch.equal(outs[0], outs[1])
    if scale_q == 1.0:
        # (with |q| x 12 the bf16 rounding of the folded q * scale * log2 e alone moves scores of ~100
        # exp2 units by ~0.2: the two launches agree exactly, the float64 check holds at scale 1)
        ref = _attn_ref(q.cpu(), k.cpu(), v.cpu(), 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
        assert (outs[0].double() - ref).abs().max().item() < 2e-2


def test_gemm_dma_conv1d3_lowp(N, dev):
    g = torch.Generator().manual_seed(12)
    L, B, Nq, C, O = 3, 2, 37, 256, 128
    x = torch.randn(L, B * Nq, C, generator=g).bfloat16()
    w = (torch.randn(L * O, C, 3, generator=g) / 30).bfloat16()
    wp = w.view(L, O, C, 3).permute(0, 1, 3, 2).reshape(L, O, 3 * C).contiguous()
    out = torch.empty(L, B * Nq, O, device=dev)
    N.gemm(x.to(dev), wp.to(dev), out, M=B * Nq, N=O, K=3 * C, lda=C, ldw=3 * C, ldc=O, batch=L,
           a_bstride=B * Nq * C, w_bstride=O * 3 * C, c_bstride=B * Nq * O, a_mode=N.A_CONV1D3, seg_len=Nq)
    xin = x.view(L, B, Nq, C).permute(1, 0, 3, 2).reshape(B, L * C, Nq).double()
    ref = torch.nn.functional.conv1d(xin, w.double(), padding=1, groups=L)
    ref = ref.view(B, L, O, Nq).permute(1, 0, 3, 2).reshape(L, B * Nq, O)
    assert (out.cpu().double() - ref).abs().max().item() < 1e-3


def test_gemm_dma_conv3x3_big(N, dev):
    """Implicit 3x3 conv on the 128x128 DMA tiles (gathered rows, zero page)."""
    g = torch.Generator().manual_seed(13)
    B, Cin, H, W, Cout = 1, 128, 61, 67, 256
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / 34
    b = torch.randn(Cout, generator=g)
    xin = torch.empty(B * H * W, Cin, dtype=torch.bfloat16, device=dev)
    N.nchw_to_rows(x.to(dev), xin, nb=B, nv=1, C=Cin, HW=H * W, ldy=Cin, rows_per_batch=H * W)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).bfloat16().to(dev).contiguous()
    out = torch.empty((B * H * W, Cout), dtype=torch.bfloat16, device=dev)
    N.gemm(xin, wp, out, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout, bias=b.to(dev), relu=True,
           a_mode=N.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin, c_bstride=H * W * Cout)
    ref = torch.relu(torch.nn.functional.conv2d(_rt(x, torch.bfloat16), _rt(w, torch.bfloat16), b.double(),
                                                padding=1))
    ref = ref.flatten(2).permute(0, 2, 1).reshape(-1, Cout)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err < 1e-2 + ref.abs().max().item() * 2 ** -8, err


def test_gemm_conv3x3_8wave_batched(N, dev):
    """The 8-wave 256x128 conv kernel (bf16 in/out): two images written into a
    larger per-batch row block (the fusion memory's gap), M not a multiple of
    256, every row outside the conv's untouched."""
    g = torch.Generator().manual_seed(17)
    B, Cin, H, W, Cout = 2, 64, 19, 23, 256
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / 24
    b = torch.randn(Cout, generator=g)
    xin = torch.empty(B * H * W, Cin, dtype=torch.bfloat16, device=dev)
    N.nchw_to_rows(x.to(dev), xin, nb=B, nv=1, C=Cin, HW=H * W, ldy=Cin, rows_per_batch=H * W)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).bfloat16().to(dev).contiguous()
    Nk = H * W + 7
    out = torch.full((B * Nk, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    N.gemm(xin, wp, out, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout, bias=b.to(dev), relu=True,
           a_mode=N.A_CONV3X3, conv=(H, W, Cin), batch=B, a_bstride=H * W * Cin, c_bstride=Nk * Cout)
    ref = torch.relu(torch.nn.functional.conv2d(_rt(x, torch.bfloat16), _rt(w, torch.bfloat16), b.double(),
                                                padding=1)).flatten(2).permute(0, 2, 1)
    got = out.view(B, Nk, Cout)[:, :H * W].cpu().double()
    err = (got - ref).abs().max().item()
    assert err < 1e-2 + ref.abs().max().item() * 2 ** -8, err
    assert torch.isnan(out.view(B, Nk, Cout)[:, H * W:].float()).all(), "conv wrote outside its rows"


def _attn_ref(q, k, v, scale):
    s = (q.double() @ k.double().transpose(-1, -2)) * scale
    return torch.softmax(s, -1) @ v.double()


@pytest.mark.parametrize("fold", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,H,Nq,Nk,splits", [(1, 8, 900, 32400, 0), (2, 8, 130, 1000, 0), (1, 2, 33, 65, 1),
                                              (1, 8, 900, 900, 0), (1, 1, 1, 1, 1), (2, 3, 200, 4097, 3)])
def test_attention(N, dev, dt, B, H, Nq, Nk, splits, fold):
    if fold and dt == torch.float32:
        pytest.skip("the exact-f32 kernel never folds the scale")
    g = torch.Generator().manual_seed(B * 1000 + Nk)
    q = (torch.randn(B, H, Nq, 32, generator=g) * 1.5).to(dt)
    k = (torch.randn(B, H, Nk, 32, generator=g) * 1.5).to(dt)
    v = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    O = torch.empty(B, Nq, H * 32, device=dev)
    N.attention(q.to(dev), k.to(dev), v.to(dev), O, B=B, H=H, Nq=Nq, Nk=Nk,
                q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32),
                kv_splits=splits, fold_scale=fold)
    ref = _attn_ref(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
    err = (O.cpu().double() - ref).abs().max().item()
    tol = {torch.float32: 2e-5, torch.float16: 3e-3, torch.bfloat16: 2e-2}[dt]
    assert err < tol, err


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,H,Nq,Nk,mode", [(1, 8, 900, 900, "rand"), (2, 3, 70, 65, "rand"), (1, 1, 5, 1, "rand"),
                                            (1, 2, 40, 4096, "rand"), (1, 1, 33, 700, "spike"),
                                            (1, 2, 70, 200, "negative")])
def test_attention_key_split_workgroup(N, dev, dt, B, H, Nq, Nk, mode):
    """Short key ranges (self-attention): KW waves of one workgroup split the
    keys of the same 32 queries and merge (O, row sum, offset) through LDS.
    Fewer tiles than waves (waves without keys), a ragged last tile, 64 tiles,
    a late spike (the merge's max comes from a later wave than the first), all
    scores ~ -200 exp2 units (no underflow in the merge); both scale folds;
    against float64 and against the split-partials + combine path."""
    g = torch.Generator().manual_seed(Nk * 7 + Nq)
    if mode == "negative":
        q = (5 + 0.1 * torch.randn(B, H, Nq, 32, generator=g)).to(dt)
        k = (-5 + 0.1 * torch.randn(B, H, Nk, 32, generator=g)).to(dt)
    else:
        q = (torch.randn(B, H, Nq, 32, generator=g) * 1.5).to(dt)
        k = (torch.randn(B, H, Nk, 32, generator=g) * (0.1 if mode == "spike" else 1.5)).to(dt)
    if mode == "spike":
        k[0, 0, 650] = q[0, 0, 5] * 4            # query 5's max sits in the last (ragged) tile
    v = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    ref = _attn_ref(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
    qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
    for fold in (False, True):
        outs = []
        for splits in (0, 2):   # 0: the in-workgroup key split; 2: split partials + combine
            O = torch.full((B, Nq, H * 32), float("nan"), device=dev)
            N.attention(qd, kd, vd, O, B=B, H=H, Nq=Nq, Nk=Nk,
                        q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                        v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32),
                        scale=1 / math.sqrt(32), fold_scale=fold, kv_splits=splits)
            torch.cuda.synchronize()
            outs.append(O.cpu().double())
        assert torch.isfinite(outs[0]).all()
        err = (outs[0] - ref).abs().max().item()
        tol = {torch.float16: 3e-3, torch.bfloat16: 2e-2}[dt] * (10 if mode == "negative" else 1)
        assert err < tol, (fold, err)
        assert (outs[0] - outs[1]).abs().max().item() < tol


def test_attention_spike_rescale(N, dev):
    """Force the online-softmax running max to jump late (rule 26)."""
    B, H, Nq, Nk = 1, 1, 64, 2048
    g = torch.Generator().manual_seed(11)
    q = torch.randn(B, H, Nq, 32, generator=g).half()
    k = (torch.randn(B, H, Nk, 32, generator=g) * 0.1).half()
    k[0, 0, 1900] = q[0, 0, 5] * 4          # spike for query 5 in a late tile
    v = torch.randn(B, H, Nk, 32, generator=g).half()
    for splits, fold in ((1, False), (4, False), (1, True), (4, True)):
        O = torch.empty(B, Nq, 32, device=dev)
        N.attention(q.to(dev), k.to(dev), v.to(dev), O, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(Nq * 32, Nq * 32, 32),
                    k_strides=(Nk * 32, Nk * 32, 32), v_strides=(Nk * 32, Nk * 32, 32), o_strides=(Nq * 32, 32),
                    scale=1 / math.sqrt(32), kv_splits=splits, fold_scale=fold)
        ref = _attn_ref(q, k, v, 1 / math.sqrt(32))[0].transpose(0, 1).reshape(Nq, 32)
        assert (O.cpu().double()[0] - ref).abs().max().item() < 3e-3


@pytest.mark.parametrize("fold", [False, True])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_attention_empty_split_negative_scores(N, dev, dt, fold):
    """Nk = 200 (4 key tiles) in 3 splits of 2 tiles: the last split is empty.
    All scores ~ -140 (exp2 units ~ -200): an empty split must not enter the
    combine's maximum, or every weight underflows."""
    B, H, Nq, Nk = 1, 2, 70, 200
    g = torch.Generator().manual_seed(5)
    q = (5 + 0.1 * torch.randn(B, H, Nq, 32, generator=g)).to(dt)
    k = (-5 + 0.1 * torch.randn(B, H, Nk, 32, generator=g)).to(dt)
    v = torch.randn(B, H, Nk, 32, generator=g).to(dt)
    O = torch.empty(B, Nq, H * 32, device=dev)
    N.attention(q.to(dev), k.to(dev), v.to(dev), O, B=B, H=H, Nq=Nq, Nk=Nk,
                q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32),
                kv_splits=3, fold_scale=fold)
    ref = _attn_ref(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
    got = O.cpu().double()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 3e-2


def test_attention_seq_first_strides(N, dev):
    """sequence-first [S, B, C] layout via strides (module-level API path)."""
    B, H, S = 2, 8, 100
    C = H * 32
    g = torch.Generator().manual_seed(2)
    x = torch.randn(S, B, C, generator=g).half()
    O = torch.empty(S, B, C, device=dev)
    xd = x.to(dev)
    N.attention(xd, xd, xd, O, B=B, H=H, Nq=S, Nk=S, q_strides=(C, 32, B * C), k_strides=(C, 32, B * C),
                v_strides=(C, 32, B * C), o_strides=(C, B * C), scale=0.2)
    xb = x.permute(1, 0, 2).reshape(B, S, H, 32).permute(0, 2, 1, 3)
    ref = _attn_ref(xb, xb, xb, 0.2).permute(2, 0, 1, 3).reshape(S, B, C)
    assert (O.cpu().double() - ref).abs().max().item() < 3e-3


def test_layernorm_fused_post(N, dev):
    g = torch.Generator().manual_seed(4)
    rows, C = 333, 256
    x = torch.randn(rows, C, generator=g) * 3 + 1
    w, b = torch.randn(C, generator=g), torch.randn(C, generator=g)
    w2, b2 = torch.randn(C, generator=g), torch.randn(C, generator=g)
    prev = torch.randn(rows, C, generator=g)
    x[7, 3] = float("inf")
    Y = torch.empty(rows, C, device=dev)
    Y2 = prev.clone().to(dev)
    N.layernorm(x.to(dev), w.to(dev), b.to(dev), Y, rows=rows, C=C, ldx=C, ldy=C, W2=w2.to(dev), B2=b2.to(dev),
                Y2=Y2, ldy2=C, flags2=N.LN_NAN_TO_NUM | N.LN_MAX_INTO)
    F = torch.nn.functional
    r1 = F.layer_norm(x, (C,), w, b, 1e-5)
    r2 = torch.maximum(torch.nan_to_num(F.layer_norm(r1, (C,), w2, b2, 1e-5)), prev)
    ok = torch.isfinite(r1).all(1)
    assert (Y.cpu()[ok] - r1[ok]).abs().max().item() < 1e-4
    assert torch.isfinite(Y2.cpu()).all()
    assert (Y2.cpu()[ok] - r2[ok]).abs().max().item() < 1e-4


@pytest.mark.parametrize("lp", [torch.float16, torch.bfloat16])
def test_layernorm_ex_lowp_outputs(N, dev, lp):
    """lowp(y) and lowp(y + P) written beside the fp32 output (decoder operands)."""
    g = torch.Generator().manual_seed(9)
    rows, C = 301, 256
    x = torch.randn(rows, C, generator=g) * 2
    w, b = torch.randn(C, generator=g), torch.randn(C, generator=g)
    P = torch.randn(rows, C, generator=g)
    Y = torch.empty(rows, C, device=dev)
    Yl = torch.empty(rows, C, dtype=lp, device=dev)
    Yp = torch.empty(rows, C, dtype=lp, device=dev)
    N.layernorm_ex(x.to(dev), w.to(dev), b.to(dev), rows=rows, C=C, ldx=C, Y=Y, ldy=C, Yl=Yl, Yp=Yp, P=P.to(dev))
    r = torch.nn.functional.layer_norm(x, (C,), w, b, 1e-5)
    assert (Y.cpu() - r).abs().max().item() < 1e-4
    assert torch.equal(Yl.cpu(), Y.cpu().to(lp))
    assert torch.equal(Yp.cpu(), (Y.cpu() + P).to(lp))
    # add_cast: the first-layer operands from the initial target
    Zl = torch.empty_like(Yl)
    Zp = torch.empty_like(Yp)
    N.add_cast(Y, rows=rows, C=C, Yl=Zl, Yp=Zp, P=P.to(dev))
    assert torch.equal(Zl, Yl) and torch.equal(Zp, Yp)


@pytest.mark.parametrize("lp", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,K,r_lowp", [(900, 256, False), (133, 1024, True), (32, 256, False)])
def test_gemm_ln_matches_unfused(N, dev, lp, M, K, r_lowp):
    """cmt_gemm_ln == cmt_gemm (+bias +R) followed by cmt_layernorm_ex, for
    every LN output (Y, lowp(y), lowp(y + P), post-norm Y2 with nan_to_num and
    coop max-into)."""
    g = torch.Generator().manual_seed(M + K)
    C = 256
    A = torch.randn(M, K, generator=g).to(lp).to(dev)
    W = (torch.randn(C, K, generator=g) / math.sqrt(K)).to(lp).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    R = torch.randn(M, C, generator=g).to(dev)
    if r_lowp:
        R = R.to(lp)
    lw, lb, w2, b2 = (torch.randn(C, generator=g).to(dev) for _ in range(4))
    P = torch.randn(M, C, generator=g).to(dev)
    prev = torch.randn(M, C, generator=g).to(dev)
    # unfused reference path (both native)
    t = torch.empty(M, C, device=dev)
    N.gemm(A, W, t, M=M, N=C, K=K, lda=K, ldw=K, ldc=C, bias=bias, R=R, ldr=C)
    Y0, Yl0, Yp0 = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev, dtype=lp), torch.empty(M, C, device=dev, dtype=lp)
    Y20 = prev.clone()
    N.layernorm_ex(t, lw, lb, rows=M, C=C, ldx=C, Y=Y0, ldy=C, Yl=Yl0, Yp=Yp0, P=P, W2=w2, B2=b2, Y2=Y20, ldy2=C,
                   flags2=N.LN_NAN_TO_NUM | N.LN_MAX_INTO)
    Y1, Yl1, Yp1 = torch.empty_like(Y0), torch.empty_like(Yl0), torch.empty_like(Yp0)
    Y21 = prev.clone()
    N.gemm_ln(A, W, M=M, K=K, lda=K, ldw=K, bias=bias, R=R, ldr=C, ln_w=lw, ln_b=lb, Y=Y1, Yl=Yl1, Yp=Yp1, P=P,
              W2=w2, B2=b2, Y2=Y21, flags2=N.LN_NAN_TO_NUM | N.LN_MAX_INTO)
    assert (Y1 - Y0).abs().max().item() < 2e-4
    assert (Y21 - Y20).abs().max().item() < 2e-4
    ulp = 2 ** -7 if lp == torch.bfloat16 else 2 ** -10
    for a_, b_ in ((Yl1, Yl0), (Yp1, Yp0)):
        d = (a_.float() - b_.float()).abs()
        assert (d <= ulp * b_.float().abs().clamp(min=1.0) + 1e-4).all()


@pytest.mark.parametrize("odt", [torch.float16, torch.bfloat16])
def test_attention_lowp_output(N, dev, odt):
    g = torch.Generator().manual_seed(21)
    B, H, Nq, Nk = 1, 8, 200, 3000
    q = torch.randn(B, H, Nq, 32, generator=g)
    k = torch.randn(B, H, Nk, 32, generator=g)
    v = torch.randn(B, H, Nk, 32, generator=g)
    dt = torch.bfloat16
    O32 = torch.empty(B, Nq, H * 32, device=dev)
    Ol = torch.empty(B, Nq, H * 32, device=dev, dtype=odt)
    for O in (O32, Ol):
        N.attention(q.to(dt).to(dev), k.to(dt).to(dev), v.to(dt).to(dev), O, B=B, H=H, Nq=Nq, Nk=Nk,
                    q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                    v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32), scale=32 ** -0.5)
    assert torch.equal(Ol.cpu(), O32.cpu().to(odt))


def test_pos2embed_lowp_matches_f32(N, dev):
    pos = torch.rand(1000, 3, device=dev)
    o32 = torch.empty(1000, 512, device=dev)
    ob = torch.empty(1000, 512, device=dev, dtype=torch.bfloat16)
    N.pos2embed(pos, o32, n=1000, F=256, mode=1, pos_stride=3)
    N.pos2embed(pos, ob, n=1000, F=256, mode=1, pos_stride=3)
    assert torch.equal(ob, o32.to(torch.bfloat16))
    g32 = torch.empty(180 * 180, 512, device=dev)
    N.pos2embed(None, g32, n=180 * 180, F=256, grid=(180, 180))
    from oracle import cmt_oracle as O
    ref = O.pos2embed(O.coords_bev([1440, 1440, 40], 8), 256)
    assert (g32.cpu() - ref).abs().max().item() < 2e-5


def test_pos2embed_kat(N, dev):
    """SURVEY 8(a) row a1 KAT: (x, y) = (0.4963, 0.7682), F = 256."""
    pos = torch.tensor([[0.4963, 0.7682]], device=dev)
    out = torch.empty(1, 512, device=dev)
    N.pos2embed(pos, out, n=1, F=256)
    exp = [math.sin(2 * math.pi * 0.7682), math.cos(2 * math.pi * 0.7682),
           math.sin(2 * math.pi * 0.7682 / 1.0078125), math.cos(2 * math.pi * 0.7682 / 1.0078125)]
    assert np.allclose(out[0, :4].cpu().numpy(), exp, atol=2e-5)
    assert abs(out[0, 256].item() - math.sin(2 * math.pi * 0.4963)) < 2e-5


def test_voxelize_bitexact(N, dev):
    """Scatter-mean vs the C restatement: bit-exact voxel sets and means,
    including an overfull voxel, out-of-range points and the voxel budget."""
    import ctypes
    import os
    from conftest import ROOT
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libvoxel_oracle.so"))
    g = torch.Generator().manual_seed(9)
    pc = [-54.0, -54.0, -5.0, 54.0, 54.0, 3.0]
    vs = [0.075, 0.075, 0.2]
    grid = [1440, 1440, 40]
    for N_pts, max_vox, dense in ((30000, 160000, False), (5000, 1000, True), (1, 10, False)):
        lo, hi = torch.tensor(pc[:3]) - 1.0, torch.tensor(pc[3:]) + 1.0
        xyz = lo + torch.rand(N_pts, 3, generator=g) * (hi - lo)
        if dense:   # pile points into a few voxels -> overfull voxels
            xyz[: N_pts // 2] = torch.tensor([1.01, 2.02, 0.05]) + torch.rand(N_pts // 2, 3, generator=g) * 0.1
        pts = torch.cat([xyz, torch.rand(N_pts, 2, generator=g)], 1).contiguous()
        vox, coors, num, means, nvox = N.voxelize(pts.to(dev), voxel_size=vs, coors_range=pc, grid=grid,
                                                  max_points=10, max_voxels=max_vox, nfeat_mean=5)
        M = int(nvox.item())
        rv = np.zeros((max_vox, 10, 5), np.float32)
        rc = np.zeros((max_vox, 3), np.int32)
        rn = np.zeros((max_vox,), np.int32)
        rm = np.zeros((max_vox, 5), np.float32)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        pn = pts.numpy()
        Mr = lib.cmt_oracle_voxelize(pn.ctypes.data_as(fp), N_pts, 5, np.array(vs, np.float32).ctypes.data_as(fp),
                                     np.array(pc, np.float32).ctypes.data_as(fp),
                                     np.array(grid, np.int32).ctypes.data_as(ip), 10, max_vox, 5,
                                     rv.ctypes.data_as(fp), rc.ctypes.data_as(ip), rn.ctypes.data_as(ip),
                                     rm.ctypes.data_as(fp))
        assert M == Mr
        assert np.array_equal(coors[:M].cpu().numpy(), rc[:M])
        assert np.array_equal(num[:M].cpu().numpy(), rn[:M])
        assert np.array_equal(vox[:M].cpu().numpy(), rv[:M])
        assert np.array_equal(means[:M].cpu().numpy(), rm[:M])


def _ln64(x, w, b, eps=1e-5):
    m = x.mean(-1, keepdim=True)
    v = ((x - m) ** 2).mean(-1, keepdim=True)
    return (x - m) / torch.sqrt(v + eps) * w + b


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Nq,with_r", [(1, 900, True), (2, 37, False)])
def test_chain_a(N, dev, dt, B, Nq, with_r):
    """Row-block chain A (out_proj + bias + residual -> norms[0] -> lowp(y + pos)
    -> cross-attn Q projection, head split) vs fp64 math on the same rounded
    operands; ragged last row block, no-residual (layer 0) form."""
    g = torch.Generator().manual_seed(B * 100 + Nq)
    C, rows = 256, B * Nq
    X = torch.randn(rows, C, generator=g).to(dt)
    R = torch.randn(rows, C, generator=g) if with_r else None
    P = torch.randn(rows, C, generator=g)
    Wo = (torch.randn(C, C, generator=g) / 16).to(dt)
    Wq = (torch.randn(C, C, generator=g) / 16).to(dt)
    bo, lb, bq = (torch.randn(C, generator=g) * 0.1 for _ in range(3))
    lw = 1 + 0.1 * torch.randn(C, generator=g)
    prm = torch.cat([bo, lw, lb, bq])
    Y = torch.empty(rows, C, device=dev)
    Q = torch.empty(B * 8 * Nq * 32, dtype=dt, device=dev)
    N.chain(0, X.to(dev), P.to(dev), prm.to(dev), Wo.to(dev), N.pack_chain_wn(Wq.to(dev)), Y, rows=rows, Nq=Nq, eps=1e-5,
            R=R.to(dev) if R is not None else None, Q=Q)
    d = lambda t: t.double()
    t = d(X) @ d(Wo).T + d(bo) + (d(R) if R is not None else 0)
    y = _ln64(t, d(lw), d(lb))
    q = d((y + d(P)).to(dt)) @ d(Wq).T + d(bq)
    qref = q.view(B, Nq, 8, 32).permute(0, 2, 1, 3).reshape(-1)
    assert (Y.cpu().double() - y).abs().max().item() < 2e-3
    rel = (Q.cpu().double() - qref).abs().max().item() / qref.abs().max().item()
    assert rel < 1.5e-2, rel
    # fragment-major Wo (wo_frag: register-streamed out_proj, no LDS weight ring): the same
    # MFMA k-order, so bit-identical outputs
    Y2 = torch.empty_like(Y)
    Q2 = torch.empty_like(Q)
    N.chain(0, X.to(dev), P.to(dev), prm.to(dev), N.pack_chain_wn(Wo.to(dev)), N.pack_chain_wn(Wq.to(dev)), Y2,
            rows=rows, Nq=Nq, eps=1e-5, R=R.to(dev) if R is not None else None, Q=Q2)
    assert torch.equal(Y, Y2) and torch.equal(Q, Q2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Nq,last,flags", [(1, 900, False, 1), (2, 37, True, 3)])
def test_chain_b(N, dev, dt, B, Nq, last, flags):
    """Row-block chains B1 (out_proj + residual -> norms[1] -> one FFN quarter per
    workgroup -> fp32 partials) and B2 (partials -> norms[2] and post_norm
    (nan_to_num / coop max-into) -> next in_proj, head split) vs fp64 math on the
    same rounded operands."""
    g = torch.Generator().manual_seed(B * 1000 + Nq)
    C, F, rows = 256, 1024, B * Nq
    X = torch.randn(rows, C, generator=g).to(dt)
    R = torch.randn(rows, C, generator=g)
    P = torch.randn(rows, C, generator=g)
    Wo = (torch.randn(C, C, generator=g) / 16).to(dt)
    W1 = (torch.randn(F, C, generator=g) / 16).to(dt)
    W2 = (torch.randn(C, F, generator=g) / 32).to(dt)
    Wn = (torch.randn(3 * C, C, generator=g) / 16).to(dt)
    v = lambda n, s=0.1: torch.randn(n, generator=g) * s
    bo, b1, b2, bn = v(C), v(F), v(C), v(3 * C)
    l1w, l2w, pw = (1 + v(C) for _ in range(3))
    l1b, l2b, pb = v(C), v(C), v(C)
    prm = torch.cat([bo, l1w, l1b, b1, b2, l2w, l2b, pw, pb, torch.zeros(3 * C) if last else bn])
    Y = torch.empty(rows, C, device=dev)
    old = torch.randn(rows, C, generator=g)
    OUT = old.clone().to(dev)
    OUT16 = torch.full(OUT.shape, float("nan"), dtype=dt, device=dev)
    QKV = torch.empty(B * 24 * Nq * 32, dtype=dt, device=dev)
    WS = torch.full((N.chain_ws_numel(rows),), float("nan"), device=dev)
    prm_d = prm.to(dev)
    N.chain(1, X.to(dev), None, prm_d, Wo.to(dev), W1.to(dev), Y, rows=rows, Nq=Nq, eps=1e-5,
            R=R.to(dev), W2=N.pack_chain_fc2(W2.to(dev)), WS=WS)
    N.chain(2, None, None if last else P.to(dev), prm_d, None, None, Y, rows=rows, Nq=Nq, eps=1e-5,
            Wn=None if last else N.pack_chain_wn(Wn.to(dev)), OUT=OUT, out_flags=flags, Q=None if last else QKV, WS=WS,
            OUT16=OUT16)
    d = lambda t: t.double()
    o = _ln64(d(X) @ d(Wo).T + d(bo) + d(R), d(l1w), d(l1b))
    h = torch.relu(d(o.to(dt)) @ d(W1).T + d(b1)).to(dt)
    y = _ln64(d(h) @ d(W2).T + d(b2) + o, d(l2w), d(l2b))
    out = _ln64(y, d(pw), d(pb))
    if flags & 2:
        out = torch.maximum(out, d(old))
    assert (Y.cpu().double() - y).abs().max().item() < 2e-2
    assert (OUT.cpu().double() - out).abs().max().item() < 2e-2
    assert torch.equal(OUT16, OUT.to(dt))      # the 16-bit copy is the rounded fp32 output
    if not last:
        qk = d((y + d(P)).to(dt)) @ d(Wn[:2 * C]).T + d(bn[:2 * C])
        vv = d(y.to(dt)) @ d(Wn[2 * C:]).T + d(bn[2 * C:])
        ref = torch.cat([qk, vv], 1).view(B, Nq, 24, 32).permute(0, 2, 1, 3).reshape(-1)
        rel = (QKV.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nb,nv,C,HW,off", [(1, 1, 512, 32400, 0), (2, 3, 128, 100, 7), (1, 2, 64, 4, 3),
                                            (1, 1, 96, 44, 0)])
def test_nchw_to_rows_layouts(N, dev, dt, nb, nv, C, HW, off):
    """NCHW fp32 -> batch-major rows (vector path when HW % 4 == 0 and C % 64 == 0,
    scalar path otherwise): exact against permute + cast, gap rows untouched."""
    g = torch.Generator().manual_seed(HW + C)
    x = torch.randn(nb * nv, C, HW, generator=g)
    rpb = off + nv * HW + 5
    y = torch.full((nb * rpb, C), float("nan"), dtype=dt, device=dev)
    N.nchw_to_rows(x.to(dev), y, nb=nb, nv=nv, C=C, HW=HW, ldy=C, rows_per_batch=rpb, row_offset=off)
    ref = x.view(nb, nv, C, HW).permute(0, 1, 3, 2).reshape(nb, nv * HW, C).to(dt)
    got = y.view(nb, rpb, C).cpu()
    assert torch.equal(got[:, off:off + nv * HW], ref)
    assert torch.isnan(got[:, :off].float()).all() and torch.isnan(got[:, off + nv * HW:].float()).all()


@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16, torch.float16])
def test_rv_pe_coords_vector_path_bitexact(N, dev, odt):
    """The 8-depths-per-thread rv_pe_coords kernel (16/32-byte stores) equals the
    one-thread-per-depth kernel bit for bit (forced by a misaligned output view);
    the formula itself is held to the oracle by the head parity tests."""
    g = torch.Generator().manual_seed(7)
    BV, h, w, D = 6, 8, 20, 64
    l2i = torch.randn(BV, 4, 4, generator=g, dtype=torch.float64) + 4 * torch.eye(4, dtype=torch.float64)
    i2l = torch.linalg.inv(l2i).float().to(dev)
    pcr = [-54.0, -54.0, -5.0, 54.0, 54.0, 3.0]
    n = BV * h * w * 3 * D
    a = torch.empty(n, dtype=odt, device=dev)
    N.rv_pe_coords(i2l, a, BV=BV, h=h, w=w, D=D, pad_h=128.0, pad_w=320.0, depth_max=pcr[3], pc_range=pcr)
    buf = torch.empty(n + 8, dtype=odt, device=dev)
    b = buf[1:n + 1]                                        # 2- or 4-byte offset: the generic kernel
    N.rv_pe_coords(i2l, b, BV=BV, h=h, w=w, D=D, pad_h=128.0, pad_w=320.0, depth_max=pcr[3], pc_range=pcr)
    torch.cuda.synchronize()
    assert torch.equal(a.cpu(), b.cpu())


@pytest.mark.parametrize("Nq,Nk,B,want", [(900, 56400, 1, 8), (900, 32400, 1, 8), (900, 44400, 1, 8),
                                          (1500, 48400, 1, 5), (900, 56400, 2, 4)])
def test_attention_split_choice(N, dev, Nq, Nk, B, want):
    """cmt_attn_splits on the long-key f16 kernel: whole rounds of the chip's 256 CUs -- the frame
    shapes keep 8 splits (chain B1 combines exactly 8, ABI 19), configs[4]'s 1 500 queries take 5
    (240 workgroups in one round instead of 384 in 1.5: 120 vs 142 us, r6v)."""
    a = N.AttnArgs()
    a.B, a.H, a.Nq, a.Nk, a.dtype = B, 8, Nq, Nk, N.F16
    assert int(N.lib().cmt_attn_splits(ctypes.byref(a))) == want
