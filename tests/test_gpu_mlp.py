"""cmt_mlp2_x3 (csrc/mlp.hip): rv_embedding (cmt_head.py:297-301) --
Linear(K, Hd) + ReLU + Linear(Hd, 256) -- in one launch at the reference's
numerics, against

  * the two split GEMMs it replaces (cmt_gemm fc1 -> hidden pair rows -> cmt_gemm
    fc2): the hidden values are bit-identical (same k order); fc2 sums the same
    products with each 16-unit k-step's elements in another order inside the
    MFMA, so the outputs agree to a few fp32 ulps of the accumulated magnitude;
  * a float64 restatement: within the split product's bound (~2^-19 of each
    output's accumulated magnitude).

Shapes: the nuScenes frustum rows (6 x 40 x 100 = 24 000, K = 192, Hd = 1024),
the query rows (900 x 6 = 5 400), ragged row counts, a batch of two with row
offsets / strides into a larger buffer, pair and fp32 outputs, pair and fp32
residuals.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(x):
    hi = x.half()
    lo = (x - hi.float()).half()
    return torch.stack([hi, lo], dim=-2).contiguous().view(torch.uint16)


def _unpair(p):
    h = p.view(torch.float16)
    return h[..., 0, :].double() + h[..., 1, :].double()


def _case(dev, M, K, Hd, batch=1, out="pair", res=None, seed=0):
    from projects.mmdet3d_plugin import native
    g = torch.Generator().manual_seed(seed)
    A = _pair((torch.rand(batch * M, K, generator=g) * 4 - 2)).to(dev)              # coordinate-like
    W1 = _pair(torch.randn(Hd, K, generator=g) * (1.0 / K ** 0.5)).to(dev)
    b1 = (torch.randn(Hd, generator=g) * 0.1).to(dev)
    W2 = _pair(torch.randn(256, Hd, generator=g) * (1.0 / Hd ** 0.5)).to(dev)
    b2 = (torch.randn(256, generator=g) * 0.1).to(dev)
    # C / R: rows of a larger buffer (offset 7 rows, per-batch stride M + 11 rows), as the camera
    # rows of the [B * Nk] memory buffer
    rows = batch * (M + 11) + 7
    cdt = torch.uint16 if out == "pair" else torch.float32
    C = torch.zeros((rows, 2, 256) if out == "pair" else (rows, 256), dtype=cdt, device=dev)
    R = None
    if res is not None:
        Rf = torch.randn(rows, 256, generator=g)
        R = (_pair(Rf) if res == "pair" else Rf).to(dev)
    w1p, w2p = native.mlp2_pack(W1, W2)
    native.mlp2(A, w1p, b1, w2p, b2, C, M=M, K=K, Hd=Hd, R=R, batch=batch, a_bstride=M * K, c_offset=7 * 256,
                c_bstride=(M + 11) * 256, r_offset=7 * 256, r_bstride=(M + 11) * 256)
    # the two-GEMM path
    H = torch.empty((batch * M, 2, Hd), dtype=torch.uint16, device=dev)
    native.gemm(A, W1, H, M=batch * M, N=Hd, K=K, lda=K, ldw=K, ldc=Hd, bias=b1, relu=True)
    C2 = torch.zeros_like(C)
    native.gemm(H, W2, C2, M=M, N=256, K=Hd, lda=Hd, ldw=Hd, ldc=256, bias=b2, batch=batch, a_bstride=M * Hd,
                c_bstride=(M + 11) * 256, c_offset=7 * 256, R=R, ldr=256 if R is not None else 0,
                r_bstride=(M + 11) * 256 if R is not None else 0, r_offset=7 * 256)
    torch.cuda.synchronize()
    # float64 restatement
    A64, W164, W264 = _unpair(A.cpu()), _unpair(W1.cpu()), _unpair(W2.cpu())
    h64 = torch.relu(A64 @ W164.T + b1.cpu().double())
    o64 = h64 @ W264.T + b2.cpu().double()
    mag = (h64.abs() @ W264.abs().T + b2.cpu().double().abs())                    # accumulated magnitude
    got = _unpair(C.cpu()) if out == "pair" else C.cpu().double()
    two = _unpair(C2.cpu()) if out == "pair" else C2.cpu().double()
    for z in range(batch):
        sl = slice(7 + z * (M + 11), 7 + z * (M + 11) + M)
        r64 = 0.0
        if R is not None:
            r64 = _unpair(R.cpu()[sl]) if res == "pair" else R.cpu()[sl].double()
        ref = o64[z * M:(z + 1) * M] + r64
        m = mag[z * M:(z + 1) * M] + (r64.abs() if R is not None else 0.0)
        # output rounding: pair ~2^-22 relative, fp32 2^-24
        e_ref = ((got[sl] - ref).abs() / m).max().item()
        e_two = ((got[sl] - two[sl]).abs() / m).max().item()
        assert e_ref <= 2 ** -19, (M, K, Hd, z, e_ref)
        assert e_two <= 2 ** -20, (M, K, Hd, z, e_two)
    # rows outside the launch's ranges are untouched
    mask = torch.ones(rows, dtype=torch.bool)
    for z in range(batch):
        mask[7 + z * (M + 11): 7 + z * (M + 11) + M] = False
    assert (C.cpu()[mask] == 0).all()


@pytest.mark.parametrize("M,K,Hd,batch,out,res", [
    (24000, 192, 1024, 1, "pair", "pair"),     # _rv_pe of a nuScenes frame: lowp(memory + pos)
    (5400, 192, 1024, 1, "f32", None),         # _rv_query_embed: 900 queries x 6 views
    (1000, 192, 1024, 2, "pair", "pair"),      # two batch elements into a larger buffer
    (37, 64, 128, 1, "f32", "f32"),            # ragged rows, short K, four hidden blocks
    (129, 64, 64, 1, "pair", None),            # four k-steps, two hidden blocks, a partial workgroup
])
def test_mlp2_matches_two_gemms_and_float64(dev, M, K, Hd, batch, out, res):
    _case(dev, M, K, Hd, batch=batch, out=out, res=res)


def test_mlp2_rejects(dev):
    from projects.mmdet3d_plugin import native
    A = torch.zeros((32, 2, 200), dtype=torch.uint16, device=dev)
    W1 = torch.zeros((64, 2, 208), dtype=torch.uint16, device=dev)
    W2 = torch.zeros((256, 2, 64), dtype=torch.uint16, device=dev)
    with pytest.raises(RuntimeError):
        native.mlp2_pack(W1, torch.zeros((128, 2, 64), dtype=torch.uint16, device=dev))   # N != 256
    w1p = torch.zeros(64 * 2 * 208, dtype=torch.uint16, device=dev)
    w2p = torch.zeros(256 * 2 * 64, dtype=torch.uint16, device=dev)
    b1 = torch.zeros(64, device=dev)
    b2 = torch.zeros(256, device=dev)
    C = torch.zeros((32, 256), device=dev)
    with pytest.raises(RuntimeError, match="K must be"):
        native.mlp2(A, w1p, b1, w2p, b2, C, M=32, K=200, Hd=64)                      # K % 16 != 0
    with pytest.raises(RuntimeError, match="K must be"):
        native.mlp2(torch.zeros((32, 2, 208), dtype=torch.uint16, device=dev), w1p, b1, w2p, b2, C, M=32,
                    K=208, Hd=64)                                                    # K > 192
