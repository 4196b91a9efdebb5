"""Launch one of the 'ref' policy's memory-side kernels at the fusion frame's
shape a few times (for rocprofv3 counter passes, dev/kernel_pmc.sh):

    python dev/kernel_probe.py kv|conv|convh|mlp [--iters N]
kv:   cmt_kv_proj split form, M = 56 400 tokens, N = 3072 (all layers' K|V), K = 256
conv: shared_conv as the split implicit 3x3 GEMM, 180 x 180 x 512 -> 256
convh: shared_conv straight from the NCHW fp32 map (conv_halo_x3_kernel, the 'ref' path)
mlp:  rv_embedding in one launch (cmt_mlp2_x3), 24 000 camera tokens, 192 -> 1024 -> 256"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

import torch  # noqa: E402

from projects.mmdet3d_plugin import native as N  # noqa: E402


def pairs(*shape):
    return torch.randint(0, 1 << 14, shape, dtype=torch.int16, device="cuda").view(torch.uint16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["kv", "conv", "convh", "mlp"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--time", action="store_true", help="also print the mean of 20 back-to-back launches")
    a = ap.parse_args()
    N.lib()
    if a.what == "kv":
        M, Nn = 56400, 3072
        A, A2 = pairs(M, 2, 256), pairs(M, 2, 256)
        W = pairs(2 * Nn * 256)          # fragment-packed hi planes, then lo planes
        C = torch.empty(M * Nn, dtype=torch.float16, device="cuda")
        pm = torch.empty(-(-M // 64), Nn // 2 // 32, device="cuda")
        bias = torch.randn(Nn, device="cuda")
        run = lambda: N.kv_proj(A, W, C, M=M, N=Nn, bias=bias, A2=A2, headsplit_rows=M, plane_max2=pm,  # noqa: E731
                                plane_max_cols=Nn // 2)
    elif a.what == "mlp":
        M, K, Hd = 24000, 192, 1024
        A = pairs(M, 2, K)
        W1p, W2p = N.mlp2_pack(pairs(Hd, 2, K), pairs(256, 2, Hd))
        b1, b2 = torch.randn(Hd, device="cuda"), torch.randn(256, device="cuda")
        C = torch.empty(M, 2, 256, dtype=torch.uint16, device="cuda")
        run = lambda: N.mlp2(A, W1p, b1, W2p, b2, C, M=M, K=K, Hd=Hd)  # noqa: E731
    elif a.what == "convh":
        X = torch.randn(1, 512, 180, 180, device="cuda")
        W = pairs(256, 2, 4608)
        C = torch.empty(32400, 2, 256, dtype=torch.uint16, device="cuda")
        bias = torch.randn(256, device="cuda")
        run = lambda: N.gemm(X, W, C, M=32400, N=256, K=4608, lda=32400, ldw=4608, ldc=256, bias=bias,  # noqa: E731
                             relu=True, a_mode=N.A_CONV3X3_NCHW, conv=(180, 180, 512), batch=1,
                             a_bstride=512 * 32400, c_bstride=32400 * 256)
    else:
        A = pairs(32400, 2, 512)
        W = pairs(256, 2, 4608)
        C = torch.empty(32400, 2, 256, dtype=torch.uint16, device="cuda")
        bias = torch.randn(256, device="cuda")
        run = lambda: N.gemm(A, W, C, M=32400, N=256, K=4608, lda=512, ldw=4608, ldc=256, bias=bias,  # noqa: E731
                             relu=True, a_mode=N.A_CONV3X3, conv=(180, 180, 512))
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    if a.time:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        e1.synchronize()
        print(f"{a.what}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per launch")
    print("ok")


if __name__ == "__main__":
    main()
