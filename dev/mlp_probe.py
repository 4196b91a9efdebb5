"""Time cmt_mlp2_x3 against the two split GEMMs it replaces at the _rv_pe shape
(24 000 rows, K 192, Hd 1024, pair output + pair residual) and the query shape
(5 400 rows, fp32 output).  HIP events, median of 7 x 20 launches.
    python dev/mlp_probe.py"""
import statistics
import sys

import torch

sys.path.insert(0, "cmt-cooperative-perception_amd")
from projects.mmdet3d_plugin import native  # noqa: E402


def pair(x):
    hi = x.half()
    return torch.stack([hi, (x - hi.float()).half()], dim=-2).contiguous().view(torch.uint16)


def timeit(fn, reps=20, rounds=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return statistics.median(ts)


dev = torch.device("cuda")
for M, out in ((24000, "pair"), (5400, "f32")):
    K, Hd = 192, 1024
    A = pair(torch.rand(M, K) * 4 - 2).to(dev)
    W1 = pair(torch.randn(Hd, K) / K ** 0.5).to(dev)
    W2 = pair(torch.randn(256, Hd) / Hd ** 0.5).to(dev)
    b1, b2 = torch.randn(Hd, device=dev) * 0.1, torch.randn(256, device=dev) * 0.1
    C = torch.empty((M, 2, 256), dtype=torch.uint16, device=dev) if out == "pair" else torch.empty((M, 256), device=dev)
    R = pair(torch.randn(M, 256)).to(dev) if out == "pair" else None
    w1p, w2p = native.mlp2_pack(W1, W2)
    H = torch.empty((M, 2, Hd), dtype=torch.uint16, device=dev)

    def fused():
        native.mlp2(A, w1p, b1, w2p, b2, C, M=M, K=K, Hd=Hd, R=R)

    def fc1():
        native.gemm(A, W1, H, M=M, N=Hd, K=K, lda=K, ldw=K, ldc=Hd, bias=b1, relu=True)

    def fc2():
        native.gemm(H, W2, C, M=M, N=256, K=Hd, lda=Hd, ldw=Hd, ldc=256, bias=b2, R=R, ldr=256 if R is not None else 0)

    tf, t1, t2 = timeit(fused), timeit(fc1), timeit(fc2)
    flop = 3 * 2 * M * (K * Hd + Hd * 256)
    print(f"mlp M={M} {out}: fused {tf:7.1f} us ({flop / tf / 1e6:6.0f} TF/s 3-pass)  two GEMMs {t1:6.1f} + {t2:6.1f} "
          f"= {t1 + t2:6.1f} us", flush=True)
