"""Diagnostics: error pattern of the split f16 GEMM over shapes (GPU)."""
import math
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cmt-cooperative-perception_amd")]
import torch
from projects.mmdet3d_plugin import native as N
from projects.mmdet3d_plugin.models.utils.packing import to_dtype

dev = torch.device("cuda:0")
N.lib()
for (M, N_, K) in [(2000, 3072, 256), (2048, 3072, 256), (2000, 256, 256), (900, 3072, 256), (128, 3072, 256),
                   (128, 1024, 256), (128, 512, 256), (64, 512, 256), (64, 256, 256)]:
    g = torch.Generator().manual_seed(1)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N_, K, generator=g) / math.sqrt(K)
    ref = A.double() @ W.double().t()
    out = torch.zeros(M, N_, device=dev)
    N.gemm(to_dtype(A.to(dev), torch.uint16), to_dtype(W.to(dev), torch.uint16), out, M=M, N=N_, K=K, lda=K, ldw=K,
           ldc=N_)
    ob = torch.zeros(M, N_, device=dev)
    N.gemm(A.bfloat16().to(dev), W.bfloat16().to(dev), ob, M=M, N=N_, K=K, lda=K, ldw=K, ldc=N_)
    torch.cuda.synchronize()
    e = (out.cpu().double() - ref).abs()
    eb = (ob.cpu().double() - ref).abs()
    bad = (e > 1e-3).nonzero()
    print(f"{M}x{N_}x{K}: split max {e.max().item():.2e} bad {bad.shape[0]} | bf16 dma max {eb.max().item():.2e}",
          flush=True)
    if bad.shape[0]:
        r, c = bad[:, 0], bad[:, 1]
        print("   rows", r.min().item(), r.max().item(), "cols", c.min().item(), c.max().item(),
              "col%64 set", sorted(set((c % 64).tolist()))[:10], "row%64", sorted(set((r % 64).tolist()))[:10],
              "n col tiles", len(set((c // 64).tolist())), flush=True)
