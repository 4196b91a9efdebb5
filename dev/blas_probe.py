"""hipBLASLt (torch.matmul, bf16) on the head's GEMM shapes: what the library
reaches on this box, as a yardstick for the fused native kernels (which also
apply pos-add / head-split / epilogues the library does not)."""
import torch

def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3

dev = torch.device("cuda")
bf = torch.bfloat16
for name, M, N, K in (("kv proj (fusion)", 56400, 3072, 256), ("kv proj (lidar)", 32400, 3072, 256),
                      ("shared_conv as GEMM", 32400, 256, 4608), ("bev mlp fc1", 32400, 256, 512),
                      ("out proj", 900, 256, 256), ("ffn fc1", 900, 1024, 256)):
    a = torch.randn(M, K, device=dev, dtype=bf)
    w = torch.randn(K, N, device=dev, dtype=bf)
    us = t(lambda: torch.matmul(a, w))
    print(f"{name:22s} M={M:6d} N={N:5d} K={K:5d} {us:9.2f} us {2*M*N*K/us/1e6:8.1f} TF/s", flush=True)
