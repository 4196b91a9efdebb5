"""Time the training bf16x3 GEMM (cmt_gemm_bf16x3_ex) at the training step's shapes and check it
against a float64 product.  CMT_HIP_LIB selects the library (A/B of two builds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cmt-cooperative-perception_amd"))
from projects.mmdet3d_plugin import native_train as T  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


def main():
    torch.manual_seed(0)
    dev = "cuda"
    lib = os.environ.get("CMT_HIP_LIB", "lib")
    for name, M, K, Nn in [("dec_fwd", 1100, 256, 256), ("dec_ffn1", 1100, 256, 512),
                           ("kv_fwd", 44400, 256, 256), ("conv_like", 32400, 256, 4608)]:
        X = torch.randn(M, K, device=dev)
        W = torch.randn(Nn, K, device=dev) * 0.05
        b = torch.randn(Nn, device=dev)
        dY = torch.randn(M, Nn, device=dev)
        Y = T.linear_fwd(X, W, b)
        ref = (X.double() @ W.double().T + b.double())
        e_f = ((Y.double() - ref).abs().max() / ref.abs().max()).item()
        dX, dW, _ = T.linear_bwd(dY, X, W, need_db=False)
        rx = dY.double() @ W.double()
        rw = dY.double().T @ X.double()
        e_x = ((dX.double() - rx).abs().max() / rx.abs().max()).item()
        e_w = ((dW.double() - rw).abs().max() / rw.abs().max()).item()
        tf = timed(lambda: T.linear_fwd(X, W, b))
        tx = timed(lambda: T.linear_bwd(dY, X, W, need_dw=False, need_db=False))
        tw = timed(lambda: T.linear_bwd(dY, X, W, need_dx=False, need_db=False))
        print(f"{lib} {name:10s} M={M} K={K} N={Nn}: fwd {tf:7.1f} us  dX {tx:7.1f} us  dW {tw:7.1f} us"
              f"  (ks {T._ksplit(M, Nn, K)})  rel err {e_f:.1e} {e_x:.1e} {e_w:.1e}", flush=True)


if __name__ == "__main__":
    main()
