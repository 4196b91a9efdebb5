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


def conv_wgrad():
    """shared_conv's weight gradient at the coop shape: im2col + GEMM vs the implicit form."""
    torch.manual_seed(0)
    lib = os.environ.get("CMT_HIP_LIB", "lib")
    H = W = 180
    Cin, Cout = 512, 256
    x = torch.randn(H * W, Cin, device="cuda")
    dy = torch.randn(H * W, Cout, device="cuda")
    ks = max(T._ksplit(H * W, Cout, 9 * Cin), 2)

    def im2col():
        col = T.im2col3x3(x, 1, H, W, Cin)
        dw = torch.zeros(Cout, 9 * Cin, device="cuda")
        T.gemm_ex(dy, (1, Cout), col, (1, 9 * Cin), dw, M=Cout, N_=9 * Cin, K=H * W, ldc=9 * Cin, beta=1.0, ksplit=ks)
        return dw
    a, b = im2col(), T.conv3x3_wgrad(x, dy, 1, H, W, Cin, ks)
    err = ((a - b).abs().max() / a.abs().max()).item()
    print(f"{lib} conv_wgrad 180x180 {Cin}->{Cout} ks {ks}: im2col+gemm {timed(im2col, 5):8.1f} us  implicit "
          f"{timed(lambda: T.conv3x3_wgrad(x, dy, 1, H, W, Cin, ks), 5):8.1f} us  rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    conv_wgrad()
    main()
