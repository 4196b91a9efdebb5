"""Per-kernel microbenchmark of libcmt_hip.so at the CMT-L frame's shapes
(HIP events on the launching stream, median of N launches).

    python dev/bench_kernels.py [--only gemm|attn|attn_sweep|chain|misc]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

import torch  # noqa: E402

from projects.mmdet3d_plugin import native as N  # noqa: E402


def timeit(fn, reps=5, inner=50, warm=3):
    """Median over `reps` of the mean time of `inner` back-to-back launches
    (queued ahead, so host-side argument packing does not show)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2_000_000)   # let the host queue the launches ahead of the GPU
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / inner)
    ts.sort()
    return ts[len(ts) // 2] * 1e3   # us


def gemm_case(name, M, Nn, K, dt, a_f32=True, A2_cols=0, out_dt=torch.float32, headsplit=0, relu=False, R=False,
              conv=None, batch=1):
    dev = torch.device("cuda")
    A = torch.randn(M * batch if conv is None else M * batch, K if conv is None else conv[2], device=dev)
    if not a_f32:
        A = A.to(dt)
    W = (torch.randn(Nn, K, device=dev) / math.sqrt(K)).to(dt)
    bias = torch.randn(Nn, device=dev)
    A2 = torch.randn_like(A) if A2_cols else None
    if conv is None and K % 64:   # pragma: no cover
        raise ValueError(K)
    Rt = torch.randn(M, Nn, device=dev) if R else None
    C = torch.empty(M * Nn * batch, dtype=out_dt, device=dev)
    kw = dict(M=M, N=Nn, K=K, lda=A.shape[1], ldw=K, ldc=Nn, bias=bias, relu=relu, R=Rt, ldr=Nn, A2=A2,
              lda2=K if A2 is not None else 0, a2_cols=A2_cols, headsplit_rows=headsplit)
    if conv is not None:
        kw.update(a_mode=N.A_CONV3X3, conv=conv, batch=batch, a_bstride=M * conv[2], c_bstride=M * Nn)
    us = timeit(lambda: N.gemm(A, W, C, **kw))
    tf = 2.0 * M * Nn * K * batch / (us * 1e-6) / 1e12
    line = f"gemm {name:28s} M={M:6d} N={Nn:5d} K={K:5d} {str(dt)[6:]:9s} {us:9.2f} us {tf:8.1f} TF/s"
    if conv is None and batch == 1:   # hipBLASLt on the same shape, same dtype A
        Al = A.to(dt)
        Ct = torch.empty(M, Nn, dtype=dt, device=dev)
        ut = timeit(lambda: torch.matmul(Al, W.t(), out=Ct))
        line += f"   | torch {ut:8.2f} us"
    print(line, flush=True)


def split_case(name, M, Nn, K, conv=None, relu=False, R=False, out="pair", nchw=False):
    """A split (f16-pair) GEMM of the 'ref' policy: A / W / C as [rows, 2, width] 16-bit pairs."""
    dev = torch.device("cuda")
    rows_a = M if conv is None else M
    width = K if conv is None else conv[2]
    A = torch.randint(0, 1 << 14, (rows_a, 2, width), dtype=torch.int16, device=dev).view(torch.uint16)
    W = torch.randint(0, 1 << 14, (Nn, 2, K), dtype=torch.int16, device=dev).view(torch.uint16)
    bias = torch.randn(Nn, device=dev)
    C = (torch.empty(M, 2, Nn, dtype=torch.uint16, device=dev) if out == "pair"
         else torch.empty(M, Nn, device=dev))
    Rt = torch.empty(M, 2, Nn, dtype=torch.uint16, device=dev).fill_(0) if R else None
    kw = dict(M=M, N=Nn, K=K, lda=width, ldw=K, ldc=Nn, bias=bias, relu=relu, R=Rt, ldr=Nn if R else 0)
    if conv is not None:
        kw.update(a_mode=N.A_CONV3X3, conv=conv)
    if conv is not None and nchw:
        # the NCHW fp32 map itself (CMT_A_CONV3X3_NCHW: halo split in the kernel)
        A = torch.randn(conv[2], M, device=dev)
        kw.update(a_mode=N.A_CONV3X3_NCHW, lda=M, a_bstride=conv[2] * M)
    us = timeit(lambda: N.gemm(A, W, C, **kw))
    tf = 3 * 2.0 * M * Nn * K / (us * 1e-6) / 1e12
    print(f"split {name:28s} M={M:6d} N={Nn:5d} K={K:5d} {us:9.2f} us {tf:8.1f} TF/s (3 f16 passes)", flush=True)


def attn_case(name, Nq, Nk, dt, B=1, H=8, splits=0, fold=False):
    dev = torch.device("cuda")
    q = torch.randn(B * H * Nq * 32, device=dev).to(dt)
    k = torch.randn(B * H * Nk * 32, device=dev).to(dt)
    v = torch.randn(B * H * Nk * 32, device=dev).to(dt)
    O = torch.empty(B * Nq * H * 32, device=dev)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)

    def run():
        N.attention(q, k, v, O, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(H * Nq * 32, Nq * 32, 32),
                    k_strides=(H * Nk * 32, Nk * 32, 32), v_strides=(H * Nk * 32, Nk * 32, 32),
                    o_strides=(Nq * H * 32, H * 32), scale=1 / math.sqrt(32), kv_splits=splits, workspace=ws,
                    fold_scale=fold)
    us = timeit(run)
    tf = 4.0 * B * Nq * Nk * H * 32 / (us * 1e-6) / 1e12
    print(f"attn {name:28s} Nq={Nq:5d} Nk={Nk:6d} {str(dt)[6:]:9s} splits={splits:3d} fold={int(fold)} {us:9.2f} us "
          f"{tf:8.1f} TF/s", flush=True)


def chain_case(kind, rows=900, Nq=900, dt=torch.bfloat16, last=False, cold=False, wo_frag=False):
    """Row-block chain A (kind 0), B1 (1) or B2 (2) at the decoder's query shape.
    cold: a 64 MB streaming read between launches (evicts the weights from L2,
    as the cross-attention's K/V stream does in the frame); its own time is
    measured alone and subtracted."""
    dev = torch.device("cuda")
    C, F = 256, 1024
    X = torch.randn(rows, C, device=dev).to(dt)
    R, P = torch.randn(rows, C, device=dev), torch.randn(rows, C, device=dev)
    Wo = (torch.randn(C, C, device=dev) / 16).to(dt)
    W1 = (torch.randn(F if kind else C, C, device=dev) / 16).to(dt)
    W2 = (torch.randn(C, F, device=dev) / 32).to(dt)
    Wn = None if last else N.pack_chain_wn((torch.randn(3 * C, C, device=dev) / 16).to(dt))
    prm = torch.randn(N.CHAIN_PRM[kind], device=dev) * 0.1
    Y, OUT = torch.empty(rows, C, device=dev), torch.empty(rows, C, device=dev)
    WS = torch.randn(N.chain_ws_numel(rows), device=dev)
    Q = torch.empty(rows * 3 * C, dtype=dt, device=dev)
    if kind == 0:
        W1p = N.pack_chain_wn(W1[:256].contiguous())
        Wa = N.pack_chain_wn(Wo) if wo_frag else Wo
        fn = lambda: N.chain(0, X, P, prm, Wa, W1p, Y, rows=rows, Nq=Nq, eps=1e-5, R=R, Q=Q)
        fl = 2 * rows * C * C * 2
    elif kind == 1:
        W2p = N.pack_chain_fc2(W2)
        fn = lambda: N.chain(1, X, None, prm, Wo, W1, Y, rows=rows, Nq=Nq, eps=1e-5, R=R, W2=W2p, WS=WS)
        fl = 2 * rows * C * C * 9
    else:
        fn = lambda: N.chain(2, None, None if last else P, prm, None, None, Y, rows=rows, Nq=Nq, eps=1e-5,
                             Wn=Wn, OUT=OUT, Q=None if last else Q, WS=WS)
        fl = 2 * rows * C * C * (0 if last else 3)
    if cold:
        junk = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        flush = lambda: junk.view(torch.float32).sum()  # noqa: E731
        t_flush = timeit(flush)
        us = timeit(lambda: (flush(), fn())) - t_flush
    else:
        us = timeit(fn)
    tag = (" cold" if cold else "") + (" wo_frag" if wo_frag else "")
    print(f"chain {['A ', 'B1', 'B2'][kind]}{' last' if last else '     '}{tag} rows={rows:5d} {us:9.2f} us "
          f"{fl / (us * 1e-6) / 1e12:8.1f} TF/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    N.lib()
    bf = torch.bfloat16
    if args.only in ("", "gemm"):
        gemm_case("kv (all layers, pos add)", 32400, 3072, 256, bf, A2_cols=1536, out_dt=bf, headsplit=32400)
        gemm_case("bev mlp fc1 (relu)", 32400, 256, 512, bf, relu=True)
        gemm_case("bev mlp fc2", 32400, 256, 256, bf)
        gemm_case("shared_conv 3x3 (implicit)", 32400, 256, 4608, bf, a_f32=False, conv=(180, 180, 512), relu=True,
                  out_dt=bf)
        gemm_case("self qkv (pos add)", 900, 768, 256, bf, A2_cols=512, out_dt=bf, headsplit=900)
        gemm_case("out proj (+res)", 900, 256, 256, bf, R=True)
        gemm_case("cross q (pos add)", 900, 256, 256, bf, A2_cols=256, out_dt=bf, headsplit=900)
        gemm_case("ffn fc1 (relu)", 900, 1024, 256, bf, relu=True)
        gemm_case("ffn fc2 (+res)", 900, 256, 1024, bf, R=True)
        gemm_case("ffn fc1 f32", 900, 1024, 256, torch.float32, relu=True)
        gemm_case("square 4096 bf16", 4096, 4096, 4096, bf, a_f32=False)
        print("-- compute-dtype A (LDS-DMA path)")
        gemm_case("kv (select)", 32400, 3072, 256, bf, a_f32=False, A2_cols=1536, out_dt=bf, headsplit=32400)
        gemm_case("bev mlp fc1 (relu)", 32400, 256, 512, bf, a_f32=False, relu=True, out_dt=bf)
        gemm_case("bev mlp fc2 (+R)", 32400, 256, 256, bf, a_f32=False, R=True, out_dt=bf)
        gemm_case("self qkv (select)", 900, 768, 256, bf, a_f32=False, A2_cols=512, out_dt=bf, headsplit=900)
        gemm_case("out proj (+res)", 900, 256, 256, bf, a_f32=False, R=True)
        gemm_case("ffn fc1 (relu)", 900, 1024, 256, bf, a_f32=False, relu=True, out_dt=bf)
        gemm_case("ffn fc2 (+res)", 900, 256, 1024, bf, a_f32=False, R=True)
    if args.only in ("", "enc"):
        # the encoding GEMMs of the fusion frame (compute-dtype A, LDS-DMA path)
        gemm_case("rv fc1 (relu)", 24000, 1024, 192, bf, a_f32=False, relu=True, out_dt=bf)
        gemm_case("rv fc2 (+R)", 24000, 256, 1024, bf, a_f32=False, R=True, out_dt=bf)
        gemm_case("rv query fc1 (relu)", 5400, 1024, 192, bf, a_f32=False, relu=True, out_dt=bf)
        gemm_case("rv query fc2", 5400, 256, 1024, bf, a_f32=False)
        gemm_case("shared_conv 3x3 (implicit)", 32400, 256, 4608, bf, a_f32=False, conv=(180, 180, 512), relu=True,
                  out_dt=bf)
        gemm_case("shared_conv shape, plain rows", 32400, 256, 4608, bf, a_f32=False, relu=True, out_dt=bf)
    if args.only in ("", "gemm", "kv"):
        dev = torch.device("cuda")
        A = torch.randn(32400, 256, device=dev).to(bf)
        A2 = torch.randn(32400, 256, device=dev).to(bf)
        Wp = N.kv_pack((torch.randn(3072, 256, device=dev) / 16).to(bf))
        bias = torch.randn(3072, device=dev)
        C = torch.empty(32400 * 3072, dtype=bf, device=dev)
        pm = torch.empty(507, 48, device=dev)
        us = timeit(lambda: N.kv_proj(A, Wp, C, M=32400, N=3072, bias=bias, A2=A2, headsplit_rows=32400,
                                      plane_max2=pm, plane_max_cols=1536))
        print(f"kv_proj (A-stationary, packed W)  M= 32400 N= 3072 K=  256 {us:9.2f} us "
              f"{2 * 32400 * 3072 * 256 / (us * 1e-6) / 1e12:8.1f} TF/s", flush=True)
    if args.only in ("", "split"):
        split_case("shared_conv 3x3 (implicit)", 32400, 256, 4608, conv=(180, 180, 512), relu=True)
        split_case("shared_conv 3x3 (NCHW halo)", 32400, 256, 4608, conv=(180, 180, 512), relu=True, nchw=True)
        split_case("rv fc1 (relu)", 24000, 1024, 192, relu=True)
        split_case("rv fc2 (+R)", 24000, 256, 1024, R=True)
        split_case("bev fc2 (+R)", 32400, 256, 256, R=True)
        split_case("rv query fc1 (relu)", 5400, 1024, 192, relu=True)
        split_case("rv query fc2", 5400, 256, 1024, out="f32")
    if args.only in ("", "chain"):
        for kind, last in ((0, False), (1, False), (2, False), (2, True)):
            chain_case(kind, last=last)
            chain_case(kind, last=last, cold=True)
        chain_case(0, wo_frag=True)
        chain_case(0, wo_frag=True, cold=True)
        chain_case(1, rows=1800)
    if args.only in ("", "attn"):
        for s in (0, 8, 16):
            for fold in (False, True):
                attn_case("cross 900x32400", 900, 32400, bf, splits=s, fold=fold)
        attn_case("cross fp16", 900, 32400, torch.float16)
        attn_case("self 900x900", 900, 900, bf)
        attn_case("self 900x900", 900, 900, bf, fold=True)
        attn_case("self f32", 900, 900, torch.float32)
        attn_case("cross fusion 900x56400", 900, 56400, bf)
    if args.only == "chain_sweep":
        for rows in (32, 288, 900, 1800, 3600):
            chain_case(2, rows=rows, Nq=rows, last=True)
            chain_case(2, rows=rows, Nq=rows)
            chain_case(0, rows=rows, Nq=rows)
    if args.only == "attn_sweep":
        # split-count sweep at the decoder's shapes (0 = the library's choice)
        for s in (0, 1, 2, 3, 4, 6, 8):
            attn_case("self 900x900", 900, 900, bf, splits=s, fold=True)
        for s in (0, 4, 6, 8, 12, 16):
            attn_case("cross 900x32400", 900, 32400, bf, splits=s, fold=True)


if __name__ == "__main__":
    main()
