"""Cross-attention core microbenchmark for kernel experiments: the decoder's
cross-attention shape (900 queries x Nk keys, 8 heads x 32, head-split bf16
operands as the K/V projection writes them, optional max-|k| partials =
bounded-max mode as the bf16 bench path runs it).  HIP events, median of
reps x inner back-to-back launches.  Variant switches are read by the library
from the environment (CMT_ATTN_*), so run one process per variant.

    python dev/attn_exp.py --nk 56400 --bound [--splits S] [--check]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

import torch  # noqa: E402

from projects.mmdet3d_plugin import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nk", type=int, default=56400)
    ap.add_argument("--nq", type=int, default=900)
    ap.add_argument("--bound", action="store_true")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--check", action="store_true", help="compare with an fp32 torch reference")
    ap.add_argument("--qs", action="store_true", help="keep Q*scale*log2e as hi+lo (the 'ref' policy), no fold")
    ap.add_argument("--round", action="store_true", help="round the output to the attention dtype (flash-attn)")
    ap.add_argument("--tag", default=os.environ.get("CMT_ATTN_VARIANT", "base"))
    a = ap.parse_args()
    dev = torch.device("cuda")
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    B, H, Nq, Nk = 1, 8, a.nq, a.nk
    g = torch.Generator(device="cpu").manual_seed(0)
    q = (torch.randn(B * H * Nq * 32, generator=g) * 0.6).to(dt).to(dev)
    k = (torch.randn(B * H * Nk * 32, generator=g) * 0.6).to(dt).to(dev)
    v = torch.randn(B * H * Nk * 32, generator=g).to(dt).to(dev)
    O = torch.empty(B * Nq * H * 32, dtype=dt, device=dev)
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    kmax2 = None
    if a.bound:
        nb = -(-Nk // 64)
        ss = (k.float().view(H, Nk, 32) ** 2).sum(-1)
        ss = torch.cat([ss, ss.new_zeros(H, nb * 64 - Nk)], 1).view(H, nb, 64).amax(-1)
        kmax2 = ss.t().contiguous()

    def run():
        N.attention(q, k, v, O, B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(H * Nq * 32, Nq * 32, 32),
                    k_strides=(H * Nk * 32, Nk * 32, 32), v_strides=(H * Nk * 32, Nk * 32, 32),
                    o_strides=(Nq * H * 32, H * 32), scale=32 ** -0.5, kv_splits=a.splits, workspace=ws,
                    fold_scale=not a.qs, round_output=a.round, kmax2=kmax2, kmax_ld=H, kmax_plane0=0)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2_000_000)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    us = ts[len(ts) // 2]
    tf = 4.0 * B * Nq * Nk * H * 32 / (us * 1e-6) / 1e12
    msg = f"attn[{a.tag}] {a.dtype} qs={int(a.qs)} Nq={Nq} Nk={Nk} bound={int(a.bound)} splits={a.splits} {us:8.2f} us {tf:7.1f} TF/s frac {tf / 2500:.3f}"
    if a.check:
        qh = q.float().view(H, Nq, 32)
        kh = k.float().view(H, Nk, 32)
        vh = v.float().view(H, Nk, 32)
        ref = torch.softmax(qh @ kh.transpose(1, 2) / math.sqrt(32), -1) @ vh      # [H, Nq, 32]
        got = O.float().view(Nq, H, 32).transpose(0, 1)
        msg += f" maxerr {(got - ref).abs().max().item():.2e}"
    print(msg, flush=True)


if __name__ == "__main__":
    main()
