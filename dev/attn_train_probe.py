"""Time the training attention kernels at the coop self-attention shape (both agents' queries:
B = 2, H = 8, Nq = Nk = 900 + DN padding, the DN mask, attn_drop 0.1; exact f32) or the long-key
fp16 cross core (--cross).  HIP events, median of 7 x 10 launches.
    python dev/attn_train_probe.py [--cross] [--nq 1100] [--pad 200] [--group 20] [--drop 0.1]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

import torch  # noqa: E402

from projects.mmdet3d_plugin import native_train as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cross", action="store_true")
    ap.add_argument("--nq", type=int, default=1100)
    ap.add_argument("--nk", type=int, default=0)
    ap.add_argument("--pad", type=int, default=200)
    ap.add_argument("--group", type=int, default=20)
    ap.add_argument("--drop", type=float, default=0.1)
    ap.add_argument("--tag", default=os.environ.get("CMT_HIP_LIB", "base").split("/")[-1])
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, C = 2, 8, 256
    Nq = a.nq
    Nk = a.nk or (40000 if a.cross else Nq)
    pad, grp, drop = (0, 0, 0.0) if a.cross else (a.pad, a.group, a.drop)
    g = torch.Generator(device="cpu").manual_seed(0)
    q, k, v = (torch.randn(B, n, C, generator=g).to(dev) for n in (Nq, Nk, Nk))
    o, do = torch.empty_like(q), torch.randn(B, Nq, C, generator=g).to(dev)
    lse = torch.empty(B * H * Nq, device=dev)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    kw = dict(B=B, H=H, Nq=Nq, Nk=Nk, q_strides=(Nq * C, 32, C), k_strides=(Nk * C, 32, C), v_strides=(Nk * C, 32, C),
              o_strides=(Nq * C, 32, C), scale=32 ** -0.5, dn_pad=pad, dn_group=grp, fp16_inputs=a.cross,
              dropout_p=drop, seed=7)

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        return sorted(ts)[3]
    tf = t(lambda: T.attn_train_fwd(q, k, v, o, lse, **kw))
    tb = t(lambda: T.attn_train_bwd(q, k, v, o, lse, do, dq, dk, dv, **kw))
    print(f"attn_train[{a.tag}] {'cross fp16' if a.cross else 'self f32'} B={B} Nq={Nq} Nk={Nk} pad={pad} drop={drop}: "
          f"fwd {tf:.1f} us, bwd {tb:.1f} us (incl. delta / f16 copies); dq[0,0,:4]={dq[0, 0, :4].tolist()}", flush=True)


if __name__ == "__main__":
    main()
