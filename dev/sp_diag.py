"""Diagnostic: attn_sp_kernel vs attn_pb2_kernel vs a float64 flash-f16 reference
on bounded f16 inputs; where and how much the two kernels differ."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))
import torch  # noqa: E402

from projects.mmdet3d_plugin import native as N  # noqa: E402


def kmax2(k, B, Nk, H):
    ss = (k.double().permute(0, 2, 1, 3).reshape(B * Nk, H, 32) ** 2).sum(-1)
    nb = -(-B * Nk // 64)
    return torch.cat([ss, torch.zeros(nb * 64 - B * Nk, H, dtype=ss.dtype)], 0).view(nb, 64, H).amax(1).float()


def ref16(q, k, v, scale):
    s = (q.double() @ k.double().transpose(-1, -2)) * scale
    p = torch.exp(s - s.amax(-1, keepdim=True))
    return ((p.half().double() @ v.double()) / p.sum(-1, keepdim=True)).half().double()


def main():
    dev = torch.device("cuda")
    for (B, Nq, Nk, splits) in [(1, 900, 56400, 0), (1, 256, 4096, 1), (1, 256, 64 * 12, 1), (1, 32, 64 * 4, 1)]:
        H = 8
        g = torch.Generator().manual_seed(Nk + 3 * Nq)
        q = torch.randn(B, H, Nq, 32, generator=g).half()
        k = torch.randn(B, H, Nk, 32, generator=g).half()
        v = torch.randn(B, H, Nk, 32, generator=g).half()
        km = kmax2(k, B, Nk, H).to(dev)
        qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
        ref = ref16(q, k, v, 1 / math.sqrt(32)).permute(0, 2, 1, 3).reshape(B, Nq, H * 32)
        res = {}
        for diag in (0, 256):
            for fold in (False, True):
                O = torch.full((B, Nq, H * 32), float("nan"), device=dev)
                N.attention(qd, kd, vd, O, B=B, H=H, Nq=Nq, Nk=Nk,
                            q_strides=(H * Nq * 32, Nq * 32, 32), k_strides=(H * Nk * 32, Nk * 32, 32),
                            v_strides=(H * Nk * 32, Nk * 32, 32), o_strides=(Nq * H * 32, H * 32),
                            scale=1 / math.sqrt(32), kv_splits=splits, round_output=True, fold_scale=fold, kmax2=km,
                            kmax_ld=H, kmax_plane0=0, _diag_flags=diag)
                torch.cuda.synchronize()
                res[(diag, fold)] = O.cpu().double()
        for fold in (False, True):
            sp, pp = res[(0, fold)], res[(256, fold)]
            d = (sp - pp).abs()
            nd = (d > 0).sum().item()
            idx = (d > 0).nonzero()
            print(f"B{B} Nq{Nq} Nk{Nk} s{splits} fold{int(fold)}: differing {nd}/{d.numel()} max {d.max().item():.3e}; "
                  f"err vs ref sp {(sp - ref).abs().max().item():.3e} pp {(pp - ref).abs().max().item():.3e}", flush=True)
            if nd:
                qs = idx[:, 1].unique()
                cs = idx[:, 2].unique()
                print(f"   queries {qs[:20].tolist()} (n={len(qs)}), cols {cs[:20].tolist()} (n={len(cs)}), "
                      f"heads {(cs // 32).unique().tolist()}", flush=True)
                j = d.view(-1).argmax().item()
                print(f"   worst: sp {sp.view(-1)[j]:.6e} pp {pp.view(-1)[j]:.6e} ref {ref.reshape(-1)[j]:.6e}", flush=True)


if __name__ == "__main__":
    main()
