"""Executes the INTEGRATION.md reference-side stub verbatim on flash-layout
tensors (q [B*Sq, H, D], kv [B*Sk, 2, H, D] fp16, attention.py:63-75) and
compares it with the oracle's flash-attn 0.2.2 fp16 core."""
import math

import pytest
import torch

from _stub import load_stub

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,Sq,Sk", [(1, 900, 4000), (2, 96, 1000), (1, 900, 32400)])
def test_stub_matches_fp16_core(dev, B, Sq, Sk):
    from oracle import cmt_oracle as O
    ns = load_stub()
    H, D = 8, 32
    g = torch.Generator().manual_seed(B * 7 + Sk)
    q = (torch.randn((B * Sq, H, D), generator=g) * 1.5).half()
    kv = (torch.randn((B * Sk, 2, H, D), generator=g) * 1.5).half()
    cu_q = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=dev)
    cu_k = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device=dev)
    out = ns["flash_attn_unpadded_kvpacked_func"](q.to(dev), kv.to(dev), cu_q, cu_k, Sq, Sk, 0.0)
    torch.cuda.synchronize()
    assert out.dtype == torch.float16 and out.shape == q.shape
    qh = q.view(B, Sq, H, D).transpose(1, 2)
    kh = kv[:, 0].reshape(B, Sk, H, D).transpose(1, 2)
    vh = kv[:, 1].reshape(B, Sk, H, D).transpose(1, 2)
    ref = O.flash_core_fp16(qh, kh, vh, 1.0 / math.sqrt(D)).transpose(1, 2).reshape(B * Sq, H, D)
    err = (out.cpu().float() - ref).abs().max().item()
    print(f"stub vs fp16 core (B={B}, Sq={Sq}, Sk={Sk}): max abs {err:.2e}")
    # |o| <= max|v| ~ 7; fp16 output rounding is 2^-11 relative: allow 2 ulps at |o| ~ 2
    assert err <= 2e-3
