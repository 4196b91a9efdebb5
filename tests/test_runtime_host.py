"""Host-side numerics-policy checks (no GPU): the f16 operand range guard of
the 'ref' and 'fp16' policies (runtime.check_f16_range)."""
import pytest
import torch

from projects.mmdet3d_plugin.runtime import F16_MAX, PRECISIONS, check_f16_range


@pytest.mark.parametrize("prec", ["ref", "fp16"])
def test_f16_range_guard_raises_for_out_of_range_inputs(prec):
    p = PRECISIONS[prec]
    ok = torch.full((4, 8), F16_MAX)
    check_f16_range(p, [ok, None, torch.empty(0)])
    for bad in (F16_MAX * 1.01, float("inf"), float("nan")):
        x = ok.clone()
        x[2, 3] = -bad
        with pytest.raises(ValueError, match="exact"):
            check_f16_range(p, [ok, x])


@pytest.mark.parametrize("prec", ["exact", "bf16"])
def test_f16_range_guard_is_off_for_wide_policies(prec):
    check_f16_range(PRECISIONS[prec], [torch.full((2, 2), 1e30)])


def test_mlp2_pack_layout():
    """native.mlp2_pack (cmt_hip.h cmt_mlp2_x3): W1p / W2p index maps, checked
    element by element against the header's formulas on distinct values."""
    import torch
    from projects.mmdet3d_plugin import native
    Hd, K = 64, 48
    W1 = torch.arange(Hd * 2 * K, dtype=torch.int32).to(torch.uint16).view(Hd, 2, K)
    W2 = torch.arange(256 * 2 * Hd, dtype=torch.int32).remainder(65536).to(torch.uint16).view(256, 2, Hd)
    w1p, w2p = native.mlp2_pack(W1, W2)
    f1 = w1p.reshape(-1).to(torch.int32)
    f2 = w2p.reshape(-1).to(torch.int32)
    KS = K // 16
    for hb in range(Hd // 32):
        for ks in range(KS):
            for pl in range(2):
                for lane in (0, 5, 31, 32, 47, 63):
                    for j in range(8):
                        got = f1[(((hb * KS + ks) * 2 + pl) * 64 + lane) * 8 + j].item()
                        want = int(W1[32 * hb + (lane & 31), pl, 16 * ks + 8 * (lane >> 5) + j])
                        assert got == want
    for hb in range(Hd // 32):
        for ot in (0, 3, 7):
            for s in range(2):
                for pl in range(2):
                    for lane in (0, 9, 31, 32, 50, 63):
                        for j in range(8):
                            got = f2[((((hb * 8 + ot) * 2 + s) * 2 + pl) * 64 + lane) * 8 + j].item()
                            k = 32 * hb + 16 * s + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3)
                            want = int(W2[32 * ot + (lane & 31), pl, k])
                            assert got == want
